# round 6 (l): GPU suite on the current tree; C5 all 300 frames, one frame at a time (round 5) vs two in flight
set -e
O=gpurun_out/r06l; rm -rf $O; mkdir -p $O
export DT_PARITY_LOG=$O/parity.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
timeout -k 10 400 python tools/archive/r06/animate_r05.py --frames 0:300:1 --per-frame > $O/c5_r05.json 2> $O/c5_r05.log
tail -1 $O/c5_r05.json
timeout -k 10 400 python tools/animate.py --frames 0:300:1 --per-frame > $O/c5_new.json 2> $O/c5_new.log
tail -1 $O/c5_new.json
