# round 6 (r): C5 all 300 frames (two frames in flight, shapes-first blur tests)
set -e
O=gpurun_out/r06r; rm -rf $O; mkdir -p $O
timeout -k 10 400 python tools/animate.py --frames 0:300:1 --per-frame > $O/c5_full.json 2> $O/c5_full.log
tail -1 $O/c5_full.json
