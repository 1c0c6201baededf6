# parity suite, C5 animation sample (per frame), C3 bench
set -e
O=gpurun_out/${TAG:-r02aw}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
echo tests ok
timeout -k 10 300 python tools/animate.py --frames 0:300:30 --per-frame > $O/c5_animate.log 2>&1
echo c5 ok
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
echo done
