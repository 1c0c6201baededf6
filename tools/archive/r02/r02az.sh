set -e
O=gpurun_out/r02az; mkdir -p $O
DT_TIMING=1 timeout -k 10 300 python tools/animate.py --frames 210:300:30 --per-frame > $O/c5_timing.log 2>&1
echo done
