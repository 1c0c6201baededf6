set -e
O=gpurun_out/r02ax; mkdir -p $O
DT_TIMING=1 timeout -k 10 300 python tools/pl_timing.py 3840x2160 30,150,270 > $O/pl_timing.log 2>&1
echo done
