set -e
O=gpurun_out/r02bq; mkdir -p $O
DT_TIMING=1 timeout -k 10 300 python tools/pl_timing.py 1920x1080 30,30 > $O/c3_timing.log 2>&1
echo done
