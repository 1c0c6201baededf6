# deferred per-lane sky for 1-spp frames: parity suite, cloud-frame timings with and without
set -e
O=gpurun_out/r02al; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
echo tests ok
for f in 1952 2160 2392; do
  timeout -k 10 120 python3 tools/frame_ab.py $f 1920x1080 64 "" >> $O/frames.log 2>&1
  DT_SKY_DEFER=0 timeout -k 10 120 python3 tools/frame_ab.py $f 1920x1080 64 "" >> $O/frames.log 2>&1
done
echo done
