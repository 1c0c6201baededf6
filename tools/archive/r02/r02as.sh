# one-sided bump padding: parity suite, then blur frames with DT_BUMP_UP on/off (960x540, 64 spp)
set -e
O=gpurun_out/${TAG:-r02as}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
echo tests ok
for f in 1200 1680 1760 1840 1920; do
  timeout -k 10 120 python3 tools/frame_ab.py $f 960x540 64 "" >> $O/frames.log 2>&1
  DT_BUMP_UP=0 timeout -k 10 120 python3 tools/frame_ab.py $f 960x540 64 "" >> $O/frames.log 2>&1
done
echo done
