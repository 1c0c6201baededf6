# pass-0 grid: parity suite, then tunnel blur frames with DT_SG_PASS0 on/off (960x540, 64 spp)
set -e
O=gpurun_out/r02ar; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
echo tests ok
for f in 1680 1760 1840 1920; do
  timeout -k 10 120 python3 tools/frame_ab.py $f 960x540 64 "" >> $O/frames.log 2>&1
  DT_SG_PASS0=0 timeout -k 10 120 python3 tools/frame_ab.py $f 960x540 64 "" >> $O/frames.log 2>&1
  DT_SG_PASS0=1 timeout -k 10 120 python3 tools/frame_ab.py $f 960x540 64 "" >> $O/frames.log 2>&1
done
echo done
