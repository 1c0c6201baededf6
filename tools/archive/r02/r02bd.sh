# per-lane content filter in the bumped gather: parity suite, blur frames and C3/C2 vs DT_BUMP_CONTENT=0
set -e
O=gpurun_out/r02bd; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
echo tests ok
for f in 1680 1840 1920; do
  timeout -k 10 120 python3 tools/frame_ab.py $f 960x540 64 "" >> $O/frames.log 2>&1
  DT_LIB=distraytracer_amd/variants/libdt_prev.so timeout -k 10 120 python3 tools/frame_ab.py $f 960x540 64 "" >> $O/frames.log 2>&1
done
TAG=r02bd CFGS="c3 c2" bash tools/ab_lib.sh > $O/ab.log 2>&1
echo done
