# A/B of the work-sharing trace kernel (dt_trace_kernel_dn, DT_DONATE=1) against the product kernel:
# parity tests, per-rank shares of C3 (tools/rank_balance.py) and the C5 transition frame 1088 at 4K.
# DT_DONATE_AFTER values to try: $AFTERS (default "4"). Output under gpurun_out/$TAG.
set -e
O=gpurun_out/${TAG:-donate}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_donate.py -x -v -s --timeout 200 --timeout-method thread > $O/donate_tests.log 2>&1
DT_DONATE=0 timeout -k 10 200 python tools/rank_balance.py c3 2 > $O/rb_off.log 2>&1
DT_DONATE=0 timeout -k 10 200 python tools/frame_ab.py 1088 3840x2160 64 "" > $O/f1088_off.log 2>&1
for a in ${AFTERS:-4}; do
  DT_DONATE=1 DT_DONATE_AFTER=$a timeout -k 10 200 python tools/rank_balance.py c3 2 > $O/rb_on_$a.log 2>&1
  DT_DONATE=1 DT_DONATE_AFTER=$a timeout -k 10 200 python tools/frame_ab.py 1088 3840x2160 64 "" > $O/f1088_on_$a.log 2>&1
done
