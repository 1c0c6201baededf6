# C5 transition frames (n = 121..139, deep glossy cascades) with the product kernel, with the
# work-sharing kernel chosen per frame by the probe (--donate auto), and forced on for
# DT_DONATE_AFTER in $AFTERS. Output under gpurun_out/$TAG.
set -e
O=gpurun_out/${TAG:-donate_c5}; mkdir -p $O
F=${FRAMES:-121:140:1}
timeout -k 10 300 python tools/animate.py --frames $F --donate off --per-frame > $O/tr_off.log 2>&1
timeout -k 10 300 python tools/animate.py --frames $F --donate auto --per-frame > $O/tr_auto.log 2>&1
for a in ${AFTERS:-}; do
  DT_DONATE_AFTER=$a timeout -k 10 300 python tools/animate.py --frames $F --donate on --per-frame > $O/tr_on_$a.log 2>&1
done
