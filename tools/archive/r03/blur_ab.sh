# Blur-heavy C5 frames at 4K / 64 spp (tools/frame_ab.py kernel ms) with the padded bump tree
# (DT_BUMP_PARENT=0) and the parent-box bump tree (=1). FRAMES, output under gpurun_out/$TAG.
set -e
O=gpurun_out/${TAG:-blur_ab}; mkdir -p $O
for f in ${FRAMES:-1200 1680 1760 1840 1920}; do
  for p in 0 1; do
    DT_BUMP_PARENT=$p timeout -k 10 200 python tools/frame_ab.py $f 3840x2160 64 "" > $O/f${f}_p$p.log 2>&1
    echo "$f $p $(grep kernel_ms $O/f${f}_p$p.log)"
  done
done
