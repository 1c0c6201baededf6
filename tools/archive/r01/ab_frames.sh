#!/bin/bash
# A/B the library variants in distraytracer_amd/variants/ on single C5 frames (tools/frame_ab.py).
# FRAMES (default "2160 1200") at 1920x1080, 64 spp (cloud frames render 1 spp).
R=${GRAFT_REPO_ROOT:-$(pwd)}
for so in "$R"/distraytracer_amd/variants/*.so; do
  n=$(basename "$so" .so)
  for f in ${FRAMES:-2160 1200}; do
    echo -n "$n frame $f "
    DT_LIB="$so" timeout -k 10 200 python "$R/tools/frame_ab.py" $f 1920x1080 64 "" 2>/dev/null | tail -1 || exit 1
  done
done
