#!/bin/bash
# C5 A/B: the given frame range (default the tunnel frames 120:244:4) at 4K, 64 spp, depth 10, with
# this tree's libdt.so and with each variant in $VARS; prints seconds and frames/s per library.
set -e
O=gpurun_out/${TAG:-c5ab}; mkdir -p $O
F=${FRAMES:-120:244:4}
for v in base $VARS; do
  lib=""; [ $v != base ] && lib=distraytracer_amd/variants/libdt_$v.so
  DT_LIB=$lib timeout -k 10 400 python tools/animate.py --frames $F --per-frame > $O/c5_$v.json 2> $O/c5_$v.log
  python -c "import json;d=json.loads(open('$O/c5_$v.json').read().strip().splitlines()[-1]);print('$v', d['seconds'], d['frames_per_s'], d['abort_counters'])"
done
