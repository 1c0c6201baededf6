#!/bin/bash
# A/B every library variant in distraytracer_amd/variants/ on C3 (3 steps), C2, C4 (1 step) and
# C5 frames (tools/frame_ab.py, FRAMES default "1200 2160" at 1920x1080). SKIP_C4=1 skips C4.
R=${GRAFT_REPO_ROOT:-$(pwd)}
for so in "$R"/distraytracer_amd/variants/*.so; do
  n=$(basename "$so" .so)
  line="$n"
  for cfg in c3 c2 ${SKIP_C4:+}c4; do
    [ "$cfg" = c4 ] && [ -n "$SKIP_C4" ] && continue
    st=3; [ "$cfg" = c4 ] && st=1
    env ${ENVS:-} DT_LIB="$so" timeout -k 10 300 python "$R/bench.py" --config $cfg --steps $st --warmup 1 --no-cpu-baseline > "$R/gpurun_out/ab_${n}_$cfg.json" 2> "$R/gpurun_out/ab_${n}_$cfg.err" || { echo "$n $cfg failed"; tail -3 "$R/gpurun_out/ab_${n}_$cfg.err"; exit 1; }
    v=$(python -c "import json; d=json.loads(open('$R/gpurun_out/ab_${n}_$cfg.json').read().splitlines()[-1]); print(round(d['value'],1))")
    line="$line $cfg=$v"
  done
  for f in ${FRAMES:-1200 2160}; do
    v=$(env ${ENVS:-} DT_LIB="$so" timeout -k 10 200 python "$R/tools/frame_ab.py" $f 1920x1080 64 "" 2>/dev/null | tail -1 | python -c "import json,sys; print(json.loads(sys.stdin.read())['kernel_ms'])") || { echo "$n frame $f failed"; exit 1; }
    line="$line f$f=${v}ms"
  done
  echo "$line"
done
