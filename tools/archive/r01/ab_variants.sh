#!/bin/bash
# A/B the library variants in distraytracer_amd/variants/ on the GPU box (bench c3, 1 step).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
for so in "$R"/distraytracer_amd/variants/*.so; do
  n=$(basename "$so" .so)
  DT_LIB="$so" timeout -k 10 300 python "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$R/gpurun_out/ab_$n.json" 2> "$R/gpurun_out/ab_$n.err" || { echo "$n failed"; tail -3 "$R/gpurun_out/ab_$n.err"; break; }
  python -c "import json,sys; d=json.load(open('$R/gpurun_out/ab_$n.json')); print('$n', d['value'], d['ms_per_step'])"
done
