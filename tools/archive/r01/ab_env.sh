#!/bin/bash
# A/B of environment settings on the current libdt (bench c3, 1 step): ab_env.sh NAME "ENV=..." ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
while [ $# -gt 1 ]; do
  n=$1; e=$2; shift 2
  env $e DT_LIB=${DT_LIB_OVERRIDE:-$R/distraytracer_amd/libdt.so} timeout -k 10 300 python "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/abenv_$n.json" 2> "$R/gpurun_out/abenv_$n.err" || { echo "$n failed"; break; }
  python -c "import json; d=json.load(open('$R/gpurun_out/abenv_$n.json')); print('$n', d['value'], d['ms_per_step'])"
done
