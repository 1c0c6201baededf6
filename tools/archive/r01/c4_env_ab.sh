R=${GRAFT_REPO_ROOT:-$(pwd)}
for kv in "ftc:DT_FAST_TREE=c" "ft1:DT_FAST_TREE=1" "ft0:DT_FAST_TREE=0" "cells64k:DT_SG_CELLS=65536" "reach1:DT_SG_REACH=1"; do
  n=${kv%%:*}; e=${kv#*:}
  env $e timeout -k 10 300 python $R/bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > $R/gpurun_out/c4_$n.json 2>/dev/null || { echo "$n failed"; break; }
  python -c "import json; d=json.loads(open('$R/gpurun_out/c4_$n.json').read().strip().split(chr(10))[-1]); print('$n', d['value'], d['ms_per_step'])"
done
