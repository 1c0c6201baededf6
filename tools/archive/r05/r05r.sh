# round-5 GPU check r: three items per queue atomic for whole large frames (default now); the
# longest-tiles-first slot order from measured tile costs (experiment, DT_TILE_ORDER=dir:)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05r}; mkdir -p $O
V=distraytracer_amd/variants
export DT_PARITY_LOG=$O/parity.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
echo tests ok
DT_LIB=$V/libdt_itemrt.so timeout -k 10 300 python tools/lpt_order.py c3 $O/lpt 1,8 > $O/lpt_order.log 2>&1
echo lpt done
b() {   # name, env, config, steps
  env $2 timeout -k 10 200 python bench.py --config $3 --steps $4 --warmup 1 --no-cpu-baseline --no-roofline > $O/$1.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/$1.json').read().splitlines()[-1]);print('$1',d['value'],d['roofline']['kernel_ms'])" >> $O/ab.txt
}
for rep in 1 2; do
  b c3_batch3_$rep "DT_X=0" c3 8; b c3_batch2_$rep "DT_BATCH_SIZE=2" c3 8; b c3_lpt_$rep "DT_TILE_ORDER=dir:$O/lpt" c3 8
done
echo ab done
WORLDS=1,8 INFLIGHT=2 timeout -k 10 300 python tools/rank_balance.py c3 3 > $O/rb_base.log 2>&1
DT_TILE_ORDER=dir:$O/lpt WORLDS=1,8 INFLIGHT=2 timeout -k 10 300 python tools/rank_balance.py c3 3 > $O/rb_lpt.log 2>&1
echo all done
