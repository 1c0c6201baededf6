# round-5 GPU check q: small switches re-measured on the final kernel: the 5-wave build for C2
# (DT_W5=1), the deep-cascade priority at N=8 (DT_PRIO_STEPS=0), three items per queue atomic
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05q}; mkdir -p $O
b() {   # name, env, config, steps
  env $2 timeout -k 10 200 python bench.py --config $3 --steps $4 --warmup 1 --no-cpu-baseline --no-roofline > $O/$1.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/$1.json').read().splitlines()[-1]);print('$1',d['value'],d['roofline']['kernel_ms'])" >> $O/ab.txt
}
for rep in 1 2; do
  b c2_base_$rep "DT_X=0" c2 10; b c2_w5_$rep "DT_W5=1" c2 10
  b c3_base_$rep "DT_X=0" c3 8; b c3_batch3_$rep "DT_BATCH_SIZE=3" c3 8
done
echo ab done
WORLDS=1,8 INFLIGHT=2 timeout -k 10 300 python tools/rank_balance.py c3 3 > $O/rb_base.log 2>&1
DT_PRIO_STEPS=0 WORLDS=1,8 INFLIGHT=2 timeout -k 10 300 python tools/rank_balance.py c3 3 > $O/rb_noprio.log 2>&1
echo all done
