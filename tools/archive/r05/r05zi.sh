# round 5: home segment from the XCD register (variant xcc, DT_QUEUE_HOME=1) against the block index; C4/C2 shares with and without segments
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05zi}; mkdir -p $O
cd $R
V=distraytracer_amd/variants/libdt_xcc.so
DT_LIB=$V DT_QUEUE_HOME=1 DT_QUEUE_SEGS=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_launch_path.py tests/test_gpu_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_xcc.log 2>&1 || { tail -30 $O/tests_xcc.log; exit 1; }
tail -1 $O/tests_xcc.log
b() {   # name, env, config, steps
  env $2 timeout -k 10 200 python bench.py --config $3 --steps $4 --warmup 1 --no-cpu-baseline --no-roofline > $O/$1.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/$1.json').read().splitlines()[-1]);print('$1',d['value'],d['roofline']['kernel_ms'])" >> $O/ab.txt
}
for rep in 1 2; do
  b c3_one_$rep "DT_LIB=$V" c3 8; b c3_blk8_$rep "DT_LIB=$V DT_QUEUE_SEGS=8" c3 8; b c3_xcc8_$rep "DT_LIB=$V DT_QUEUE_SEGS=8 DT_QUEUE_HOME=1" c3 8
done
b c4_one "DT_LIB=$V" c4 2; b c4_xcc8 "DT_LIB=$V DT_QUEUE_SEGS=8 DT_QUEUE_HOME=1" c4 2
echo ab done
for v in "DT_X=0" "DT_QUEUE_HOME=1"; do
  echo "# c3 $v" >> $O/rb.log
  env DT_LIB=$V $v INFLIGHT=2 WORLDS=1,8 timeout -k 10 200 python3 $R/tools/rank_balance.py c3 3 2>/dev/null >> $O/rb.log
done
for cfg in c4 c2; do
for v in "DT_X=0" "DT_QUEUE_SEGS=1"; do
  echo "# $cfg $v" >> $O/rb.log
  env DT_LIB=$V $v INFLIGHT=2 WORLDS=1,8 timeout -k 10 300 python3 $R/tools/rank_balance.py $cfg 2 2>/dev/null >> $O/rb.log
done
done
echo all done
