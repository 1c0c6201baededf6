# round 5: segmented item queue (DT_QUEUE_SEGS=8): GPU suite under it, then C3/C2/C4 A/B and world-8 shares
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05zf}; mkdir -p $O
cd $R
DT_QUEUE_SEGS=8 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_segs8.log 2>&1 || { tail -30 $O/gpu_tests_segs8.log; exit 1; }
tail -2 $O/gpu_tests_segs8.log
b() {   # name, env, config, steps
  env $2 timeout -k 10 200 python bench.py --config $3 --steps $4 --warmup 1 --no-cpu-baseline --no-roofline > $O/$1.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/$1.json').read().splitlines()[-1]);print('$1',d['value'],d['roofline']['kernel_ms'])" >> $O/ab.txt
}
for rep in 1 2; do
  b c3_s1_$rep "DT_QUEUE_SEGS=1" c3 8; b c3_s8_$rep "DT_QUEUE_SEGS=8" c3 8; b c3_s8b2_$rep "DT_QUEUE_SEGS=8 DT_BATCH_SIZE=2" c3 8
  b c3_s8b1_$rep "DT_QUEUE_SEGS=8 DT_BATCH_ITEMS=100000000" c3 8
  b c2_s1_$rep "DT_QUEUE_SEGS=1" c2 10; b c2_s8_$rep "DT_QUEUE_SEGS=8" c2 10
  b c4_s1_$rep "DT_QUEUE_SEGS=1" c4 2; b c4_s8_$rep "DT_QUEUE_SEGS=8" c4 2
done
echo ab done
for v in "DT_QUEUE_SEGS=1" "DT_QUEUE_SEGS=8" "DT_QUEUE_SEGS=8 DT_BATCH_ITEMS=100000000"; do
  echo "# $v" >> $O/rb.log
  env $v INFLIGHT=2 WORLDS=1,8 timeout -k 10 180 python3 $R/tools/rank_balance.py c3 3 2>/dev/null >> $O/rb.log
done
echo all done
