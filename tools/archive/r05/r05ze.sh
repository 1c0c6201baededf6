# round 5: one item per queue atomic for the world-8 shares (DT_BATCH_ITEMS above the share's items) against the default two
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05ze}; mkdir -p $O
for rep in 1 2; do
  echo "# default (rep $rep)" >> $O/rb.log
  INFLIGHT=2 WORLDS=1,8 timeout -k 10 180 python3 $R/tools/rank_balance.py c3 3 2>/dev/null >> $O/rb.log
  echo "# DT_BATCH_ITEMS=100000000: one item per atomic (rep $rep)" >> $O/rb.log
  DT_BATCH_ITEMS=100000000 INFLIGHT=2 WORLDS=1,8 timeout -k 10 180 python3 $R/tools/rank_balance.py c3 3 2>/dev/null >> $O/rb.log
done
echo all done
