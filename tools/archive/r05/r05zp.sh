# round 5: deep-cascade priority steps for split frames (DT_PRIO_STEPS 8 default, 0, 16), C3 and C4 world-8 shares, twice
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05zp}; mkdir -p $O
cd $R
for rep in 1 2; do
for v in "DT_PRIO_STEPS=8" "DT_PRIO_STEPS=0" "DT_PRIO_STEPS=16"; do
  echo "# c3 $v (rep $rep)" >> $O/rb.log
  env $v INFLIGHT=2 WORLDS=1,8 timeout -k 10 200 python3 tools/rank_balance.py c3 3 2>/dev/null >> $O/rb.log
done
done
for v in "DT_PRIO_STEPS=8" "DT_PRIO_STEPS=0"; do
  echo "# c4 $v" >> $O/rb.log
  env $v INFLIGHT=2 WORLDS=1,8 timeout -k 10 300 python3 tools/rank_balance.py c4 2 2>/dev/null >> $O/rb.log
done
echo all done
