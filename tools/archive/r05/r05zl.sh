# round 5: C4 split tile side 8 against 16 at N = 2, 4, 8 (two frames in flight), twice
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05zl}; mkdir -p $O
cd $R
for rep in 1 2; do
for t in 8 16; do
  echo "# TILE=$t (rep $rep)" >> $O/rb.log
  TILE=$t INFLIGHT=2 WORLDS=1,2,4,8 timeout -k 10 300 python3 tools/rank_balance.py c4 2 2>/dev/null >> $O/rb.log
done
done
echo all done
