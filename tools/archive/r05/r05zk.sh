# round 5: C4's world-8 share excess: deep-cascade priority off, tile side 16/32, and the 8x8 split at world 1
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05zk}; mkdir -p $O
cd $R
for v in "DT_X=0" "DT_PRIO_STEPS=0" "TILE=16" "TILE=32"; do
  echo "# $v" >> $O/rb.log
  env $v INFLIGHT=2 WORLDS=1,8 timeout -k 10 300 python3 tools/rank_balance.py c4 2 2>/dev/null >> $O/rb.log
done
echo "# TILE_W=8 TILE_H=8 at world 1 (TILE=8)" >> $O/rb.log
TILE=8 INFLIGHT=2 WORLDS=1 timeout -k 10 300 python3 tools/rank_balance.py c4 2 2>/dev/null >> $O/rb.log
echo all done
