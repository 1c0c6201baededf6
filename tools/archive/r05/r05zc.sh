# round 5: tile shapes of the world-8 split (share locality against balance), 16 copies per launch and two frames in flight
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05zc}; mkdir -p $O
for shape in 8x8 16x16 32x8 64x4 240x8 240x4 1920x4 1920x8 1920x2; do
  w=${shape%x*}; h=${shape#*x}
  echo "# tile ${w}x${h}" >> $O/multi16.log
  MULTI=16 WORLDS=1,8 TILE_W=$w TILE_H=$h timeout -k 10 180 python3 $R/tools/rank_balance.py c3 3 2>/dev/null >> $O/multi16.log
done
for shape in 8x8 64x4 240x8 1920x4; do
  w=${shape%x*}; h=${shape#*x}
  echo "# tile ${w}x${h}" >> $O/inflight2.log
  INFLIGHT=2 WORLDS=1,8 TILE_W=$w TILE_H=$h timeout -k 10 180 python3 $R/tools/rank_balance.py c3 3 2>/dev/null >> $O/inflight2.log
done
echo all done
