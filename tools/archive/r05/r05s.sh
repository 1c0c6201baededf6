# round-5 GPU check s: the N=1 tile side (one launch at a time, whole C3 frame as a slab)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05s}; mkdir -p $O
for t in 32 64 16 128 32 64; do
  TILE=$t WORLDS=1 timeout -k 10 200 python tools/rank_balance.py c3 4 > $O/rb_t$t.log 2>&1
  echo "tile $t $(grep -v amdgpu $O/rb_t$t.log | tail -1)" >> $O/tiles.txt
done
echo all done
