# round-5 GPU check j: dispatch overlap of two frames in flight at the N=8 share with the no-copy
# launch path (kernel trace), INFLIGHT 2 and 3; then the 3-D block subtrees (r05h)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05j}; mkdir -p $O
cd /tmp
WORLDS=8 INFLIGHT=2 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/ovl -o ovl --output-format csv -- python3 $R/tools/rank_balance.py c3 1 > $O/ovl_rank_balance.log 2>&1
cd $R
python tools/overlap.py $O/ovl > $O/overlap.txt 2>&1 || true
python tools/overlap.py $O/ovl __amd > $O/overlap_blits.txt 2>&1 || true
WORLDS=1,8 INFLIGHT=3 timeout -k 10 300 python tools/rank_balance.py c3 3 > $O/rb_inflight3.log 2>&1
echo overlap done
TAG=r05h bash tools/r05h.sh
