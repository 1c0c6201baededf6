# round 6 (s): C3 split tile side 8 vs 2 at N=2/4/8 (two frames in flight), twice
set -e
O=gpurun_out/r06s; rm -rf $O; mkdir -p $O
rb() { n=$1; shift; env "$@" INFLIGHT=2 timeout -k 10 500 python tools/rank_balance.py c3 2 > $O/rb_$n.log 2>&1; echo "rb $n $*"; grep -o '"world": [0-9]*\|"max_ms": [0-9.]*\|"mean_ms": [0-9.]*\|"kernel_efficiency": [0-9.]*' $O/rb_$n.log | paste -sd' '; }
rb t8a TILE=8 WORLDS=1,2,4,8
rb t2a TILE=2 WORLDS=1,2,4,8
rb t8b TILE=8 WORLDS=1,2,4,8
rb t2b TILE=2 WORLDS=1,2,4,8
