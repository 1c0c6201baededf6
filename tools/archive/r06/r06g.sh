# round 6 (g): C4 rank balance by tile side with chunk items (the default at world > 1)
set -e
O=gpurun_out/r06g; rm -rf $O; mkdir -p $O
rb() { n=$1; shift; env "$@" INFLIGHT=2 timeout -k 10 500 python tools/rank_balance.py c4 2 > $O/rb_$n.log 2>&1; echo "rb $n $*"; grep -o '"world": [0-9]*\|"max_ms": [0-9.]*\|"mean_ms": [0-9.]*\|"kernel_efficiency": [0-9.]*' $O/rb_$n.log | paste -sd' '; }
rb t16 TILE=16 WORLDS=1,2,4,8
rb t8 TILE=8 WORLDS=2,4,8
rb t4 TILE=4 WORLDS=2,4,8
