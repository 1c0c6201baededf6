# round 6 (i): longest items of C2 and C3 (item-time build); C3 world-8 bound by tile side; C4 2x2 at N=2/4
set -e
O=gpurun_out/r06i; rm -rf $O; mkdir -p $O
DT_LIB=distraytracer_amd/variants/libdt_itemrt.so timeout -k 10 300 python tools/chunk_costs.py c2 1 > $O/costs_c2.log 2>&1
DT_LIB=distraytracer_amd/variants/libdt_itemrt.so timeout -k 10 300 python tools/chunk_costs.py c3 1 > $O/costs_c3.log 2>&1
rb() { n=$1; c=$2; shift 2; env "$@" INFLIGHT=2 timeout -k 10 500 python tools/rank_balance.py $c 2 > $O/rb_$n.log 2>&1; echo "rb $n $*"; grep -o '"world": [0-9]*\|"max_ms": [0-9.]*\|"mean_ms": [0-9.]*' $O/rb_$n.log | paste -sd' '; }
rb c3_t8 c3 TILE=8 WORLDS=1,8
rb c3_t4 c3 TILE=4 WORLDS=8
rb c3_t2 c3 TILE=2 WORLDS=8
rb c4_t2 c4 TILE=2 WORLDS=2,4
rb c2_t8 c2 TILE=8 WORLDS=1,8
rb c2_t4 c2 TILE=4 WORLDS=8
