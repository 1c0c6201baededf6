# round 6 (k): counters spread over 16 slots — C3/C2/C4 against HEAD, C3 world-8 shares
set -e
O=gpurun_out/r06k; rm -rf $O; mkdir -p $O
j() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2',d['value'],d['roofline']['kernel_ms'],d['ms_per_step'])"; }
b() { n=$1; c=$2; shift 2; st=5; [ $c = c3 ] && st=10; [ $c = c2 ] && st=40; env "$@" timeout -k 10 300 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline > $O/$n.json 2>/dev/null; j $O/$n.json "$n $*"; }
for rep in 1 2; do
for c in c3 c2 c4; do
b ${c}_base_$rep $c DT_LIB=distraytracer_amd/variants/libdt_base.so
b ${c}_new_$rep $c A=1
done
done
rb() { n=$1; c=$2; shift 2; env "$@" INFLIGHT=2 timeout -k 10 500 python tools/rank_balance.py $c 2 > $O/rb_$n.log 2>&1; echo "rb $n $*"; grep -o '"world": [0-9]*\|"max_ms": [0-9.]*\|"mean_ms": [0-9.]*' $O/rb_$n.log | paste -sd' '; }
rb c3_base c3 DT_LIB=distraytracer_amd/variants/libdt_base.so WORLDS=1,8
rb c3_new c3 WORLDS=1,8
rb c3_new_t2 c3 WORLDS=8 TILE=2
