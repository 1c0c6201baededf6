# round 6 (c): C3 against round 5 (allocation check), C4 world-8 bound with chunk items
set -e
O=gpurun_out/r06c; rm -rf $O; mkdir -p $O
j() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2',d['value'],d['roofline']['kernel_ms'])"; }
b() { n=$1; c=$2; shift 2; st=3; [ $c = c3 ] && st=10; env "$@" timeout -k 10 300 python bench.py --config $c --steps $st --warmup 1 --no-cpu-baseline > $O/$n.json 2>/dev/null; j $O/$n.json "$n $*"; }
for rep in 1 2; do
b c3_r05_$rep c3 DT_LIB=distraytracer_amd/variants/libdt_r05.so
b c3_b1_$rep c3 DT_LIB=distraytracer_amd/variants/libdt_b1.so
b c3_cur_$rep c3 A=1
done
rb() { n=$1; shift; env "$@" INFLIGHT=2 WORLDS=1,8 timeout -k 10 400 python tools/rank_balance.py c4 2 > $O/rb_$n.log 2>&1; echo "rb $n $*"; grep -o '"world": [0-9]*\|"max_ms": [0-9.]*\|"mean_ms": [0-9.]*\|"kernel_efficiency": [0-9.]*' $O/rb_$n.log | paste -sd' '; }
rb m0 DT_CHUNK_ITEMS=0
rb m1 DT_CHUNK_ITEMS=1
rb m1s8 DT_CHUNK_ITEMS=1 DT_QUEUE_SEGS=8
rb m1b2 DT_CHUNK_ITEMS=1 DT_BATCH_SIZE=2
rb m1s8b2 DT_CHUNK_ITEMS=1 DT_QUEUE_SEGS=8 DT_BATCH_SIZE=2
