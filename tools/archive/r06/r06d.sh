# round 6 (d): C3 allocation variants; C4 world-8 with chunk items + work sharing / priority
set -e
O=gpurun_out/r06d; rm -rf $O; mkdir -p $O
j() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2',d['value'],d['roofline']['kernel_ms'])"; }
b() { n=$1; c=$2; shift 2; st=3; [ $c = c3 ] && st=10; env "$@" timeout -k 10 300 python bench.py --config $c --steps $st --warmup 1 --no-cpu-baseline > $O/$n.json 2>/dev/null; j $O/$n.json "$n $*"; }
for rep in 1 2; do
for v in r05 v3 v5; do b c3_${v}_$rep c3 DT_LIB=distraytracer_amd/variants/libdt_$v.so; done
b c3_cur_$rep c3 A=1
done
rb() { n=$1; shift; env "$@" INFLIGHT=2 WORLDS=8 timeout -k 10 400 python tools/rank_balance.py c4 2 > $O/rb_$n.log 2>&1; echo "rb $n $*"; grep -o '"kernel_ms_per_rank": [^]]*\]\|"max_ms": [0-9.]*\|"mean_ms": [0-9.]*' $O/rb_$n.log | paste -sd' '; }
rb dn DT_CHUNK_ITEMS=1 DT_QUEUE_SEGS=8 DT_DONATE=1
rb p0 DT_CHUNK_ITEMS=1 DT_QUEUE_SEGS=8 DT_PRIO_STEPS=0
rb p2 DT_CHUNK_ITEMS=1 DT_QUEUE_SEGS=8 DT_PRIO_STEPS=2
rb m2s8 DT_CHUNK_ITEMS=2 DT_QUEUE_SEGS=8
