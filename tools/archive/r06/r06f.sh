# round 6 (f): hot order — tests; C3 against round 5; C4 N=1 and world-8 bound with/without hot order
set -e
O=gpurun_out/r06f; rm -rf $O; mkdir -p $O
export DT_PARITY_LOG=$O/parity.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_chunks.py tests/test_gpu_launch_path.py tests/test_gpu_dist.py > $O/tests.log 2>&1
j() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2',d['value'],d['roofline']['kernel_ms'])"; }
b() { n=$1; c=$2; shift 2; st=3; [ $c = c3 ] && st=10; env "$@" timeout -k 10 300 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline > $O/$n.json 2>/dev/null; j $O/$n.json "$n $*"; }
for rep in 1 2; do
b c3_r05_$rep c3 DT_LIB=distraytracer_amd/variants/libdt_r05.so
b c3_cur_$rep c3 A=1
b c3_nohot_$rep c3 DT_HOT_ORDER=0
b c4_m0_$rep c4 DT_CHUNK_ITEMS=0 DT_HOT_ORDER=0
b c4_m0hot_$rep c4 DT_CHUNK_ITEMS=0
b c4_m1hot_$rep c4 DT_CHUNK_ITEMS=1 DT_QUEUE_SEGS=8
done
rb() { n=$1; shift; env "$@" INFLIGHT=2 WORLDS=1,8 timeout -k 10 400 python tools/rank_balance.py c4 2 > $O/rb_$n.log 2>&1; echo "rb $n $*"; grep -o '"kernel_ms_per_rank": [^]]*\]\|"max_ms": [0-9.]*\|"mean_ms": [0-9.]*' $O/rb_$n.log | paste -sd' '; }
rb m1s8hot DT_CHUNK_ITEMS=1 DT_QUEUE_SEGS=8
rb m1s8 DT_CHUNK_ITEMS=1 DT_QUEUE_SEGS=8 DT_HOT_ORDER=0
rb m0hot DT_CHUNK_ITEMS=0
n=c3hot; INFLIGHT=2 WORLDS=1,8 timeout -k 10 400 python tools/rank_balance.py c3 2 > $O/rb_c3hot.log 2>&1; grep -o "\"max_ms\": [0-9.]*\|\"mean_ms\": [0-9.]*" $O/rb_c3hot.log | paste -sd" "
