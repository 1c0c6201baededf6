# round 6 (e): C3 of the current tree; C4 per-chunk durations (item-time build) at world 8 and 1
set -e
O=gpurun_out/r06e; rm -rf $O; mkdir -p $O
j() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2',d['value'],d['roofline']['kernel_ms'])"; }
b() { n=$1; c=$2; shift 2; st=3; [ $c = c3 ] && st=10; env "$@" timeout -k 10 300 python bench.py --config $c --steps $st --warmup 1 --no-cpu-baseline > $O/$n.json 2>/dev/null; j $O/$n.json "$n $*"; }
b c3_r05 c3 DT_LIB=distraytracer_amd/variants/libdt_r05.so
b c3_cur c3 A=1
b c3_r05b c3 DT_LIB=distraytracer_amd/variants/libdt_r05.so
b c3_curb c3 A=1
DT_LIB=distraytracer_amd/variants/libdt_itemrt.so DT_QUEUE_SEGS=8 timeout -k 10 300 python tools/chunk_costs.py c4 8 > $O/costs_c4_w8.log 2>&1
python -c "
import json
for l in open('$O/costs_c4_w8.log'):
    d=json.loads(l); print(d['rank'], d['kernel_ms'], d['ideal_ms'], d['replay_queue_ms'], d['replay_hot16x_first_ms'], d['replay_longest_first_ms'], d['top0.1pct_share'], d['longest'][:3])
"
DT_LIB=distraytracer_amd/variants/libdt_itemrt.so timeout -k 10 300 python tools/chunk_costs.py c4 1 > $O/costs_c4_w1.log 2>&1
python -c "
import json
for l in open('$O/costs_c4_w1.log'):
    d=json.loads(l); print(d['rank'], d['kernel_ms'], d['ideal_ms'], d['replay_queue_ms'], d['replay_hot16x_first_ms'], d['replay_longest_first_ms'], d['top0.1pct_share'], d['longest'][:3])
"
