# A/B on one box: previous commit's kernel (variants/libdt_prev.so, host of this tree with umbra off)
# against this tree with DT_SG_UMBRA = 0 / default, on C3, C2, C4 (bench kernel throughput and e2e)
set -e
O=gpurun_out/${TAG:-r02q}; mkdir -p $O
run() { n=$1; cfg=$2; st=$3; shift 3; env "$@" timeout -k 10 300 python bench.py --config $cfg --steps $st --warmup 1 --no-cpu-baseline > $O/$n.json 2>/dev/null; python -c "import json;d=json.loads(open('$O/$n.json').read().splitlines()[-1]);print('$n',d['value'],d['roofline']['kernel_ms'],d.get('end_to_end_ms_per_frame'))"; }
for rep in 1 2; do
for cfg in c3 c2 c4; do
st=10; [ $cfg = c4 ] && st=2
run prev_$cfg $cfg $st DT_SG_UMBRA=0 DT_LIB=distraytracer_amd/variants/libdt_prev.so
run new0_$cfg $cfg $st DT_SG_UMBRA=0
run new1_$cfg $cfg $st DT_SG_UMBRA=1
done
done
