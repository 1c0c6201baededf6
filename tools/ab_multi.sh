# A/B of several variants on one box: distraytracer_amd/variants/libdt_<v>.so for v in $VARS against
# this tree's libdt.so, on $CFGS (default c3 c2), $REPS interleaved repetitions (default 2).
# TAG names the output directory under gpurun_out/. Prints "name Mpixel-samples/s kernel-ms".
set -e
O=gpurun_out/${TAG:-ab}; mkdir -p $O
run() { n=$1; cfg=$2; st=$3; shift 3; env "$@" timeout -k 10 300 python bench.py --config $cfg --steps $st --warmup 1 --no-cpu-baseline --no-roofline > $O/$n.json 2>/dev/null; python -c "import json;d=json.loads(open('$O/$n.json').read().splitlines()[-1]);print('$n',d['value'],d['roofline']['kernel_ms'])"; }
for rep in $(seq 1 ${REPS:-2}); do
for cfg in ${CFGS:-c3 c2}; do
st=10; [ $cfg = c4 ] && st=2
for v in $VARS; do run ${v}_${cfg}_$rep $cfg $st DT_LIB=distraytracer_amd/variants/libdt_$v.so; done
run new_${cfg}_$rep $cfg $st A=1
done
done
