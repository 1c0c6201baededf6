# A/B on one box: variants/libdt_$VAR.so (default prev) against this tree's libdt.so on C3, C2, C4
# (bench kernel throughput), twice, interleaved. TAG names the output directory.
set -e
O=gpurun_out/${TAG:-ab}; mkdir -p $O; V=${VAR:-prev}
run() { n=$1; cfg=$2; st=$3; shift 3; env "$@" timeout -k 10 300 python bench.py --config $cfg --steps $st --warmup 1 --no-cpu-baseline > $O/$n.json 2>/dev/null; python -c "import json;d=json.loads(open('$O/$n.json').read().splitlines()[-1]);print('$n',d['value'],d['roofline']['kernel_ms'])"; }
for rep in 1 2; do
for cfg in ${CFGS:-c3 c2 c4}; do
st=10; [ $cfg = c4 ] && st=2
run ${V}_$cfg $cfg $st DT_LIB=distraytracer_amd/variants/libdt_$V.so
run new_$cfg $cfg $st A=1
done
done
