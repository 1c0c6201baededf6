# round 6 (zn): early umbra off in the 4-wave room build (C2's kernel) — C2/C3 A/B against HEAD's library
set -e
O=gpurun_out/r06zn; rm -rf $O; mkdir -p $O
j() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2',d['value'],d['roofline']['kernel_ms'],d['ms_per_step'])"; }
b() { n=$1; c=$2; shift 2; st=10; [ $c = c2 ] && st=40; env "$@" timeout -k 10 300 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline > $O/$n.json 2>/dev/null; j $O/$n.json "$n $*"; }
for rep in 1 2 3; do
b c2_mid_$rep c2 DT_LIB=distraytracer_amd/variants/libdt_mid.so
b c2_new_$rep c2 A=1
done
b c3_mid c3 DT_LIB=distraytracer_amd/variants/libdt_mid.so
b c3_new c3 A=1
echo all done
