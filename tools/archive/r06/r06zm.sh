# round 6 (zm): umbra cells of point lights decided before the light sample — GPU suite (oracle parity),
# variant bit-identity against HEAD's library (mid), C3/C2/C4 A/B, C5 every 10th frame
set -e
O=gpurun_out/r06zm; rm -rf $O; mkdir -p $O
export DT_PARITY_LOG=$O/parity.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
unset DT_PARITY_LOG
DT_LIB=distraytracer_amd/variants/libdt_mid.so timeout -k 10 300 python tools/variant_check.py $O/mid.npz > $O/vc_mid.log 2>&1
timeout -k 10 300 python tools/variant_check.py $O/new.npz > $O/vc_new.log 2>&1
python tools/variant_check.py --compare $O/mid.npz $O/new.npz | tee $O/variant_compare.log
j() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2',d['value'],d['roofline']['kernel_ms'],d['ms_per_step'])"; }
b() { n=$1; c=$2; shift 2; st=10; [ $c = c2 ] && st=40; [ $c = c4 ] && st=3; env "$@" timeout -k 10 300 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline > $O/$n.json 2>/dev/null; j $O/$n.json "$n $*"; }
for rep in 1 2; do
for c in c3 c2; do
b ${c}_mid_$rep $c DT_LIB=distraytracer_amd/variants/libdt_mid.so
b ${c}_new_$rep $c A=1
done
done
b c4_mid c4 DT_LIB=distraytracer_amd/variants/libdt_mid.so
b c4_new c4 A=1
a() { n=$1; shift; env "$@" timeout -k 10 300 python tools/animate.py --frames 0:300:10 --per-frame > $O/c5_$n.json 2> $O/c5_$n.log; python -c "import json;d=json.loads(open('$O/c5_$n.json').read().splitlines()[-1]);print('c5 0:300:10 $n',d['seconds'],d['abort_counters'])"; }
a mid DT_LIB=distraytracer_amd/variants/libdt_mid.so
a new A=1
echo all done
