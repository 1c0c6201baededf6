# round 6 (zj): start-side culling, second step: own-plane bound of tilted rectangles, cylinder boxes,
# one-sided blur movement — bit identity, GPU shadow-grid tests, A/B against HEAD~1 (base) and HEAD (mid)
set -e
O=gpurun_out/r06zj; rm -rf $O; mkdir -p $O
timeout -k 10 600 python tools/sg_start_check.py > $O/sg_start_check.log 2>&1; cat $O/sg_start_check.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_sg_start.py tests/test_gpu_parity.py -m gpu -x -q -k "sg_start or shadow_grid" --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -20 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
j() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2',d['value'],d['roofline']['kernel_ms'],d['ms_per_step'])"; }
b() { n=$1; c=$2; shift 2; st=10; [ $c = c2 ] && st=40; [ $c = c4 ] && st=3; env "$@" timeout -k 10 300 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline > $O/$n.json 2>/dev/null; j $O/$n.json "$n $*"; }
for rep in 1 2; do
for c in c3 c2; do
b ${c}_base_$rep $c DT_LIB=distraytracer_amd/variants/libdt_base.so
b ${c}_mid_$rep $c DT_LIB=distraytracer_amd/variants/libdt_mid.so
b ${c}_new_$rep $c A=1
done
done
b c4_base c4 DT_LIB=distraytracer_amd/variants/libdt_base.so
b c4_new c4 A=1
a() { n=$1; shift; env "$@" timeout -k 10 300 python tools/animate.py --frames 0:300:10 --per-frame > $O/c5_$n.json 2> $O/c5_$n.log; python -c "import json;d=json.loads(open('$O/c5_$n.json').read().splitlines()[-1]);print('c5 0:300:10 $n',d['seconds'],d['abort_counters'])"; }
a base DT_LIB=distraytracer_amd/variants/libdt_base.so
a new A=1
echo all done
