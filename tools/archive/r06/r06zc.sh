# round 6 (zc): hull culling of sphere and cylinder leaves — bit identity against the round-5 lists,
# grid-vs-tree-walk tests, C3/C2/C4 and a C5 sample against HEAD
set -e
O=gpurun_out/r06zc; rm -rf $O; mkdir -p $O
timeout -k 10 600 python tools/sg_start_check.py > $O/sg_start_check.log 2>&1; cat $O/sg_start_check.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_sg_start.py tests/test_gpu_configs.py > $O/gpu_tests.log 2>&1; tail -1 $O/gpu_tests.log
j() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2',d['value'],d['roofline']['kernel_ms'],d['ms_per_step'])"; }
b() { n=$1; c=$2; shift 2; st=10; [ $c = c2 ] && st=40; [ $c = c4 ] && st=4; env "$@" timeout -k 10 300 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline --no-roofline > $O/$n.json 2>/dev/null; python -c "import json;d=json.loads(open('$O/$n.json').read().splitlines()[-1]);print('$n $*',d['value'],d['ms_per_step'])"; }
for rep in 1 2; do
for c in c3 c2 c4; do
b ${c}_base_$rep $c DT_LIB=distraytracer_amd/variants/libdt_base.so
b ${c}_new_$rep $c A=1
done
done
a() { n=$1; shift; env "$@" timeout -k 10 300 python tools/animate.py --frames 0:300:10 --per-frame > $O/c5_$n.json 2> $O/c5_$n.log; python -c "import json;d=json.loads(open('$O/c5_$n.json').read().splitlines()[-1]);print('c5 0:300:10 $n',d['seconds'],d['abort_counters'])"; }
a base DT_LIB=distraytracer_amd/variants/libdt_base.so
a new A=1
a base2 DT_LIB=distraytracer_amd/variants/libdt_base.so
a new2 A=1
