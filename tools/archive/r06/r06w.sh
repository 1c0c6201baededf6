# round 6 (w): umbra lanes in scattered shadow waves — C3/C2/C4 against HEAD, grid tests, configs
set -e
O=gpurun_out/r06w; rm -rf $O; mkdir -p $O
j() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2',d['value'],d['roofline']['kernel_ms'],d['ms_per_step'])"; }
b() { n=$1; c=$2; shift 2; st=10; [ $c = c2 ] && st=40; [ $c = c4 ] && st=4; env "$@" timeout -k 10 300 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline > $O/$n.json 2>/dev/null; j $O/$n.json "$n $*"; }
for rep in 1 2; do
for c in c3 c2 c4; do
b ${c}_base_$rep $c DT_LIB=distraytracer_amd/variants/libdt_base.so
b ${c}_new_$rep $c A=1
done
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_parity.py -k "grid or config or final" > $O/gpu_tests.log 2>&1; tail -3 $O/gpu_tests.log
