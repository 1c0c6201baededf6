# round 6 (u): start-side culling of the shadow-grid lists — bit identity (lists built with and
# without it), C3/C2 A/B, the oracle tests of the configs
set -e
O=gpurun_out/r06u; rm -rf $O; mkdir -p $O
timeout -k 10 600 python tools/sg_start_check.py > $O/sg_start_check.log 2>&1; cat $O/sg_start_check.log
j() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2',d['value'],d['roofline']['kernel_ms'],d['ms_per_step'])"; }
b() { n=$1; c=$2; shift 2; st=10; [ $c = c2 ] && st=40; env "$@" timeout -k 10 300 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline > $O/$n.json 2>/dev/null; j $O/$n.json "$n $*"; }
for rep in 1 2; do
for c in c3 c2; do
b ${c}_off_$rep $c DT_SG_START=0
b ${c}_on_$rep $c A=1
done
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_configs.py > $O/gpu_configs.log 2>&1; tail -3 $O/gpu_configs.log
