# round 6 (n): light packing — GPU suite, then C3/C2/C4 and C5 transition frames by DT_PACK_LANES
set -e
O=gpurun_out/r06n; rm -rf $O; mkdir -p $O
export DT_PARITY_LOG=$O/parity.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
j() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2',d['value'],d['roofline']['kernel_ms'],d['ms_per_step'])"; }
b() { n=$1; c=$2; shift 2; st=5; [ $c = c3 ] && st=10; [ $c = c2 ] && st=40; env "$@" timeout -k 10 300 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline > $O/$n.json 2>/dev/null; j $O/$n.json "$n $*"; }
for c in c3 c2 c4; do
b ${c}_base $c DT_LIB=distraytracer_amd/variants/libdt_base.so
b ${c}_p0 $c DT_PACK_LANES=0
b ${c}_p16 $c DT_PACK_LANES=16
b ${c}_p32 $c DT_PACK_LANES=32
b ${c}_p64 $c DT_PACK_LANES=64
done
a() { n=$1; shift; env "$@" timeout -k 10 300 python tools/animate.py --frames 126:140:2 > $O/c5_$n.json 2>/dev/null; python -c "import json;d=json.loads(open('$O/c5_$n.json').read().splitlines()[-1]);print('c5 126:140:2 $n',d['seconds'])"; }
a base DT_LIB=distraytracer_amd/variants/libdt_base.so
a p0 DT_PACK_LANES=0
a p32 DT_PACK_LANES=32
a p64 DT_PACK_LANES=64
