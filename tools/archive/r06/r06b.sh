# round 6 (b): chunk items with the sum kernel — tests, C4 queue matrix at N=1, C3 against round 5
set -e
O=gpurun_out/r06b; rm -rf $O; mkdir -p $O
export DT_PARITY_LOG=$O/parity.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_chunks.py tests/test_gpu_configs.py::test_c4_256spp_share tests/test_gpu_launch_path.py > $O/tests.log 2>&1
j() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2',d['value'],d['roofline']['kernel_ms'])"; }
b() { n=$1; c=$2; shift 2; st=3; [ $c = c3 ] && st=10; env "$@" timeout -k 10 300 python bench.py --config $c --steps $st --warmup 1 --no-cpu-baseline > $O/$n.json 2>/dev/null; j $O/$n.json "$n $*"; }
for rep in 1 2; do
b c4_m0_$rep c4 DT_CHUNK_ITEMS=0
b c4_b1_s1_$rep c4 DT_CHUNK_ITEMS=1
b c4_b2_s1_$rep c4 DT_CHUNK_ITEMS=1 DT_BATCH_SIZE=2
b c4_b4_s1_$rep c4 DT_CHUNK_ITEMS=1 DT_BATCH_SIZE=4
b c4_b1_s8_$rep c4 DT_CHUNK_ITEMS=1 DT_QUEUE_SEGS=8
b c4_b2_s8_$rep c4 DT_CHUNK_ITEMS=1 DT_QUEUE_SEGS=8 DT_BATCH_SIZE=2
b c3_r05_$rep c3 DT_LIB=distraytracer_amd/variants/libdt_r05.so
b c3_new_$rep c3 A=1
done
