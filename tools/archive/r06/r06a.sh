# round 6 (a): chunk items — parity tests, C4 A/B per-pixel vs chunk items, C3 A/B vs prev, C4 rank balance
set -e
O=gpurun_out/r06a; mkdir -p $O
export DT_PARITY_LOG=$O/parity.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_chunks.py tests/test_gpu_configs.py::test_c4_256spp_share tests/test_gpu_launch_path.py > $O/tests.log 2>&1
j() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2',d['value'],d['roofline']['kernel_ms'])"; }
for rep in 1 2; do
for m in 0 1; do
DT_CHUNK_ITEMS=$m timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4_m${m}_$rep.json 2>/dev/null
j $O/c4_m${m}_$rep.json "c4 chunk=$m"
done
DT_LIB=distraytracer_amd/variants/libdt_prev.so timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 1 --no-cpu-baseline > $O/c3_prev_$rep.json 2>/dev/null
j $O/c3_prev_$rep.json "c3 prev"
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 1 --no-cpu-baseline > $O/c3_new_$rep.json 2>/dev/null
j $O/c3_new_$rep.json "c3 new"
done
for m in 0 1; do
DT_CHUNK_ITEMS=$m INFLIGHT=2 WORLDS=1,4,8 timeout -k 10 400 python tools/rank_balance.py c4 2 > $O/rb_c4_m$m.log 2>&1
tail -3 $O/rb_c4_m$m.log
done
