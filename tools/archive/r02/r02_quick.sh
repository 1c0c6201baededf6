# quick GPU A/B: parity suite + bench + stamps (TAG env)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r02x}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
echo tests ok
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
python -c "import json;d=json.loads(open('$O/bench.json').read().splitlines()[-1]);print('c3',d['value'],d['roofline']['kernel_ms'])"
timeout -k 10 300 python bench.py --config c2 --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_c2.json 2>/dev/null
python -c "import json;d=json.loads(open('$O/bench_c2.json').read().splitlines()[-1]);print('c2',d['value'],d['roofline']['kernel_ms'])"
if [ -n "$C4" ]; then timeout -k 10 300 python bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > $O/bench_c4.json 2>/dev/null
python -c "import json;d=json.loads(open('$O/bench_c4.json').read().splitlines()[-1]);print('c4',d['value'],d['roofline']['kernel_ms'])"; fi
if [ -f distraytracer_amd/variants/libdt_stamps.so ]; then DT_LIB=distraytracer_amd/variants/libdt_stamps.so timeout -k 10 200 python tools/stamps.py c3 > $O/stamps_c3.log 2>&1; fi
echo all done
