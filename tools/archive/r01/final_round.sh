set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r01r; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 200 python bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c2.log 2>&1
timeout -k 10 200 python bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > $O/bench_c4.log 2>&1
timeout -k 10 300 python tools/animate.py --frames 0:300:30 --per-frame > $O/c5_animate.log 2>&1
cd /tmp; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --config c3 --steps 1 --warmup 0 --no-cpu-baseline > $O/kt.log 2>&1
echo all done
