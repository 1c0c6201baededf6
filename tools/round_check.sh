# Round GPU check (TAG env): parity suite, smoke, C3 bench, C2/C4 bench lines,
# C5 animation sample, rocprofv3 kernel-trace stats of the C3 bench.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r02x}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
echo tests ok
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
echo smoke ok
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
echo bench ok
timeout -k 10 200 python bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c2.log 2>&1
timeout -k 10 200 python bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > $O/bench_c4.log 2>&1
echo c2 c4 ok
if [ -z "$NO_C5" ]; then timeout -k 10 300 python tools/animate.py --frames 0:300:30 --per-frame > $O/c5_animate.log 2>&1; echo c5 ok; fi
cd /tmp; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/kt.log 2>&1
echo all done
if [ -n "$TORCHRUN" ]; then timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 $R/bench.py --gpus 1 --steps 5 --warmup 1 --no-cpu-baseline > $O/torchrun_n1.json 2> $O/torchrun_n1.err; echo torchrun ok; fi
