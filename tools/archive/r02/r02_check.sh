# round-2 GPU check: parity suite, smoke, bench (N=1), and the RCCL path of bench.py under
# torch.distributed.run at world size 1 (the only world size a 1-GPU box can run)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r02a}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo tests ok
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $O/bench.json 2> $O/bench.err
echo bench ok
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_dist1.json 2> $O/bench_dist1.err
echo all done
