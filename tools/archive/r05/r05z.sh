# round-5 final check of the shipped tree: GPU suite (parity log), smoke, the default bench line
# (C3, N=1), C2/C4 lines, torchrun world 1, rank balance (two frames in flight), the rocprofv3 kernel
# trace + PMC passes (tools/profile_gpu.sh), the VALU mix, the 300-frame C5 run
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05z}; mkdir -p $O
export DT_PARITY_LOG=$O/parity.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
echo tests ok
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
echo smoke ok
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python bench.py --config c2 --steps 10 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err
timeout -k 10 300 python bench.py --config c4 --steps 3 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err
echo bench ok
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline > $O/torchrun_n1.json 2> $O/torchrun_n1.err
echo torchrun ok
INFLIGHT=2 timeout -k 10 300 python tools/rank_balance.py c3 3 > $O/rank_balance_inflight2.log 2>&1
echo rb ok
timeout -k 10 900 bash tools/profile_gpu.sh ${TAG:-r05z} c3 > $O/profile.log 2>&1
bash tools/pmc_mix.sh ${TAG:-r05z} c3 > $O/mix.log 2>&1 || true
echo prof ok
timeout -k 10 400 python tools/animate.py --frames 0:300:1 --per-frame > $O/c5_full.log 2>&1
echo all done
