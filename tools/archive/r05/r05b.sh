# round-5 GPU check b: parity suite (+ the world-2 process test), smoke, C3 bench, torchrun world 1
# (kernel time with two frames in flight), VALU mix counters and a PC-sampling attempt
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05b}; mkdir -p $O
export DT_PARITY_LOG=$O/parity.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
echo tests ok
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
echo smoke ok
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
echo bench ok
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline > $O/torchrun_n1.json 2> $O/torchrun_n1.err
echo torchrun ok
bash tools/pmc_mix.sh ${TAG:-r05b} c3

DT_LIB=distraytracer_amd/variants/libdt_stamps.so timeout -k 10 200 python tools/stamps.py c3 > $O/stamps_c3.log 2>&1 || echo "stamps c3 failed"
DT_LIB=distraytracer_amd/variants/libdt_stamps.so timeout -k 10 300 python tools/stamps.py c4 > $O/stamps_c4.log 2>&1 || echo "stamps c4 failed"
echo stamps done
echo all done
