# round-5 GPU check x: the repeat launch with sky items (new test), then parity over all 300 C5
# animation frames at 96x54 (64 spp, depth 10) against the oracle
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05x}; mkdir -p $O
export DT_PARITY_LOG=$O/parity.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_launch_path.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/launch_path_tests.log 2>&1 || { tail -30 $O/launch_path_tests.log; exit 1; }
echo tests ok
timeout -k 10 900 python -u tools/parity_sweep.py 96x54 1 0 300 > $O/parity_sweep_all.log 2>&1
tail -1 $O/parity_sweep_all.log
