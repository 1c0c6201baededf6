# round 5: the split path after the C4 tile change: distributed and boundary GPU tests, C4 bench at world 1 via torchrun
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05zm}; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_boundary.py tests/test_gpu_edges.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
echo all done
