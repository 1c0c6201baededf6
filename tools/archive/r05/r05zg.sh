# round 5: segmented queue for split frames by default (world > 1): shares at N = 2, 4, 8 against one counter
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05zg}; mkdir -p $O
cd $R
for rep in 1 2; do
for v in "DT_X=0" "DT_QUEUE_SEGS=1"; do
  echo "# $v (rep $rep)" >> $O/rb.log
  env $v INFLIGHT=2 timeout -k 10 200 python3 $R/tools/rank_balance.py c3 3 2>/dev/null >> $O/rb.log
done
done
echo rb done
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_boundary.py tests/test_gpu_launch_path.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
echo all done
