# round-5 GPU check p: the launch-path test (cached records, parity counters); the N=8 share at 4K
# (4x the items per launch: is the share's excess per launch or per item?)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05p}; mkdir -p $O
export DT_PARITY_LOG=$O/parity.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_launch_path.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/launch_path_tests.log 2>&1 || { tail -30 $O/launch_path_tests.log; exit 1; }
echo tests ok
RES=3840x2160 WORLDS=1,8 INFLIGHT=2 timeout -k 10 400 python tools/rank_balance.py c3 2 > $O/rb_4k_inflight2.log 2>&1
RES=3840x2160 WORLDS=1,8 timeout -k 10 400 python tools/rank_balance.py c3 2 > $O/rb_4k_single.log 2>&1
echo all done
