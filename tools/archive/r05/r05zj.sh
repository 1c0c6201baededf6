# round 5: shipped queue policy (8 segments for split frames of one-chunk items): GPU suite, smoke, rank balance C3/C4
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05zj}; mkdir -p $O
cd $R
export DT_PARITY_LOG=$O/parity.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
INFLIGHT=2 timeout -k 10 300 python tools/rank_balance.py c3 3 > $O/rank_balance_c3.log 2>&1
INFLIGHT=2 WORLDS=1,8 timeout -k 10 300 python tools/rank_balance.py c4 2 > $O/rank_balance_c4.log 2>&1
echo all done
