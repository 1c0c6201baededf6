# tile order A/B: per-rank balance with and without DT_TILE_ORDER, parity suite, bench vs previous kernel
set -e
O=gpurun_out/r02ah; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
echo tests ok
timeout -k 10 300 python tools/rank_balance.py c3 3 > $O/balance_c3.log 2>&1
DT_TILE_ORDER=0 timeout -k 10 300 python tools/rank_balance.py c3 3 > $O/balance_c3_noorder.log 2>&1
timeout -k 10 300 python tools/rank_balance.py c2 3 > $O/balance_c2.log 2>&1
TAG=r02ah CFGS="c3 c2" bash tools/ab_lib.sh > $O/ab.log 2>&1
echo done
