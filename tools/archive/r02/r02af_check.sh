# GPU parity suite + tile balance + bench (after the tile-split change)
set -e
O=gpurun_out/${TAG:-r02af}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
echo tests ok
timeout -k 10 300 python tools/rank_balance.py c3 3 > $O/balance_c3.log 2>&1
timeout -k 10 300 python tools/rank_balance.py c2 3 > $O/balance_c2.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
echo done
