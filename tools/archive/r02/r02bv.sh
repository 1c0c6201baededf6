set -e
O=gpurun_out/r02bv; mkdir -p $O
timeout -k 10 300 python tools/rank_balance.py c3 3 > $O/balance_c3.log 2>&1
echo done
