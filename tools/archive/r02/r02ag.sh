set -e
O=gpurun_out/r02ag; mkdir -p $O
timeout -k 10 300 python tools/rank_balance.py c3 5 > $O/balance_c3.log 2>&1
REVERSE=1 timeout -k 10 300 python tools/rank_balance.py c3 5 > $O/balance_c3_rev.log 2>&1
echo done
