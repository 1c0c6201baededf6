# round 6 (zp): C5 parity sweep of the final tree against the oracle: all 300 frames at 96x54,
# every 3rd frame at 192x108
set -e
O=gpurun_out/r06zp; rm -rf $O; mkdir -p $O
timeout -k 10 500 python tools/parity_sweep.py 96x54 1 > $O/c5_parity_sweep_all.log 2>&1; tail -1 $O/c5_parity_sweep_all.log
timeout -k 10 500 python tools/parity_sweep.py 192x108 3 > $O/c5_parity_sweep_192.log 2>&1; tail -1 $O/c5_parity_sweep_192.log
echo all done
