# round-5 GPU check w: parity across the C5 animation (every 5th frame n of buildFinal(n*8) at 96x54,
# 64 spp, depth 10, against the oracle; the work-sharing kernel too on the transition frames)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05w}; mkdir -p $O
timeout -k 10 900 python -u tools/parity_sweep.py 96x54 5 0 300 > $O/parity_sweep.log 2>&1
tail -1 $O/parity_sweep.log
