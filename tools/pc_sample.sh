#!/bin/bash
# PC sampling of the trace kernel (rocprofv3 host-trap sampling, beta): which instructions the
# waves sit on, for tools/pc_hist.py. Run on the GPU box via gpurun; outputs under gpurun_out/pcs_<tag>/.
set -euo pipefail
TAG=${1:-r04}
CFG=${2:-c3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pcs_$TAG
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
  --pc-sampling-interval ${PCS_INTERVAL:-4} -d "$O" -o pcs --output-format csv -- \
  python3 $R/bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --no-roofline > "$O/run.log" 2>&1
ls -la "$O" >> "$O/run.log"
