#!/bin/bash
# Instruction-fetch counters of dt_trace_kernel on the C3 bench (GPU box):
#   TAG=r03ay bash tools/icache_pmc.sh [DT_LIB=path ...]
# One PMC pass of its own (SQC block only), as tools/profile_gpu.sh does for the others.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-icache}/icache
mkdir -p "$O"
cd /tmp; export TMPDIR=/tmp
B="$R/bench.py --config c3 --steps 1 --warmup 0 --no-cpu-baseline --no-roofline"
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH \
  SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --kernel-trace -d "$O" -o ic --output-format csv -- python3 $B > "$O/log" 2>&1 \
  || { echo "icache pass failed"; tail -5 "$O/log"; exit 0; }
python3 - "$O" <<'PY'
import csv, glob, sys
rows = [r for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True) for r in csv.DictReader(open(f))]
acc = {}
for r in rows:
    if "dt_trace_kernel" in r.get("Kernel_Name", ""):
        acc[r["Counter_Name"]] = acc.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
print("icache", {k: "%.4g" % v for k, v in sorted(acc.items())})
PY
