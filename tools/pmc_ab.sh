#!/bin/bash
# A/B instruction mix of dt_trace_kernel for library variants (GPU box):
#   pmc_ab.sh NAME=path/to/libdt.so ...   -> gpurun_out/pmcab_NAME/ + one summary line each
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp; export TMPDIR=/tmp
B="$R/bench.py --config c3 --steps 1 --warmup 0 --no-cpu-baseline"
for kv in "$@"; do
  n=${kv%%=*}; so=${kv#*=}
  O=$R/gpurun_out/pmcab_$n
  mkdir -p $O
  DT_LIB=$so timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_BUSY_CYCLES --kernel-trace -d $O -o sq --output-format csv -- python3 $B > $O/log 2>&1 || { echo "$n failed"; break; }
  python3 - "$O" "$n" <<'PY'
import csv, glob, sys
rows = [r for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True) for r in csv.DictReader(open(f))]
acc = {}
for r in rows:
    if "dt_trace_kernel" in r.get("Kernel_Name", ""):
        acc[r["Counter_Name"]] = acc.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
print(sys.argv[2], {k: "%.4g" % v for k, v in sorted(acc.items())})
PY
done
