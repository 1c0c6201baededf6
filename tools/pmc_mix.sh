#!/bin/bash
# Dynamic VALU instruction mix of the C3 trace kernel beyond the FP64/FP32 classes of
# profile_gpu.sh (conversions, 64-bit integer, f32 transcendentals)
# (stochastic, cycles): which instructions the waves issue. Outputs under gpurun_out/mix_<tag>/.
set -euo pipefail
TAG=${1:-r05}
CFG=${2:-c3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/mix_$TAG
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
B="$R/bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --no-roofline"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_IOPS SQ_WAVES --kernel-trace -d "$O/mix" -o mix --output-format csv -- python3 $B > "$O/mix.log" 2>&1 || echo "mix pass failed"
echo mix done
ls -laR "$O/pcs" >> "$O/pcs.log" 2>&1 || true
echo pcs done
