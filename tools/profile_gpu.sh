#!/bin/bash
# GPU profiling recipe (run on the GPU box via gpurun). Kernel trace + stats of the bench
# workload, then separate PMC passes (one TCC counter group per pass, as the MI355X guide
# prescribes; never combined with runtime/sys tracing). Outputs under gpurun_out/prof_<tag>/.
set -euo pipefail
TAG=${1:-r01}
CFG=${2:-c3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_$TAG
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
B="$R/bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --no-roofline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- python3 $B > "$O/kt.log" 2>&1
echo kt done
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$O/fetch" -o fetch --output-format csv -- python3 $B > "$O/fetch.log" 2>&1
echo fetch done
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$O/write" -o write --output-format csv -- python3 $B > "$O/write.log" 2>&1
echo write done
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS --kernel-trace -d "$O/sq" -o sq --output-format csv -- python3 $B > "$O/sq.log" 2>&1
echo sq done
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE --kernel-trace -d "$O/sq2" -o sq2 --output-format csv -- python3 $B > "$O/sq2.log" 2>&1 || echo "sq2 pass failed (counter names?)"
echo sq2 done
timeout -k 10 400 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA --kernel-trace -d "$O/sq3" -o sq3 --output-format csv -- python3 $B > "$O/sq3.log" 2>&1 || echo "sq3 pass failed"
echo sq3 done
timeout -k 10 400 rocprofv3 --pmc SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_SMEM SQ_INST_CYCLES_SALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_INT32 --kernel-trace -d "$O/sq4" -o sq4 --output-format csv -- python3 $B > "$O/sq4.log" 2>&1 || echo "sq4 pass failed"
timeout -k 10 400 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCC_HIT_sum TCC_MISS_sum SQC_ICACHE_MISSES SQC_DCACHE_MISSES --kernel-trace -d "$O/l2" -o l2 --output-format csv -- python3 $B > "$O/l2.log" 2>&1 || echo "l2 pass failed"
echo all done
