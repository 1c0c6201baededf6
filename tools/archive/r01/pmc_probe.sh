#!/bin/bash
# counter availability + cache-behaviour pass for dt_trace_kernel (GPU box)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/probe
mkdir -p $O
cd /tmp; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $O/avail.txt 2>&1 || echo "list failed"
B="$R/bench.py --config c3 --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_IFETCH --kernel-trace -d $O/ic -o ic --output-format csv -- python3 $B > $O/ic.log 2>&1 || echo "ic pass failed"
timeout -k 10 400 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $O/l2 -o l2 --output-format csv -- python3 $B > $O/l2.log 2>&1 || echo "l2 pass failed"
echo probe done
