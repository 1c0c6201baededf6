#!/bin/bash
# PC sampling of the bench workload (host-trap, time based) -> gpurun_out/pcs/
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pcs
mkdir -p $O
cd /tmp; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -i -A3 "pc.sampl\|pc_sampl" $O/avail.txt | head -40 > $O/pcs_caps.txt || true
timeout -k 10 400 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 -d $O/run -o pcs --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pcs.log 2>&1 || echo "pc sampling failed"
ls -la $O/run/* 2>/dev/null | head
tail -5 $O/pcs.log
