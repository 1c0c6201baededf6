# round 5: PMC comparison of the whole-frame repeat launch against the 8 share launches (tools/share_pmc.py)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05zb}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/share_pmc.py > $O/times.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_WAVES -d $O/pmc1 -o p --output-format csv -- python3 $R/tools/share_pmc.py > $O/pmc1.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQC_ICACHE_MISSES SQC_DCACHE_MISSES GRBM_GUI_ACTIVE -d $O/pmc2 -o p --output-format csv -- python3 $R/tools/share_pmc.py > $O/pmc2.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/pmc3 -o p --output-format csv -- python3 $R/tools/share_pmc.py > $O/pmc3.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/pmc4 -o p --output-format csv -- python3 $R/tools/share_pmc.py > $O/pmc4.log 2>&1
echo all done
