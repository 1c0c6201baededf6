#!/bin/bash
# PMC counts of the trace kernel for this tree's libdt.so ("base") and each variant in $VARS
# (distraytracer_amd/variants/libdt_<v>.so), one C3 frame each ($CFG): gpurun_out/<TAG>/pmc_<v>/.
# Summarise with tools/pmc_compare.py <TAG> [kernel].
set -e
O=gpurun_out/${TAG:-pmcv}; mkdir -p $O
CTRS=${CTRS:-SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_BRANCH}
for v in base $VARS; do
  lib=distraytracer_amd/libdt.so; [ $v != base ] && lib=distraytracer_amd/variants/libdt_$v.so
  DT_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc $CTRS --kernel-trace -d $PWD/$O/pmc_$v -o pmc --output-format csv -- python3 bench.py --config ${CFG:-c3} --steps 1 --warmup 0 --no-cpu-baseline --no-roofline > $O/pmc_$v.log 2>&1
  echo "$v done"
done
