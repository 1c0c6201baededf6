#!/bin/bash
# One GPU call of A/B work: bit-identity of every variant in $VARS against this tree's libdt.so
# (tools/variant_check.py), then tools/ab_multi.sh timings. TAG names gpurun_out/<TAG>/.
set -e
O=gpurun_out/${TAG:-ab}; mkdir -p $O
timeout -k 10 300 python tools/variant_check.py $O/base.npz > $O/check_base.log 2>&1
for v in $VARS; do
  DT_LIB=distraytracer_amd/variants/libdt_$v.so timeout -k 10 300 python tools/variant_check.py $O/$v.npz > $O/check_$v.log 2>&1
  python tools/variant_check.py --compare $O/base.npz $O/$v.npz > $O/cmp_$v.log 2>&1 || true
  echo "$v: $(tail -1 $O/cmp_$v.log)"
done
bash tools/ab_multi.sh
if [ "${PMC:-0}" = 1 ]; then
  # VALU / SALU instruction counts of the trace kernel per variant (one C3 frame each)
  for v in base $VARS; do
    lib=distraytracer_amd/libdt.so; [ $v != base ] && lib=distraytracer_amd/variants/libdt_$v.so
    DT_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 --kernel-trace -d $PWD/$O/pmc_$v -o pmc --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-roofline > $O/pmc_$v.log 2>&1
  done
fi
