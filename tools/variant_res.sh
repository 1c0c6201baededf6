#!/bin/bash
# variant_res.sh NAME KERNEL.hip [extra hipcc flags]: compile one trace-kernel variant with the
# product's code-generation flags (KIND=w5 default: the 5-wave room build; KIND=w4, w5f/w4f (any
# scene), w5b/w4b (motion blur), dn, rpc) to
# /tmp/var_NAME.o and print its registers, spills and scratch (no GPU needed). SO=1 also links
# distraytracer_amd/variants/libdt_NAME.so for a GPU A/B (tools/ab_lib.sh VAR=NAME).
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/distraytracer_amd/csrc
name=$1; src=$2; shift 2
CG="-mllvm -disable-machine-licm -mllvm -disable-machine-cse -mllvm -disable-machine-sink -mllvm -disable-licm-promotion -fno-slp-vectorize -fno-vectorize -mllvm -amdgpu-sched-strategy=max-memory-clause -mllvm -disable-tail-duplicate -mllvm -disable-early-taildup -mllvm -enable-load-pre=false -mllvm -enable-misched=false -fno-unroll-loops -mllvm -structurizecfg-skip-uniform-regions=true"
W5="-DDT_W5=1 -DDT_TRACE_MIN_WAVES=5 -DDT_PSUM_LDS=2"; ROOM="-DDT_NOSHIFT=1 -DDT_FEATURES=DT_ROOM_FEATURES"
case ${KIND:-w5} in
  w5) KF="$W5 $ROOM"; KO=dt_kernels_w5.o; KN=dt_trace_kernel_w5;;
  w4) KF="-DDT_TRACE_MIN_WAVES=4 $ROOM"; KO=dt_kernels.o; KN=dt_trace_kernel;;
  w5f) KF="$W5 -DDT_NOSHIFT=1"; KO=dt_kernels_w5_full.o; KN=dt_trace_kernel_w5_full;;
  w4f) KF="-DDT_TRACE_MIN_WAVES=4 -DDT_NOSHIFT=1"; KO=dt_kernels_full.o; KN=dt_trace_kernel_full;;
  w5b) KF="$W5"; KO=dt_kernels_w5_blur.o; KN=dt_trace_kernel_w5_blur;;
  w4b) KF="-DDT_TRACE_MIN_WAVES=4"; KO=dt_kernels_blur.o; KN=dt_trace_kernel_blur;;
  dn) KF="-DDT_TRACE_MIN_WAVES=4 -DDT_DONATE=1"; KO=dt_kernels_dn.o; KN=dt_trace_kernel_dn;;
  rpc) KF="-DDT_TRACE_MIN_WAVES=4 -DDT_WITH_RPC=1"; KO=dt_kernels_rpc.o; KN=dt_trace_kernel_rpc;;
esac
/opt/rocm/bin/hipcc -I"$C" $KF $CG "$@" --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
  -fhip-fp32-correctly-rounded-divide-sqrt -c "$src" -o /tmp/var_$name.o
python3 -c "
import sys; sys.path.insert(0, '$R/tools')
import kernel_resources as K
r = K.resources('/tmp/var_$name.o')['$KN']
print('$name', ' '.join('%s=%s' % (k, r[k]) for k in ('vgpr_count', 'vgpr_spill_count', 'sgpr_count', 'sgpr_spill_count', 'private_segment_fixed_size', 'group_segment_fixed_size')))"
if [ "${SO:-0}" = 1 ]; then
  mkdir -p "$R/distraytracer_amd/variants"
  objs=""
  for o in dt_kernels.o dt_kernels_full.o dt_kernels_blur.o dt_kernels_w5.o dt_kernels_w5_full.o dt_kernels_w5_blur.o dt_kernels_rpc.o dt_kernels_dn.o; do [ $o = $KO ] && objs="$objs /tmp/var_$name.o" || objs="$objs $C/build/$o"; done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/distraytracer_amd/variants/libdt_$name.so" $objs \
    "$C"/build/dt_kernels_isect.o "$C"/build/dt_api.o "$C"/build/host_*.o -lz
  echo "linked distraytracer_amd/variants/libdt_$name.so"
fi
