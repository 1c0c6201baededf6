#!/bin/bash
# variant_res.sh NAME KERNEL.hip [extra hipcc flags]: compile one trace-kernel variant with the
# product's code-generation flags (KIND=w5 default: the 5-wave room build; KIND=w4, w5_mesh, mesh,
# w5_full, full, w5_tunnel, tunnel, w5_blur, blur, w5_sky, sky, dn, rpc: the Makefile's builds) to
# /tmp/var_NAME.o and print its registers, spills and scratch (no GPU needed). SO=1 also links
# distraytracer_amd/variants/libdt_NAME.so for a GPU A/B (tools/ab_lib.sh VAR=NAME).
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/distraytracer_amd/csrc
name=$1; src=$2; shift 2
CG="-mllvm -disable-machine-licm -mllvm -disable-machine-cse -mllvm -disable-machine-sink -mllvm -disable-licm-promotion -fno-slp-vectorize -fno-vectorize -mllvm -amdgpu-sched-strategy=max-memory-clause -mllvm -disable-tail-duplicate -mllvm -disable-early-taildup -mllvm -enable-load-pre=false -mllvm -enable-misched=false -fno-unroll-loops -mllvm -structurizecfg-skip-uniform-regions=true"
# KIND: the Makefile build (dt_kernels_<KIND>, or dt_kernels for KIND=w4); its flags from the Makefile
case ${KIND:-w5} in
  w4) KO=dt_kernels.o;;
  *) KO=dt_kernels_${KIND:-w5}.o;;
esac
KF=$(make -s -C "$C" flags-${KO%.o})
KN=$(echo "$KF" | sed -n 's/.*-DDT_KNAME=\([a-z0-9_]*\).*/\1/p')
[ -z "$KN" ] && KN=dt_trace_kernel_${KIND}
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
  for o in $(make -s -C "$C" flags-TRACE_BUILDS_LIST 2>/dev/null); do [ $o = $KO ] && objs="$objs /tmp/var_$name.o" || objs="$objs $C/build/$o"; done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/distraytracer_amd/variants/libdt_$name.so" $objs \
    "$C"/build/dt_kernels_isect.o "$C"/build/dt_api.o "$C"/build/host_*.o -lz
  echo "linked distraytracer_amd/variants/libdt_$name.so"
fi
