#!/bin/bash
# build_variant.sh NAME KERNEL.hip [extra hipcc flags...] -> distraytracer_amd/variants/libdt_NAME.so
# (A/B experiments: same host objects, a different kernel source or flags; see ab_variants.sh)
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/distraytracer_amd/csrc
name=$1; src=$2; shift 2
make -s -C "$C" >/dev/null
mkdir -p "$R/distraytracer_amd/variants" "$C/build/var"
# the product's code-generation flags (Makefile CODEGEN) unless CODEGEN is set
CG=${CODEGEN--mllvm -disable-machine-licm -mllvm -disable-machine-cse -mllvm -disable-machine-sink -mllvm -disable-licm-promotion -fno-slp-vectorize -fno-vectorize -mllvm -amdgpu-sched-strategy=max-memory-clause -mllvm -disable-tail-duplicate -mllvm -disable-early-taildup -mllvm -enable-load-pre=false -mllvm -enable-misched=false -fno-unroll-loops -mllvm -structurizecfg-skip-uniform-regions=true}
/opt/rocm/bin/hipcc -I"$C" -DDT_TRACE_MIN_WAVES=${W:-4} $CG "$@" --offload-arch=gfx950 -O3 -std=c++17 -fPIC \
  -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt -c "$src" -o "$C/build/var/k_$name.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/distraytracer_amd/variants/libdt_$name.so" \
  "$C/build/var/k_$name.o" "$C"/build/dt_kernels_w5.o "$C"/build/dt_kernels_rpc.o "$C"/build/dt_kernels_dn.o "$C"/build/dt_kernels_isect.o "$C"/build/dt_api.o "$C"/build/host_*.o
echo "built variants/libdt_$name.so"
