#!/bin/bash
# Builds tools/call_repro/build/repro_<tag> for the called-function defect: the sky
# kernels of dt_kernels.hip's DT_REPRO mode (cloud_color_lane inlined vs called) under the product's
# code-generation flags (csrc/Makefile CODEGEN: "all"), none of them ("none"), each flag alone
# ("only_<k>") and all but one ("drop_<k>"). No GPU needed; run them with tools/call_repro/run.sh.
set -euo pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
C=$R/distraytracer_amd/csrc
B=$R/tools/call_repro/build
mkdir -p "$B"
FLAGS=("-mllvm -disable-machine-licm" "-mllvm -disable-machine-cse" "-mllvm -disable-machine-sink"
       "-mllvm -disable-licm-promotion" "-fno-slp-vectorize" "-fno-vectorize"
       "-mllvm -amdgpu-sched-strategy=max-memory-clause" "-mllvm -disable-tail-duplicate"
       "-mllvm -disable-early-taildup" "-mllvm -enable-load-pre=false" "-mllvm -enable-misched=false"
       "-fno-unroll-loops" "-mllvm -structurizecfg-skip-uniform-regions=true")
BASE="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -std=c++17 -I"$R" -c "$R/tools/call_repro/repro_main.cpp" -o "$B/main.o" 2>/dev/null
build() {   # tag, codegen flags
  local tag=$1; shift
  /opt/rocm/bin/hipcc $BASE "$@" -DDT_REPRO=1 -I"$C" -c "$C/dt_kernels.hip" -o "$B/k_$tag.o" 2>/dev/null
  /opt/rocm/bin/hipcc --offload-arch=gfx950 "$B/main.o" "$B/k_$tag.o" \
    -o "$B/repro_$tag" -L"$R/distraytracer_amd" -ldt -Wl,-rpath,"\$ORIGIN/../../../distraytracer_amd" 2>/dev/null
}
ALL="${FLAGS[*]}"
build none &
build all $ALL &
wait
for k in "${!FLAGS[@]}"; do
  build only_$k ${FLAGS[$k]} &
  drop=""
  for j in "${!FLAGS[@]}"; do [ $j = $k ] || drop="$drop ${FLAGS[$j]}"; done
  build drop_$k $drop &
  if [ $((k % 4)) = 3 ]; then wait; fi
done
wait
ls "$B" | grep -c '^repro_'
for k in "${!FLAGS[@]}"; do echo "$k ${FLAGS[$k]}"; done > "$B/flags.txt"
