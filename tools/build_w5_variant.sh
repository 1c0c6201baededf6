#!/bin/bash
# build_w5_variant.sh NAME SRC.hip [extra hipcc flags]: the 5-wave room build (dt_trace_kernel_w5, C3's
# kernel) compiled from SRC with the Makefile's flags (plus extras), linked with this tree's other
# objects -> distraytracer_amd/variants/libdt_NAME.so (same-box A/B: DT_LIB=...)
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/distraytracer_amd/csrc
name=$1; src=$2; shift 2
make -s -C "$C" >/dev/null
F=$(make -s -C "$C" var-HIPFLAGS_BASE); W=$(make -s -C "$C" flags-dt_kernels_w5)
mkdir -p "$C/build/var" "$R/distraytracer_amd/variants"
cp "$src" "$C/_var_$name.hip"
/opt/rocm/bin/hipcc $F $W "$@" -c "$C/_var_$name.hip" -o "$C/build/var/w5_$name.o"
rm -f "$C/_var_$name.hip"
OBJS=$(ls "$C"/build/*.o | grep -v "/dt_kernels_w5.o$\|/work_")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/distraytracer_amd/variants/libdt_$name.so" $OBJS "$C/build/var/w5_$name.o" -lz
python "$R/tools/kernel_resources.py" "$C/build/var/w5_$name.o" | python -c "
import json,sys; d=json.load(sys.stdin)
for k,v in d.items():
  if 'trace' in k: print('$name', k, 'vgpr spills', v['vgpr_spill_count'], 'sgpr spills', v['sgpr_spill_count'])"
