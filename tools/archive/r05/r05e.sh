# round-5 GPU check e: the product without -disable-machine-cse (the flag that makes LLVM emit
# unencodable 64-bit SALU literals) and, on top, the called sky march in the blur builds:
# bit identity against the product, then same-box A/Bs (C3, C2, C4, C5 blur frames)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05e}; mkdir -p $O
V=distraytracer_amd/variants
timeout -k 10 300 python -u tools/variant_check.py $O/base.npz > $O/base.log 2>&1
DT_LIB=$V/libdt_nocse.so timeout -k 10 300 python -u tools/variant_check.py $O/nocse.npz > $O/nocse.log 2>&1
DT_LIB=$V/libdt_nocse_skycall.so timeout -k 10 300 python -u tools/variant_check.py $O/nocse_skycall.npz > $O/nocse_skycall.log 2>&1
for v in nocse nocse_skycall; do echo "== $v"; python tools/variant_check.py --compare $O/base.npz $O/$v.npz || true; done > $O/compare.log 2>&1
echo identity done
b() {   # name, lib ("" = product), config, steps
  local lib=""; [ -n "$2" ] && lib="DT_LIB=$V/libdt_$2.so"
  env $lib timeout -k 10 200 python bench.py --config $3 --steps $4 --warmup 1 --no-cpu-baseline --no-roofline > $O/$1.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/$1.json').read().splitlines()[-1]);print('$1',d['value'],d['roofline']['kernel_ms'])" >> $O/ab.txt
}
for rep in 1 2; do
  b c3_base_$rep "" c3 10; b c3_nocse_$rep nocse c3 10
  b c2_base_$rep "" c2 10; b c2_nocse_$rep nocse c2 10
  b c4_base_$rep "" c4 2; b c4_nocse_$rep nocse c4 2
done
echo ab done
for v in base nocse nocse_skycall; do
  lib=""; [ $v != base ] && lib="DT_LIB=$V/libdt_$v.so"
  env $lib timeout -k 10 300 python tools/animate.py --frames 140:244:8 --per-frame > $O/c5_blur_$v.log 2>&1 || echo "c5 $v failed"
done
echo c5 done
