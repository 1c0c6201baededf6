# round-5 GPU check n: MachineSink back on (drop -disable-machine-sink, variant cg_d1; cg_d1d10 also
# loop unrolling): identity against the product, C3/C4 A/B, C5 sampled frames
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05n}; mkdir -p $O
V=distraytracer_amd/variants
timeout -k 10 300 python -u tools/variant_check.py $O/prod.npz > $O/prod.log 2>&1
for v in cg_d1 cg_d1d10; do
  DT_LIB=$V/libdt_$v.so timeout -k 10 300 python -u tools/variant_check.py $O/$v.npz > $O/$v.log 2>&1
  echo "== $v" >> $O/compare.log; python tools/variant_check.py --compare $O/prod.npz $O/$v.npz >> $O/compare.log 2>&1 || true
done
echo identity done
b() {   # name, lib ("" = product), config, steps
  local lib=""; [ -n "$2" ] && lib="DT_LIB=$V/libdt_$2.so"
  env $lib timeout -k 10 200 python bench.py --config $3 --steps $4 --warmup 1 --no-cpu-baseline --no-roofline > $O/$1.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/$1.json').read().splitlines()[-1]);print('$1',d['value'],d['roofline']['kernel_ms'])" >> $O/ab.txt
}
for rep in 1 2; do
  b c3_prod_$rep "" c3 8; b c3_d1_$rep cg_d1 c3 8; b c3_d1d10_$rep cg_d1d10 c3 8
  b c4_prod_$rep "" c4 2; b c4_d1_$rep cg_d1 c4 2; b c4_d1d10_$rep cg_d1d10 c4 2
done
echo ab done
for v in prod cg_d1; do
  lib=""; [ $v != prod ] && lib="DT_LIB=$V/libdt_$v.so"
  env $lib timeout -k 10 300 python tools/animate.py --frames 100:244:12 --per-frame > $O/c5_$v.log 2>&1 || echo "c5 $v failed"
done
echo all done
