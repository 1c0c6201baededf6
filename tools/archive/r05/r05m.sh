# round-5 GPU check m: code-generation flag sweep, each remaining CODEGEN flag dropped in turn (the
# flags with no effect on the code, and the additions tried, produce the product's ISA byte for byte):
# C3 and C2 A/B against the product, two rounds
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05m}; mkdir -p $O
V=distraytracer_amd/variants
b() {   # name, lib ("" = product), config, steps
  local lib=""; [ -n "$2" ] && lib="DT_LIB=$V/libdt_$2.so"
  env $lib timeout -k 10 200 python bench.py --config $3 --steps $4 --warmup 1 --no-cpu-baseline --no-roofline > $O/$1.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/$1.json').read().splitlines()[-1]);print('$1',d['value'],d['roofline']['kernel_ms'])" >> $O/ab.txt
}
for rep in 1 2; do
  b c3_prod_$rep "" c3 8
  for v in d1 d2 d3 d6 d7 d8 d9 d10; do b c3_${v}_$rep cg_$v c3 8; done
done
for rep in 1 2; do
  b c2_prod_$rep "" c2 10
  for v in d1 d2 d3 d6 d7 d8 d9 d10; do b c2_${v}_$rep cg_$v c2 10; done
done
echo all done
