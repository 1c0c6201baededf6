# round-5 GPU check u: does the repeat-launch arithmetic cost the per-frame kernels (C2, C3, C4)?
# product against the same tree with the copies compiled out (DT_REPEAT=0); batch sizes 4 and 6
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05u}; mkdir -p $O
V=distraytracer_amd/variants
b() {   # name, env, config, steps
  env $2 timeout -k 10 200 python bench.py --config $3 --steps $4 --warmup 1 --no-cpu-baseline --no-roofline > $O/$1.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/$1.json').read().splitlines()[-1]);print('$1',d['value'],d['roofline']['kernel_ms'])" >> $O/ab.txt
}
for rep in 1 2; do
  b c2_prod_$rep "DT_X=0" c2 10; b c2_norep_$rep "DT_LIB=$V/libdt_norepeat.so" c2 10
  b c3_prod_$rep "DT_X=0" c3 8; b c3_norep_$rep "DT_LIB=$V/libdt_norepeat.so" c3 8
  b c3_b4_$rep "DT_BATCH_SIZE=4" c3 8; b c3_b6_$rep "DT_BATCH_SIZE=6" c3 8
  b c4_prod_$rep "DT_X=0" c4 2; b c4_norep_$rep "DT_LIB=$V/libdt_norepeat.so" c4 2
done
echo all done
