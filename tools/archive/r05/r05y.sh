# round-5 GPU check y: Philox products as 32x32->64 multiplies (DT_PHILOX_MAD64=1, variant mad64):
# identity against the product, C3/C2/C4 A/B
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05y}; mkdir -p $O
V=distraytracer_amd/variants
timeout -k 10 300 python -u tools/variant_check.py $O/prod.npz > $O/prod.log 2>&1
DT_LIB=$V/libdt_mad64.so timeout -k 10 300 python -u tools/variant_check.py $O/mad64.npz > $O/mad64.log 2>&1
python tools/variant_check.py --compare $O/prod.npz $O/mad64.npz > $O/compare.log 2>&1 || true
echo identity done
timeout -k 10 300 python -u -m pytest tests/test_gpu_animation.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/animation_tests.log 2>&1 || { tail -30 $O/animation_tests.log; exit 1; }
echo animation ok
b() {   # name, env, config, steps
  env $2 timeout -k 10 200 python bench.py --config $3 --steps $4 --warmup 1 --no-cpu-baseline --no-roofline > $O/$1.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/$1.json').read().splitlines()[-1]);print('$1',d['value'],d['roofline']['kernel_ms'])" >> $O/ab.txt
}
for rep in 1 2 3; do
  b c3_prod_$rep "DT_X=0" c3 8; b c3_mad64_$rep "DT_LIB=$V/libdt_mad64.so" c3 8
done
for rep in 1 2; do
  b c2_prod_$rep "DT_X=0" c2 10; b c2_mad64_$rep "DT_LIB=$V/libdt_mad64.so" c2 10
  b c4_prod_$rep "DT_X=0" c4 2; b c4_mad64_$rep "DT_LIB=$V/libdt_mad64.so" c4 2
done
echo all done
