# round-5 GPU check v: the repeat launch's per-item copy arithmetic (division: product; subtraction:
# repsub; none: norepeat) on C3
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05v}; mkdir -p $O
V=distraytracer_amd/variants
b() {   # name, env, config, steps
  env $2 timeout -k 10 200 python bench.py --config $3 --steps $4 --warmup 1 --no-cpu-baseline --no-roofline > $O/$1.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/$1.json').read().splitlines()[-1]);print('$1',d['value'],d['roofline']['kernel_ms'])" >> $O/ab.txt
}
for rep in 1 2 3; do
  b c3_div_$rep "DT_X=0" c3 8; b c3_sub_$rep "DT_LIB=$V/libdt_repsub.so" c3 8; b c3_none_$rep "DT_LIB=$V/libdt_norepeat.so" c3 8
done
echo all done
