# round-5 GPU check o: MachineSink on (product); the rank's tiles handed out in Morton order
# (DT_TILE_ORDER=morton): identity, C3/C2 A/B at N=1, the N=8 share with two frames in flight
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05o}; mkdir -p $O
export DT_PARITY_LOG=$O/parity.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
echo tests ok
timeout -k 10 300 python -u tools/variant_check.py $O/raster.npz > $O/raster.log 2>&1
DT_TILE_ORDER=morton timeout -k 10 300 python -u tools/variant_check.py $O/morton.npz > $O/morton.log 2>&1
python tools/variant_check.py --compare $O/raster.npz $O/morton.npz > $O/compare.log 2>&1 || true
echo identity done
b() {   # name, env, config, steps
  env $2 timeout -k 10 200 python bench.py --config $3 --steps $4 --warmup 1 --no-cpu-baseline --no-roofline > $O/$1.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/$1.json').read().splitlines()[-1]);print('$1',d['value'],d['roofline']['kernel_ms'])" >> $O/ab.txt
}
for rep in 1 2; do
  b c3_raster_$rep "DT_TILE_ORDER=raster" c3 8; b c3_morton_$rep "DT_TILE_ORDER=morton" c3 8
  b c2_raster_$rep "DT_TILE_ORDER=raster" c2 10; b c2_morton_$rep "DT_TILE_ORDER=morton" c2 10
done
echo ab done
WORLDS=1,8 INFLIGHT=2 timeout -k 10 300 python tools/rank_balance.py c3 3 > $O/rb_raster.log 2>&1
DT_TILE_ORDER=morton WORLDS=1,8 INFLIGHT=2 timeout -k 10 300 python tools/rank_balance.py c3 3 > $O/rb_morton.log 2>&1
echo all done
