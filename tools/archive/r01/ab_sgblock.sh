# Shadow-grid build: per-cell tests (DT_SG_BLOCK=0) against block tests (default). The list hash
# (DT_SG_VERBOSE) must agree; the host stage times come from DT_TIMING.
O=gpurun_out/r01p; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests FAILED"; tail -20 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for c in c3 c2 c4; do for b in 0 1; do
  DT_SG_BLOCK=$b DT_SG_VERBOSE=1 DT_TIMING=1 timeout -k 10 200 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > $O/b_${c}_$b.json 2> $O/b_${c}_$b.err || exit 1
  echo "$c block=$b $(grep -h 'shadow grid:' $O/b_${c}_$b.err | tail -1 | grep -o 'hash.*') $(grep -h 'dt_scene_create shadow grid' $O/b_${c}_$b.err | tail -1) $(python -c "import json;d=json.loads(open('$O/b_${c}_$b.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d.get('end_to_end_ms_per_frame'))")"
done; done
for f in 1200 2160 600; do for b in 0 1; do
  echo "frame $f block=$b $(DT_SG_BLOCK=$b DT_SG_VERBOSE=1 DT_TIMING=1 timeout -k 10 200 python tools/frame_ab.py $f 1920x1080 4 "" 2>&1 | grep -h 'shadow grid:\|dt_scene_create shadow grid\|kernel_ms' | sed 's/.*hash/hash/' | tr '\n' ' ')"
done; done
