# Shadow-grid block sizes: list hash and build time per size (C4 and C3, DT_TIMING)
O=gpurun_out/r01q; mkdir -p $O
for c in c4 c3; do for b in 0 4x2 8x4 16x4 16x8 32x8; do
  DT_SG_BLOCK=$b DT_SG_VERBOSE=1 DT_TIMING=1 timeout -k 10 200 python bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline > $O/b_${c}_$b.json 2> $O/b_${c}_$b.err || exit 1
  echo "$c block=$b $(grep -h 'shadow grid:' $O/b_${c}_$b.err | tail -1 | grep -o 'hash.*') $(grep -h 'dt_scene_create shadow grid' $O/b_${c}_$b.err | tail -1) $(python -c "import json;d=json.loads(open('$O/b_${c}_$b.json').read().strip().splitlines()[-1]);print(d['value'],d.get('end_to_end_ms_per_frame'))")"
done; done
