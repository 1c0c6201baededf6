set -e
O=gpurun_out/r01n; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
for c in c3 c2 c4; do for o in 0 1; do
  DT_SG_ORDER=$o timeout -k 10 200 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/b_${c}_$o.json 2>/dev/null
  echo "$c order=$o $(python -c "import json;d=json.loads(open('$O/b_${c}_$o.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d.get('end_to_end_ms_per_frame'))")"
done; done
for f in 2160 1200; do for o in 0 1; do
  echo -n "frame $f order=$o "; DT_SG_ORDER=$o timeout -k 10 200 python tools/frame_ab.py $f 1920x1080 64 "" 2>/dev/null | tail -1
done; done
