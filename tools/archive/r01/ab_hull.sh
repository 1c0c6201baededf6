# A/B of shadow-grid hull culling (DT_SG_HULL = 0 off, 1 blocks only, 2 blocks + cells): parity
# suite with the default, then C3 / C4 bench lines and tunnel frames (tools/frame_ab.py)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r02n}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
echo tests ok
for m in ${MODES:-0 1 2}; do
  DT_SG_HULL=$m timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 1 --no-cpu-baseline > $O/c3_h$m.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/c3_h$m.json').read().splitlines()[-1]);print('c3 hull=$m',d['value'],d['roofline']['kernel_ms'],d.get('end_to_end_ms_per_frame'))"
  DT_SG_HULL=$m timeout -k 10 300 python bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > $O/c4_h$m.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/c4_h$m.json').read().splitlines()[-1]);print('c4 hull=$m',d['value'],d['roofline']['kernel_ms'],d.get('end_to_end_ms_per_frame'))"
  for f in 960 1200 1680 1920; do
    DT_SG_HULL=$m timeout -k 10 200 python tools/frame_ab.py $f 1920x1080 64 "" > $O/f${f}_h$m.json 2>/dev/null
    echo "f$f hull=$m $(tail -1 $O/f${f}_h$m.json)"
  done
done
echo all done
