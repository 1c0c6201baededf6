# A/B of primary-list hull culling and blur-pass lists: parity suite, then C3 / C4 bench and the
# tunnel frames (tools/frame_ab.py), each with DT_PL_HULL / DT_PL_BUMP off and on
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r02t}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
echo tests ok
for v in "DT_PL_HULL=0 DT_PL_BUMP=0" "DT_PL_HULL=1 DT_PL_BUMP=0" "DT_PL_HULL=1 DT_PL_BUMP=1"; do
  n=$(echo $v | tr -d "DT_PLHUBMP=" | tr " " "_")
  env $v timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 1 --no-cpu-baseline > $O/c3_$n.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/c3_$n.json').read().splitlines()[-1]);print('c3 $v',d['value'],d['roofline']['kernel_ms'],d.get('end_to_end_ms_per_frame'))"
  env $v timeout -k 10 300 python bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > $O/c4_$n.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/c4_$n.json').read().splitlines()[-1]);print('c4 $v',d['value'],d['roofline']['kernel_ms'],d.get('end_to_end_ms_per_frame'))"
  for f in 960 1200 1680 1920; do
    env $v timeout -k 10 200 python tools/frame_ab.py $f 1920x1080 64 "" > $O/f${f}_$n.json 2>/dev/null
    echo "f$f $v $(tail -1 $O/f${f}_$n.json | cut -c1-60)"
  done
done
echo all done
