# A/B of shadow-grid umbra cells (DT_SG_UMBRA=0 vs default): parity suite, then C3 / C2 / C4
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r02p}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
echo tests ok
for cfg in c3 c2 c4; do
  st=10; [ $cfg = c4 ] && st=2
  for u in 0 1; do
    DT_SG_UMBRA=$u timeout -k 10 300 python bench.py --config $cfg --steps $st --warmup 1 --no-cpu-baseline > $O/${cfg}_u$u.json 2>/dev/null
    python -c "import json;d=json.loads(open('$O/${cfg}_u$u.json').read().splitlines()[-1]);print('$cfg umbra=$u',d['value'],d['roofline']['kernel_ms'],d.get('end_to_end_ms_per_frame'))"
  done
done
echo all done
