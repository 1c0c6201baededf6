# A/B of the shadow-grid guard planes (DT_SG_GUARD=0 vs default) on C3, C2, C4
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r02j}; mkdir -p $O
for cfg in c3 c2 c4; do
  st=10; [ $cfg = c4 ] && st=2
  for gd in 0 1; do
    DT_SG_GUARD=$gd timeout -k 10 300 python bench.py --config $cfg --steps $st --warmup 1 --no-cpu-baseline > $O/ab_${cfg}_g$gd.json 2>/dev/null
    python -c "import json;d=json.loads(open('$O/ab_${cfg}_g$gd.json').read().splitlines()[-1]);print('$cfg guard=$gd',d['value'],d['roofline']['kernel_ms'])"
  done
done
echo all done
