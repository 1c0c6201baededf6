# round-5 GPU check c: block subtrees (DT_SG_SUBTREE) -- parity test, then C4 A/B (same box)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05c}; mkdir -p $O
export DT_PARITY_LOG=$O/parity.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_subtree.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/subtree_tests.log 2>&1 || { tail -30 $O/subtree_tests.log; exit 1; }
echo subtree tests ok
for rep in 1 2; do
  timeout -k 10 200 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/c4_base_$rep.json 2>/dev/null
  DT_SG_SUBTREE=1 timeout -k 10 200 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/c4_sub84_$rep.json 2>/dev/null
  DT_SG_SUBTREE=1 DT_SG_SUB_BLOCK=4x2 timeout -k 10 200 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/c4_sub42_$rep.json 2>/dev/null
  DT_LIB=distraytracer_amd/variants/libdt_sub2.so DT_SG_SUBTREE=1 DT_SG_SUB_MULTI=4 timeout -k 10 200 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/c4_sub84m4_$rep.json 2>/dev/null
  DT_LIB=distraytracer_amd/variants/libdt_sub2.so DT_SG_SUBTREE=1 DT_SG_SUB_BLOCK=4x2 DT_SG_SUB_MULTI=4 timeout -k 10 200 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/c4_sub42m4_$rep.json 2>/dev/null
done
# bit identity of the multi-block walks against the product (tree walks)
VC_CASES=c4_1of256 timeout -k 10 200 python tools/variant_check.py $O/vc_base.npz > $O/vc_base.log 2>&1
DT_LIB=distraytracer_amd/variants/libdt_sub2.so DT_SG_SUBTREE=1 DT_SG_SUB_MULTI=4 VC_CASES=c4_1of256 timeout -k 10 200 python tools/variant_check.py $O/vc_m4.npz > $O/vc_m4.log 2>&1
python tools/variant_check.py --compare $O/vc_base.npz $O/vc_m4.npz > $O/vc_compare.log 2>&1 || true
for f in $O/c4_*.json; do python -c "import json,sys;d=json.loads(open('$f').read().splitlines()[-1]);print('$f',d['value'],d['roofline']['kernel_ms'])"; done > $O/c4_ab.txt
echo c4 ab done
