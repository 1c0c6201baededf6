# round-5 GPU check d: the called-function reproducer over code-generation flags, the split block-subtree
# walks (parity, bit identity, C4 stamps and A/B)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05d}; mkdir -p $O
OUT=$O/call_repro.log bash tools/call_repro/run.sh
echo call repro done
export DT_PARITY_LOG=$O/parity.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_subtree.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/subtree_tests.log 2>&1 || { tail -30 $O/subtree_tests.log; exit 1; }
echo subtree tests ok
VC_CASES=c4_1of256 timeout -k 10 200 python tools/variant_check.py $O/vc_base.npz > $O/vc_base.log 2>&1
for m in 1 4; do
  DT_SG_SUBTREE=1 DT_SG_SUB_MULTI=$m VC_CASES=c4_1of256 timeout -k 10 200 python tools/variant_check.py $O/vc_m$m.npz > $O/vc_m$m.log 2>&1
  python tools/variant_check.py --compare $O/vc_base.npz $O/vc_m$m.npz > $O/vc_compare_m$m.log 2>&1 || true
done
DT_SG_SUBTREE=1 DT_LIB=distraytracer_amd/variants/libdt_stamps.so timeout -k 10 300 python tools/stamps.py c4 > $O/stamps_c4_sub.log 2>&1 || echo "stamps failed"
echo stamps done
for rep in 1 2; do
  for cfg in "base:" "m1:DT_SG_SUBTREE=1" "m2:DT_SG_SUBTREE=1 DT_SG_SUB_MULTI=2" "m4:DT_SG_SUBTREE=1 DT_SG_SUB_MULTI=4" "b42m4:DT_SG_SUBTREE=1 DT_SG_SUB_BLOCK=4x2 DT_SG_SUB_MULTI=4" "b168m2:DT_SG_SUBTREE=1 DT_SG_SUB_BLOCK=16x8 DT_SG_SUB_MULTI=2"; do
    n=${cfg%%:*}; e=${cfg#*:}
    env $e timeout -k 10 200 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/c4_${n}_$rep.json 2>/dev/null
    python -c "import json;d=json.loads(open('$O/c4_${n}_$rep.json').read().splitlines()[-1]);print('$n $rep',d['value'],d['roofline']['kernel_ms'])" >> $O/c4_ab.txt
  done
done
echo c4 ab done
