# round-5 GPU check l: block subtrees actually compiled into the mesh builds (the #if read the
# DT_SHAPE_TRIANGLE enum as 0 before): GPU suite (subtree identity/parity tests now exercise them),
# stamps gates, C4 A/B over block shapes
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05l}; mkdir -p $O
V=distraytracer_amd/variants
export DT_PARITY_LOG=$O/parity.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
echo tests ok
for cfg in "84m1:8x4:1" "444m2:4x4x4:2"; do
  n=${cfg%%:*}; r=${cfg#*:}; blk=${r%%:*}; m=${r#*:}
  DT_SG_SUBTREE=1 DT_SG_SUB_BLOCK=$blk DT_SG_SUB_MULTI=$m DT_LIB=$V/libdt_stamps.so timeout -k 10 300 python tools/stamps.py c4 > $O/stamps_c4_$n.log 2>&1 || echo "stamps $n failed"
done
echo stamps done
for rep in 1 2; do
  for cfg in "base:" "84m1:DT_SG_SUBTREE=1" "444m2:DT_SG_SUBTREE=1 DT_SG_SUB_BLOCK=4x4x4 DT_SG_SUB_MULTI=2" "884m4:DT_SG_SUBTREE=1 DT_SG_SUB_BLOCK=8x8x4 DT_SG_SUB_MULTI=4" "222m4:DT_SG_SUBTREE=1 DT_SG_SUB_BLOCK=2x2x2 DT_SG_SUB_MULTI=4" "442m8:DT_SG_SUBTREE=1 DT_SG_SUB_BLOCK=4x4x2 DT_SG_SUB_MULTI=8"; do
    n=${cfg%%:*}; e=${cfg#*:}
    env $e timeout -k 10 200 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/c4_${n}_$rep.json 2>/dev/null
    python -c "import json;d=json.loads(open('$O/c4_${n}_$rep.json').read().splitlines()[-1]);print('$n $rep',d['value'],d['roofline']['kernel_ms'])" >> $O/c4_ab.txt
  done
done
echo all done
