# round-5 GPU check h: shadow-grid block subtrees with 3-D blocks (XxYxZ cells): engagement (stamps),
# bit identity against the tree walks, C4 A/B over block sizes and the multi-block count
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05h}; mkdir -p $O
V=distraytracer_amd/variants

VC_CASES=c4_1of256 timeout -k 10 200 python tools/variant_check.py $O/vc_base.npz > $O/vc_base.log 2>&1
for cfg in "444m2:4x4x4:2" "884m4:8x8x4:4" "222m4:2x2x2:4"; do
  n=${cfg%%:*}; r=${cfg#*:}; blk=${r%%:*}; m=${r#*:}
  DT_SG_SUBTREE=1 DT_SG_SUB_BLOCK=$blk DT_SG_SUB_MULTI=$m VC_CASES=c4_1of256 timeout -k 10 200 python tools/variant_check.py $O/vc_$n.npz > $O/vc_$n.log 2>&1
  echo "== $n" >> $O/vc_compare.log; python tools/variant_check.py --compare $O/vc_base.npz $O/vc_$n.npz >> $O/vc_compare.log 2>&1 || true
done
echo identity done
for cfg in "444m2:4x4x4:2" "884m4:8x8x4:4"; do
  n=${cfg%%:*}; r=${cfg#*:}; blk=${r%%:*}; m=${r#*:}
  DT_SG_SUBTREE=1 DT_SG_SUB_BLOCK=$blk DT_SG_SUB_MULTI=$m DT_LIB=$V/libdt_stamps.so timeout -k 10 300 python tools/stamps.py c4 > $O/stamps_c4_$n.log 2>&1 || echo "stamps $n failed"
done
DT_LIB=$V/libdt_stamps.so timeout -k 10 300 python tools/stamps.py c3 1088 960x540 > $O/stamps_c5_1088.log 2>&1 || echo "stamps c5 failed"
echo stamps done
for rep in 1 2; do
  for cfg in "base:" "444m1:DT_SG_SUBTREE=1 DT_SG_SUB_BLOCK=4x4x4" "444m2:DT_SG_SUBTREE=1 DT_SG_SUB_BLOCK=4x4x4 DT_SG_SUB_MULTI=2" "884m4:DT_SG_SUBTREE=1 DT_SG_SUB_BLOCK=8x8x4 DT_SG_SUB_MULTI=4" "222m4:DT_SG_SUBTREE=1 DT_SG_SUB_BLOCK=2x2x2 DT_SG_SUB_MULTI=4" "888m2:DT_SG_SUBTREE=1 DT_SG_SUB_BLOCK=8x8x8 DT_SG_SUB_MULTI=2"; do
    n=${cfg%%:*}; e=${cfg#*:}
    env $e timeout -k 10 200 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $O/c4_${n}_$rep.json 2>/dev/null
    python -c "import json;d=json.loads(open('$O/c4_${n}_$rep.json').read().splitlines()[-1]);print('$n $rep',d['value'],d['roofline']['kernel_ms'])" >> $O/c4_ab.txt
  done
done
echo all done
