# round-5 GPU check k: the z table uploaded only when it changed (no copy kernel left between the frames
# of a still scene): GPU suite, C3 A/B against the old launch path, N=8 share with two frames in
# flight + its kernel trace; the C4 subtree gates (stamps)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05k}; mkdir -p $O
V=distraytracer_amd/variants
export DT_PARITY_LOG=$O/parity.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
echo tests ok
b() {   # name, lib ("" = product), config, steps
  local lib=""; [ -n "$2" ] && lib="DT_LIB=$V/libdt_$2.so"
  env $lib timeout -k 10 200 python bench.py --config $3 --steps $4 --warmup 1 --no-cpu-baseline --no-roofline > $O/$1.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/$1.json').read().splitlines()[-1]);print('$1',d['value'],d['roofline']['kernel_ms'])" >> $O/ab.txt
}
for rep in 1 2; do b c3_prod_$rep "" c3 10; b c3_bmm0_$rep bmm0 c3 10; done
echo ab done
WORLDS=1,2,4,8 INFLIGHT=2 timeout -k 10 300 python tools/rank_balance.py c3 3 > $O/rb_prod.log 2>&1
cd /tmp
WORLDS=8 INFLIGHT=2 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/ovl -o ovl --output-format csv -- python3 $R/tools/rank_balance.py c3 1 > $O/ovl_rank_balance.log 2>&1
cd $R
python tools/overlap.py $O/ovl > $O/overlap.txt 2>&1 || true
python tools/overlap.py $O/ovl __amd > $O/overlap_blits.txt 2>&1 || true
rm -rf $O/ovl
echo overlap done
DT_SG_SUBTREE=1 DT_SG_SUB_BLOCK=4x4x4 DT_SG_SUB_MULTI=2 DT_LIB=$V/libdt_stamps.so timeout -k 10 300 python tools/stamps.py c4 > $O/stamps_c4_444m2.log 2>&1 || echo "stamps failed"
echo all done
