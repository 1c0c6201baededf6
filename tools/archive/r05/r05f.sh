# round-5 GPU check f: the product without -disable-machine-cse, with the called sky march in the
# tunnel/blur builds: parity suite, smoke, C3 bench, rocprof kernel stats; then the N=8 share
# diagnostics: the grid's ramp/tail per launch (item start/end times) and whether two frames in flight
# overlap their dispatches (kernel trace of rank_balance at world 8)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05f}; mkdir -p $O
export DT_PARITY_LOG=$O/parity.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
echo tests ok
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
echo smoke ok
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
echo bench ok
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err
echo prof ok
cd $R
DT_LIB=distraytracer_amd/variants/libdt_itemrt.so timeout -k 10 200 python tools/tail.py c3 1,2,8 > $O/tail_c3.log 2>&1
echo tail ok
cd /tmp
WORLDS=8 INFLIGHT=2 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/ovl -o ovl --output-format csv -- python3 $R/tools/rank_balance.py c3 1 > $O/ovl_rank_balance.log 2>&1
cd $R
python tools/overlap.py $O/ovl > $O/overlap.txt 2>&1 || true

DT_SG_SUBTREE=1 DT_LIB=distraytracer_amd/variants/libdt_stamps.so timeout -k 10 300 python tools/stamps.py c4 > $O/stamps_c4_sub.log 2>&1 || echo "stamps c4 failed"
echo stamps done
V=distraytracer_amd/variants
b() {   # name, lib ("" = product), config, steps
  local lib=""; [ -n "$2" ] && lib="DT_LIB=$V/libdt_$2.so"
  env $lib timeout -k 10 200 python bench.py --config $3 --steps $4 --warmup 1 --no-cpu-baseline --no-roofline > $O/$1.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/$1.json').read().splitlines()[-1]);print('$1',d['value'],d['roofline']['kernel_ms'])" >> $O/ab.txt
}
for rep in 1 2; do
  b c3_bmm0_$rep bmm0 c3 10; b c3_prod_$rep "" c3 10
  b c2_bmm0_$rep bmm0 c2 10; b c2_prod_$rep "" c2 10
  b c4_bmm0_$rep bmm0 c4 2; b c4_prod_$rep "" c4 2
done
echo all done
