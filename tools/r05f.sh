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
echo all done
