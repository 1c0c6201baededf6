# round-5 GPU check t: n copies of a frame in one launch (dt_render_repeat_async, ABI 7): GPU suite
# (incl. the copies' bit identity), the N=8 share per frame with 16 copies per launch against two
# frames in flight, C3 bench regression check
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05t}; mkdir -p $O
export DT_PARITY_LOG=$O/parity.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
echo tests ok
MULTI=16 WORLDS=1,2,4,8 timeout -k 10 400 python tools/rank_balance.py c3 3 > $O/rb_multi16.log 2>&1
WORLDS=1,2,4,8 INFLIGHT=2 timeout -k 10 300 python tools/rank_balance.py c3 3 > $O/rb_inflight2.log 2>&1
echo rb done
for rep in 1 2; do timeout -k 10 200 python bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-roofline > $O/c3_$rep.json 2>/dev/null; python -c "import json;d=json.loads(open('$O/c3_$rep.json').read().splitlines()[-1]);print('c3 $rep',d['value'],d['roofline']['kernel_ms'])" >> $O/ab.txt; done
echo all done
