# round 6 (x): GPU suite after start-side culling and umbra lanes; C5 every 10th frame against HEAD~2's library
set -e
O=gpurun_out/r06x; rm -rf $O; mkdir -p $O
export DT_PARITY_LOG=$O/parity.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
a() { n=$1; shift; env "$@" timeout -k 10 300 python tools/animate.py --frames 0:300:10 --per-frame > $O/c5_$n.json 2> $O/c5_$n.log; python -c "import json;d=json.loads(open('$O/c5_$n.json').read().splitlines()[-1]);print('c5 0:300:10 $n',d['seconds'],d['abort_counters'])"; }
a base DT_LIB=distraytracer_amd/variants/libdt_base.so
a new A=1
a base2 DT_LIB=distraytracer_amd/variants/libdt_base.so
a new2 A=1
