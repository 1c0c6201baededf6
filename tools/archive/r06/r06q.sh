# round 6 (q): closest hit with shapes first in the tunnel builds — GPU suite, C5 blur frames A/B
set -e
O=gpurun_out/r06q; rm -rf $O; mkdir -p $O
export DT_PARITY_LOG=$O/parity.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
a() { n=$1; shift; env "$@" timeout -k 10 300 python tools/animate.py --frames 140:244:8 --per-frame > $O/c5_$n.json 2> $O/c5_$n.log; python -c "import json;d=json.loads(open('$O/c5_$n.json').read().splitlines()[-1]);print('c5 140:244:8 $n',d['seconds'],d['abort_counters'])"; }
a sfc0 DT_LIB=distraytracer_amd/variants/libdt_sfc0.so
a sfc1 A=1
a sfc0b DT_LIB=distraytracer_amd/variants/libdt_sfc0.so
a sfc1b A=1
