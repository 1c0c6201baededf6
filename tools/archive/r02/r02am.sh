set -e
O=gpurun_out/r02am; mkdir -p $O
timeout -k 10 100 python tools/skymiss_debug.py > $O/defer.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "cloud or sky" -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -5 $O/tests.log; exit 1; }
echo done
