# light-sample cache from the first area light (variant lsord) vs default: parity (C2/C3/C4 windows) + A/B
set -e
O=gpurun_out/r02br; mkdir -p $O
DT_LIB=distraytracer_amd/variants/libdt_lsord.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "c2 or c3 or models or tunnel" -x -v --timeout 300 --timeout-method thread > $O/gpu_tests_lsord.log 2>&1 || { tail -30 $O/gpu_tests_lsord.log; exit 1; }
echo tests ok
TAG=r02br VAR=lsord bash tools/ab_lib.sh > $O/ab.log 2>&1
echo done
