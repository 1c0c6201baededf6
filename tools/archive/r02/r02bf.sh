set -e
O=gpurun_out/r02bf; mkdir -p $O
DT_LIB=distraytracer_amd/variants/libdt_stamps.so timeout -k 10 200 python tools/stamps.py c3 960 960x540 > $O/stamps_f960.log 2>&1
DT_LIB=distraytracer_amd/variants/libdt_stamps.so timeout -k 10 200 python tools/stamps.py c3 1680 960x540 > $O/stamps_f1680.log 2>&1
echo done
