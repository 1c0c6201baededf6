set -e
O=gpurun_out/r02bc; mkdir -p $O
DT_LIB=distraytracer_amd/variants/libdt_stamps.so timeout -k 10 200 python tools/stamps.py c3 1920 960x540 > $O/stamps_f1920.log 2>&1
echo done
