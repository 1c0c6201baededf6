set -e
O=gpurun_out/r02bh; mkdir -p $O
DT_LIB=distraytracer_amd/variants/libdt_stamps.so timeout -k 10 300 python tools/stamps.py c3 1088 960x540 > $O/stamps_f1088.log 2>&1
echo done
