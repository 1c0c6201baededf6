# stamps profiles of C4 (960x540, 256 spp) and C3 (1920x1080)
set -e
O=gpurun_out/${TAG:-r02y}; mkdir -p $O
DT_LIB=distraytracer_amd/variants/libdt_stamps.so timeout -k 10 200 python tools/stamps.py c4 240 960x540 > $O/stamps_c4.log 2>&1
DT_LIB=distraytracer_amd/variants/libdt_stamps.so timeout -k 10 200 python tools/stamps.py c3 > $O/stamps_c3.log 2>&1
echo done
