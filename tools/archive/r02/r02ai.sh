set -e
O=gpurun_out/r02ai; mkdir -p $O
OUT=$O DT_TILE_ORDER=0 DT_LIB=distraytracer_amd/variants/libdt_itimes.so timeout -k 10 200 python tools/item_times.py c3 > $O/item_times_c3.log 2>&1
echo done
