# round 6 (zr): stamps of C3 of the final tree (second version of start-side culling, union on listing lanes, early umbra) (which shadow
# tests remain, by light and shape)
set -e
O=gpurun_out/r06zr; rm -rf $O; mkdir -p $O
export DT_LIB=distraytracer_amd/variants/libdt_stamps.so
timeout -k 10 300 python tools/stamps.py c3 > $O/stamps_c3.log 2>&1
cat $O/stamps_c3.log
