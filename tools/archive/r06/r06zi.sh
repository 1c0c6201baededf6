# round 6 (zi): stamps of C3 after start-side culling against the box of ray origins (which shadow
# tests remain, by light and shape)
set -e
O=gpurun_out/r06zi; rm -rf $O; mkdir -p $O
export DT_LIB=distraytracer_amd/variants/libdt_stamps.so
timeout -k 10 300 python tools/stamps.py c3 > $O/stamps_c3.log 2>&1
cat $O/stamps_c3.log
