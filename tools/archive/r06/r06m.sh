# round 6 (m): stamps (shadow cycles by path) for C3, C4, C2 and the C5 transition frame 1088
set -e
O=gpurun_out/r06m; rm -rf $O; mkdir -p $O
export DT_LIB=distraytracer_amd/variants/libdt_stamps.so
timeout -k 10 300 python tools/stamps.py c3 > $O/stamps_c3.log 2>&1
timeout -k 10 300 python tools/stamps.py c4 > $O/stamps_c4.log 2>&1
timeout -k 10 300 python tools/stamps.py c3 1088 960x540 > $O/stamps_c5_1088.log 2>&1
timeout -k 10 300 python tools/stamps.py c3 1920 960x540 > $O/stamps_c5_1920.log 2>&1
grep -h "kernel ms\|by path\|occluded \|union walks" $O/*.log
