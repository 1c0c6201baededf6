# round 6 (h): C2 profile (PMC passes, grid tail), C4 2x2 tiles at world 8
set -e
O=gpurun_out/r06h; rm -rf $O; mkdir -p $O
bash tools/profile_gpu.sh r06h_c2 c2 > $O/prof.log 2>&1
DT_LIB=distraytracer_amd/variants/libdt_itemrt.so timeout -k 10 300 python tools/tail.py c2 1 > $O/tail_c2.log 2>&1
DT_LIB=distraytracer_amd/variants/libdt_itemrt.so timeout -k 10 300 python tools/tail.py c3 1 > $O/tail_c3.log 2>&1
TILE=2 WORLDS=8 INFLIGHT=2 timeout -k 10 500 python tools/rank_balance.py c4 2 > $O/rb_c4_t2.log 2>&1
