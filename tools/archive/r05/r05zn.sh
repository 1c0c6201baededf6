# round 5: C4 queue-order replay (tools/order_sim.py on the item-time build), world 1 and the world-8 share (16x16 tiles)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05zn}; mkdir -p $O
DT_LIB=$R/distraytracer_amd/variants/libdt_itemrt.so timeout -k 10 600 python3 $R/tools/order_sim.py c4 1,8 > $O/order_sim_c4.log 2>&1
echo all done
