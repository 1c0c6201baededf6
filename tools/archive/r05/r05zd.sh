# round 5: queue-order replay from measured item times (tools/order_sim.py, item-time build)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05zd}; mkdir -p $O
SAVE=$O/d DT_LIB=$R/distraytracer_amd/variants/libdt_itemrt.so timeout -k 10 400 python3 $R/tools/order_sim.py c3 1,8 > $O/order_sim_c3.log 2>&1
SAVE=$O/d DT_LIB=$R/distraytracer_amd/variants/libdt_itemrt.so timeout -k 10 300 python3 $R/tools/order_sim.py c2 1,8 > $O/order_sim_c2.log 2>&1
echo all done
