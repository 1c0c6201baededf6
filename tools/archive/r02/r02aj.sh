# wave priority (DT_PRIO_STEPS) x tile order: per-rank kernel times of the C3 tile split
set -e
O=gpurun_out/r02aj; mkdir -p $O
for v in p8 p0 p4 p16; do
  L=""; [ $v != p8 ] && L=distraytracer_amd/variants/libdt_$v.so
  DT_LIB=$L timeout -k 10 300 python tools/rank_balance.py c3 3 > $O/bal_${v}_order.log 2>&1
  DT_LIB=$L DT_TILE_ORDER=0 timeout -k 10 300 python tools/rank_balance.py c3 3 > $O/bal_${v}_noorder.log 2>&1
done
echo done
