# transition frame 1088 (960x540, 64 spp): remaining knobs
O=gpurun_out/r02bp; mkdir -p $O
for kv in "base:A=1" "hull2:DT_SG_HULL=2" "umbra2:DT_SG_UMBRA=2" "eye0:DT_EYE_ORDER=0" "order1:DT_SG_ORDER=1" "bt0:DT_BUMP_TREE=0" "plb0:DT_PL_BUMP=0" "blk4x2:DT_SG_BLOCK=4x2"; do
  n=${kv%%:*}; e=${kv#*:}
  env $e timeout -k 10 200 python3 tools/frame_ab.py 1088 960x540 64 "" 2>/dev/null | sed "s/^/$n /" >> $O/knobs.log || { echo "$n failed"; exit 1; }
done
echo done
