# transition frame 1088 (960x540, 64 spp): shadow-grid and tree knobs
O=gpurun_out/r02bi; mkdir -p $O
for kv in "base:A=1" "ml96:DT_SG_MAX_LIST=96" "ml192:DT_SG_MAX_LIST=192" "c64k:DT_SG_CELLS=65536" "c128k:DT_SG_CELLS=131072" "reach1:DT_SG_REACH=1" "reach025:DT_SG_REACH=0.25" "ftc:DT_FAST_TREE=c" "nogrid:DT_SHADOW_GRID=0"; do
  n=${kv%%:*}; e=${kv#*:}
  env $e timeout -k 10 200 python3 tools/frame_ab.py 1088 960x540 64 "" 2>/dev/null | sed "s/^/$n /" >> $O/knobs.log || { echo "$n failed"; exit 1; }
done
echo done
