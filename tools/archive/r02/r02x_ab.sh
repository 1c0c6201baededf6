set -e
mkdir -p gpurun_out/r02x
for f in 1920 1680 1200; do
  timeout -k 10 120 python3 tools/frame_ab.py $f 960x540 64 "" >> gpurun_out/r02x/ab.log 2>&1
  DT_BUMP_TREE=0 timeout -k 10 120 python3 tools/frame_ab.py $f 960x540 64 "" >> gpurun_out/r02x/ab.log 2>&1
done
