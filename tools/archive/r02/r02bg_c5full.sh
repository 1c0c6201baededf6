# C5 in full: all 300 frames of buildFinal(n*8) at 3840x2160, 64 spp, depth 10, on one GPU
set -e
O=gpurun_out/${TAG:-r02bg}; mkdir -p $O
timeout -k 10 900 python tools/animate.py --frames 0:300:1 --per-frame > $O/c5_full.log 2>&1
echo done
