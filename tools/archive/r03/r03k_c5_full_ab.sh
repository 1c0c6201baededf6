set -e
O=gpurun_out/r03k; mkdir -p $O
timeout -k 10 420 python tools/animate.py --frames 0:300:1 --donate auto --per-frame > $O/c5_full_auto.log 2>&1
echo auto done
timeout -k 10 420 python tools/animate.py --frames 0:300:1 --donate off --per-frame > $O/c5_full_off.log 2>&1
echo off done
TAG=r03k_env REPS=2 CFGS="c3 c2" bash tools/ab_env.sh base "A=1" sgorder "DT_SG_ORDER=1" > $O/ab_env.log 2>&1
echo env done
