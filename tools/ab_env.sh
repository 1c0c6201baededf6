# A/B of environment settings on this tree's libdt.so, interleaved on one box:
#   bash tools/ab_env.sh NAME "VAR=value ..." NAME2 "..." ...   (NAME base with "A=1" = defaults)
# on $CFGS (default c3 c2), $REPS repetitions (default 2). Prints "name_cfg_rep Mpixel-samples/s kernel-ms".
set -e
O=gpurun_out/${TAG:-abenv}; mkdir -p $O
args=("$@")
for rep in $(seq 1 ${REPS:-2}); do
for cfg in ${CFGS:-c3 c2}; do
st=10; [ $cfg = c4 ] && st=2
i=0
while [ $i -lt ${#args[@]} ]; do
  n=${args[$i]}; e=${args[$((i+1))]}; i=$((i+2))
  env $e timeout -k 10 300 python bench.py --config $cfg --steps $st --warmup 1 --no-cpu-baseline --no-roofline > $O/${n}_${cfg}_$rep.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/${n}_${cfg}_$rep.json').read().splitlines()[-1]);print('${n}_${cfg}_$rep',d['value'],d['roofline']['kernel_ms'] if 'kernel_ms' in d['roofline'] else d['ms_per_step'])"
done
done
done
