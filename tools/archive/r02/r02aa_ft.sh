# DT_FAST_TREE=1 (fast tree for shadow walks too) vs default on C3, C2 and tunnel frames
O=gpurun_out/r02aa; mkdir -p $O
run() { n=$1; c=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > $O/${c}_$n.json 2>/dev/null || { echo "$n failed"; exit 1; }
  python -c "import json; d=json.loads(open('$O/${c}_$n.json').read().strip().split(chr(10))[-1]); print('$c $n', d['value'], d['roofline']['kernel_ms'])"; }
for i in 1 2; do
run base c3 A=1
run ft1 c3 DT_FAST_TREE=1
done
run base c2 A=1
run ft1 c2 DT_FAST_TREE=1
for f in 960 1680; do
  timeout -k 10 120 python3 tools/frame_ab.py $f 960x540 64 "" 2>/dev/null
  DT_FAST_TREE=1 timeout -k 10 120 python3 tools/frame_ab.py $f 960x540 64 "" 2>/dev/null
done
