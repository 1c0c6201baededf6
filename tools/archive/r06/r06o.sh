# round 6 (o): deep-cascade priority at N=1 (two frames in flight), C2/C3/C4
set -e
O=gpurun_out/r06o; rm -rf $O; mkdir -p $O
j() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2',d['value'],d['roofline']['kernel_ms'],d['ms_per_step'])"; }
b() { n=$1; c=$2; shift 2; st=5; [ $c = c3 ] && st=10; [ $c = c2 ] && st=60; env "$@" timeout -k 10 300 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline > $O/$n.json 2>/dev/null; j $O/$n.json "$n $*"; }
for rep in 1 2; do
for c in c2 c3 c4; do
b ${c}_p0_$rep $c DT_PRIO_STEPS=0
b ${c}_p2_$rep $c DT_PRIO_STEPS=2
b ${c}_p4_$rep $c DT_PRIO_STEPS=4
done
done
