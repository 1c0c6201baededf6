# round 6 (j): two frames in flight at N=1; C2 priority / work-sharing knobs
set -e
O=gpurun_out/r06j; rm -rf $O; mkdir -p $O
j() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2',d['value'],d['roofline']['kernel_ms'],d['ms_per_step'])"; }
b() { n=$1; c=$2; i=$3; shift 3; st=5; [ $c = c3 ] && st=10; [ $c = c2 ] && st=40; env "$@" timeout -k 10 300 python bench.py --config $c --steps $st --warmup 2 --inflight $i --no-cpu-baseline > $O/$n.json 2>/dev/null; j $O/$n.json "$n $*"; }
for rep in 1 2; do
for c in c2 c3 c4; do
b ${c}_i1_$rep $c 1 A=1
b ${c}_i2_$rep $c 2 A=1
done
b c2_p2_$rep c2 1 DT_PRIO_STEPS=2
b c2_p4_$rep c2 1 DT_PRIO_STEPS=4
b c2_p8_$rep c2 1 DT_PRIO_STEPS=8
b c2_dn_$rep c2 1 DT_DONATE=1
b c2_i2p4_$rep c2 2 DT_PRIO_STEPS=4
done
