# round 6 (zq): shadow-grid cell count 131072 against the default 32768 on C3, C2, C4 and the C5
# every-10th-frame sample (with the round's shorter lists)
set -e
O=gpurun_out/r06zq; rm -rf $O; mkdir -p $O
j() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2',d['value'],d['roofline']['kernel_ms'],d['ms_per_step'])"; }
b() { n=$1; c=$2; shift 2; st=10; [ $c = c2 ] && st=40; [ $c = c4 ] && st=3; env "$@" timeout -k 10 300 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline > $O/$n.json 2>/dev/null; j $O/$n.json "$n $*"; }
for rep in 1 2; do
for c in c3 c2; do
b ${c}_base_$rep $c A=1
b ${c}_c128k_$rep $c DT_SG_CELLS=131072
done
done
b c4_base c4 A=1
b c4_c128k c4 DT_SG_CELLS=131072
a() { n=$1; shift; env "$@" timeout -k 10 300 python tools/animate.py --frames 0:300:10 --per-frame > $O/c5_$n.json 2> $O/c5_$n.log; python -c "import json;d=json.loads(open('$O/c5_$n.json').read().splitlines()[-1]);print('c5 0:300:10 $n',d['seconds'])"; }
a base A=1
a c128k DT_SG_CELLS=131072
echo all done
