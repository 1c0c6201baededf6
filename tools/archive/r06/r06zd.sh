# round 6 (zd): C4 (and C3) with longer shadow-grid list caps (DT_SG_MAX_LIST)
set -e
O=gpurun_out/r06zd; rm -rf $O; mkdir -p $O
b() { n=$1; c=$2; shift 2; st=10; [ $c = c4 ] && st=4; env "$@" timeout -k 10 300 python bench.py --config $c --steps $st --warmup 1 --no-cpu-baseline --no-roofline > $O/$n.json 2>/dev/null; python -c "import json;d=json.loads(open('$O/$n.json').read().splitlines()[-1]);print('$n $*',d['value'],d['ms_per_step'])"; }
for rep in 1 2; do
b c4_96_$rep c4 A=1
b c4_160_$rep c4 DT_SG_MAX_LIST=160
b c4_256_$rep c4 DT_SG_MAX_LIST=256
b c4_512_$rep c4 DT_SG_MAX_LIST=512
done
b c3_96 c3 A=1
b c3_160 c3 DT_SG_MAX_LIST=160
