# round 6 (ze): C4 with shorter shadow-grid list caps and other reaches
set -e
O=gpurun_out/r06ze; rm -rf $O; mkdir -p $O
b() { n=$1; c=$2; shift 2; st=10; [ $c = c4 ] && st=4; env "$@" timeout -k 10 300 python bench.py --config $c --steps $st --warmup 1 --no-cpu-baseline --no-roofline > $O/$n.json 2>/dev/null; python -c "import json;d=json.loads(open('$O/$n.json').read().splitlines()[-1]);print('$n $*',d['value'],d['ms_per_step'])"; }
for rep in 1 2; do
b c4_96_$rep c4 A=1
b c4_64_$rep c4 DT_SG_MAX_LIST=64
b c4_48_$rep c4 DT_SG_MAX_LIST=48
b c4_r15_$rep c4 DT_SG_REACH=0.15
b c4_r40_$rep c4 DT_SG_REACH=0.4
done
