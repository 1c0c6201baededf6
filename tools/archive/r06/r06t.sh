# round 6 (t): upper bound of dropping the room walls from the shadow lists of lights 1-4 (not exact: measurement only)
set -e
O=gpurun_out/r06t; rm -rf $O; mkdir -p $O
j() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2',d['value'],d['roofline']['kernel_ms'],d['ms_per_step'],d.get('parity'))"; }
b() { n=$1; c=$2; shift 2; st=10; env "$@" timeout -k 10 300 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline > $O/$n.json 2>/dev/null; j $O/$n.json "$n $*"; }
for rep in 1 2; do
b c3_base_$rep c3 A=1
b c3_walls_$rep c3 DT_SG_EXP_DROP=33,34,35
b c3_wallsceil_$rep c3 DT_SG_EXP_DROP=33,34,35,40
done
