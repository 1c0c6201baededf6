# round 6 (zb): start-side culling on prism faces — bit identity (forced on every frame), C3/C2/C4 against HEAD
set -e
O=gpurun_out/r06zb; rm -rf $O; mkdir -p $O
timeout -k 10 600 python tools/sg_start_check.py > $O/sg_start_check.log 2>&1; cat $O/sg_start_check.log
j() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$2',d['value'],d['roofline']['kernel_ms'],d['ms_per_step'])"; }
b() { n=$1; c=$2; shift 2; st=10; [ $c = c2 ] && st=40; [ $c = c4 ] && st=4; env "$@" timeout -k 10 300 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline > $O/$n.json 2>/dev/null; j $O/$n.json "$n $*"; }
for rep in 1 2; do
for c in c3 c2 c4; do
b ${c}_base_$rep $c DT_LIB=distraytracer_amd/variants/libdt_base.so
b ${c}_new_$rep $c A=1
done
done
