# C4 (OBJ meshes) A/B of the shadow-walk options: tree choice and the shadow-grid leaf cap
O=gpurun_out/r01o; mkdir -p $O
run() { echo "== $1"; env $2 DT_SG_VERBOSE=1 DT_TIMING=1 timeout -k 10 200 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > $O/$1.json 2> $O/$1.err || return 1
  grep -h "shadow grid:\|stage\|ms" $O/$1.err | head -20
  python -c "import json;d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]);print('value',d['value'],'ms',d['ms_per_step'],'e2e',d.get('end_to_end_ms_per_frame'))"; }
run base "" && run ft1 "DT_FAST_TREE=1" && run ft0 "DT_FAST_TREE=0" && run sg64k "DT_SG_MAX_LEAVES=65536" && run sg64k_ft1 "DT_SG_MAX_LEAVES=65536 DT_FAST_TREE=1"
