# C4: shadow-grid resolution and list cap (env knobs), kernel time
O=gpurun_out/r02ao; mkdir -p $O
run() { n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > $O/c4_$n.json 2>/dev/null || { echo "$n failed"; exit 1; }
  python -c "import json; d=json.loads(open('$O/c4_$n.json').read().strip().split(chr(10))[-1]); print('$n', d['value'], d['roofline']['kernel_ms'], d.get('end_to_end_ms_per_frame'))"; }
run base A=1
run c64k DT_SG_CELLS=65536
run c128k DT_SG_CELLS=131072
run c256k DT_SG_CELLS=262144
run c128k_ml96 DT_SG_CELLS=131072 DT_SG_MAX_LIST=96
run c256k_ml96 DT_SG_CELLS=262144 DT_SG_MAX_LIST=96
run reach1 DT_SG_REACH=1
