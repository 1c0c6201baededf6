# C4 A/B: shadow-grid list cap, fast tree for shadow walks, mixed union+walk waves
O=gpurun_out/r02z; mkdir -p $O
run() { n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > $O/c4_$n.json 2>/dev/null || { echo "$n failed"; exit 1; }
  python -c "import json; d=json.loads(open('$O/c4_$n.json').read().strip().split(chr(10))[-1]); print('$n', d['value'], d['roofline']['kernel_ms'])"; }
run base A=1
run ml96 DT_SG_MAX_LIST=96
run ml192 DT_SG_MAX_LIST=192
run ml512 DT_SG_MAX_LIST=512
run ft1 DT_FAST_TREE=1
run mixed DT_LIB=distraytracer_amd/variants/libdt_mixed.so
run mixed_ml192 DT_LIB=distraytracer_amd/variants/libdt_mixed.so DT_SG_MAX_LIST=192
