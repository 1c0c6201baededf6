# reach 0.25 / list cap 96 / 128k cells on C3, C2, C4 (bench) and C5 frames 1088, 1200, 1920 (960x540)
O=gpurun_out/r02bj; mkdir -p $O
run() { n=$1; shift
  for c in c3 c2; do env "$@" timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > $O/${c}_$n.json 2>/dev/null; python -c "import json;d=json.loads(open('$O/${c}_$n.json').read().splitlines()[-1]);print('$n $c',d['value'],d['roofline']['kernel_ms'],d.get('end_to_end_ms_per_frame'))"; done
  env "$@" timeout -k 10 300 python bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > $O/c4_$n.json 2>/dev/null; python -c "import json;d=json.loads(open('$O/c4_$n.json').read().splitlines()[-1]);print('$n c4',d['value'],d['roofline']['kernel_ms'],d.get('end_to_end_ms_per_frame'))"
  for f in 1088 1200 1920; do env "$@" timeout -k 10 200 python3 tools/frame_ab.py $f 960x540 64 "" 2>/dev/null | python -c "import sys,json;d=json.loads(sys.stdin.read().splitlines()[-1]);print('$n f$f',d['kernel_ms'])"; done
}
run base A=1
run r025 DT_SG_REACH=0.25
run ml96 DT_SG_MAX_LIST=96
run both DT_SG_REACH=0.25 DT_SG_MAX_LIST=96
run all3 DT_SG_REACH=0.25 DT_SG_MAX_LIST=96 DT_SG_CELLS=131072
echo done
