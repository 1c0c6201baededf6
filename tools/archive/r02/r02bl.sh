# knob sweep around the new defaults on C3, C2, C4 (bench) and C5 frame 1088 (960x540)
O=gpurun_out/r02bl; mkdir -p $O
run() { n=$1; shift
  for c in c3 c2; do env "$@" timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > $O/${c}_$n.json 2>/dev/null; python -c "import json;d=json.loads(open('$O/${c}_$n.json').read().splitlines()[-1]);print('$n $c',d['value'],d['roofline']['kernel_ms'],d.get('end_to_end_ms_per_frame'))"; done
  env "$@" timeout -k 10 300 python bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > $O/c4_$n.json 2>/dev/null; python -c "import json;d=json.loads(open('$O/c4_$n.json').read().splitlines()[-1]);print('$n c4',d['value'],d['roofline']['kernel_ms'],d.get('end_to_end_ms_per_frame'))"
  env "$@" timeout -k 10 200 python3 tools/frame_ab.py 1088 960x540 64 "" 2>/dev/null | python -c "import sys,json;d=json.loads(sys.stdin.read().splitlines()[-1]);print('$n f1088',d['kernel_ms'])"
}
run base A=1
run r0125 DT_SG_REACH=0.125
run ml160 DT_SG_MAX_LIST=160
run pl4 DT_PL_BLOCK=4
run pl16 DT_PL_BLOCK=16
run sup4 DT_PL_SUPER=4
echo done
