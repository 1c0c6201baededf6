# round-5 GPU check i: per-parity launch records uploaded only when changed and counters zeroed by the
# previous launch (no copy/fill kernels between the frames of a still scene): parity suite, identity,
# A/B against the old launch path (bmm0), the N=8 share time with two frames in flight
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05i}; mkdir -p $O
V=distraytracer_amd/variants
export DT_PARITY_LOG=$O/parity.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
echo tests ok
timeout -k 10 300 python -u tools/variant_check.py $O/prod.npz > $O/prod.log 2>&1
DT_LIB=$V/libdt_bmm0.so timeout -k 10 300 python -u tools/variant_check.py $O/bmm0.npz > $O/bmm0.log 2>&1
python tools/variant_check.py --compare $O/prod.npz $O/bmm0.npz > $O/compare.log 2>&1 || true
echo identity done
b() {   # name, lib ("" = product), config, steps
  local lib=""; [ -n "$2" ] && lib="DT_LIB=$V/libdt_$2.so"
  env $lib timeout -k 10 200 python bench.py --config $3 --steps $4 --warmup 1 --no-cpu-baseline --no-roofline > $O/$1.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/$1.json').read().splitlines()[-1]);print('$1',d['value'],d['roofline']['kernel_ms'])" >> $O/ab.txt
}
for rep in 1 2; do
  b c3_prod_$rep "" c3 10; b c3_bmm0_$rep bmm0 c3 10
  b c2_prod_$rep "" c2 10; b c2_bmm0_$rep bmm0 c2 10
done
echo ab done
WORLDS=1,8 INFLIGHT=2 timeout -k 10 300 python tools/rank_balance.py c3 3 > $O/rb_prod.log 2>&1
DT_LIB=$V/libdt_bmm0.so WORLDS=1,8 INFLIGHT=2 timeout -k 10 300 python tools/rank_balance.py c3 3 > $O/rb_bmm0.log 2>&1
echo rb done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline > $O/torchrun_n1.json 2> $O/torchrun_n1.err
echo all done
