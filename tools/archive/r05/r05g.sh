# round-5 GPU check g: the launch record in the kernel arguments and double-buffered counters (no
# blit kernels between frames), the axis-aligned plane shadow tests: parity suite, identity of the
# variants, A/B (C3, C2, C4), and the N=8 share time with two frames in flight against the old path
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05g}; mkdir -p $O
V=distraytracer_amd/variants
export DT_PARITY_LOG=$O/parity.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
echo tests ok
timeout -k 10 300 python -u tools/variant_check.py $O/prod.npz > $O/prod.log 2>&1
for v in ax0 aw0 bmm0; do
  DT_LIB=$V/libdt_$v.so timeout -k 10 300 python -u tools/variant_check.py $O/$v.npz > $O/$v.log 2>&1
  echo "== $v" >> $O/compare.log; python tools/variant_check.py --compare $O/prod.npz $O/$v.npz >> $O/compare.log 2>&1 || true
done
echo identity done
b() {   # name, lib ("" = product), config, steps
  local lib=""; [ -n "$2" ] && lib="DT_LIB=$V/libdt_$2.so"
  env $lib timeout -k 10 200 python bench.py --config $3 --steps $4 --warmup 1 --no-cpu-baseline --no-roofline > $O/$1.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/$1.json').read().splitlines()[-1]);print('$1',d['value'],d['roofline']['kernel_ms'])" >> $O/ab.txt
}
for rep in 1 2; do
  b c3_prod_$rep "" c3 10; b c3_ax0_$rep ax0 c3 10; b c3_aw0_$rep aw0 c3 10; b c3_bmm0_$rep bmm0 c3 10
  b c2_prod_$rep "" c2 10; b c2_ax0_$rep ax0 c2 10
  b c4_prod_$rep "" c4 2; b c4_ax0_$rep ax0 c4 2
done
echo ab done
WORLDS=1,8 INFLIGHT=2 timeout -k 10 300 python tools/rank_balance.py c3 3 > $O/rb_prod.log 2>&1
DT_LIB=$V/libdt_bmm0.so WORLDS=1,8 INFLIGHT=2 timeout -k 10 300 python tools/rank_balance.py c3 3 > $O/rb_bmm0.log 2>&1
echo all done
