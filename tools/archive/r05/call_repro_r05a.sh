set -o pipefail
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 300 python -u tools/variant_check.py $O/base.npz > $O/base.log 2>&1 &&
DT_LIB=distraytracer_amd/variants/libdt_skycall1.so timeout -k 10 300 python -u tools/variant_check.py $O/sc1.npz > $O/sc1.log 2>&1 &&
DT_LIB=distraytracer_amd/variants/libdt_skycall2.so timeout -k 10 300 python -u tools/variant_check.py $O/sc2.npz > $O/sc2.log 2>&1 &&
DT_LIB=distraytracer_amd/variants/libdt_skycall1_nocg.so timeout -k 10 300 python -u tools/variant_check.py $O/sc1n.npz > $O/sc1n.log 2>&1 &&
DT_LIB=distraytracer_amd/variants/libdt_skycall1_noipra.so timeout -k 10 300 python -u tools/variant_check.py $O/sc1i.npz > $O/sc1i.log 2>&1
rc=$?
for v in sc1 sc2 sc1n sc1i; do echo "== $v"; python tools/variant_check.py --compare $O/base.npz $O/$v.npz; done > $O/compare.log 2>&1
exit $rc
