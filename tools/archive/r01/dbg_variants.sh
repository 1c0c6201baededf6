for v in nocull general; do echo "== $v"; DT_LIB=distraytracer_amd/variants/libdt_$v.so timeout -k 10 300 python tools/debug_c5.py 2>&1 | grep -v amdgpu.ids | head -12; done
