R=${GRAFT_REPO_ROOT:-$(pwd)}
for so in "$R"/distraytracer_amd/variants/*.so; do n=$(basename "$so" .so); echo -n "$n "; DT_LIB="$so" timeout -k 10 120 python "$R/tools/sky_bench.py" 2>/dev/null || exit 1; done
