# round-5 final: the rocprofv3 kernel trace + stats of the bench command itself (timed launches)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05za}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-roofline > $O/prof_bench.json 2> $O/prof_bench.err
echo all done
