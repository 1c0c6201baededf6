# round 6 re-entry check of HEAD (hull culling + 81-spp device-path test landed after r06fb):
# GPU suite with the parity log, smoke, default bench line, C2/C4 lines, rocprofv3 kernel trace +
# PMC passes of C3 (tools/profile_gpu.sh), C5 over all 300 frames
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06zg; rm -rf $O; mkdir -p $O
cd $R
export DT_PARITY_LOG=$O/parity.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
tail -1 $O/bench.json | cut -c1-200
timeout -k 10 300 python bench.py --config c2 --steps 40 --warmup 2 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err
tail -1 $O/bench_c2.json | cut -c1-200
timeout -k 10 300 python bench.py --config c4 --steps 4 --warmup 1 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err
tail -1 $O/bench_c4.json | cut -c1-200
bash tools/profile_gpu.sh r06zg c3 > $O/profile.log 2>&1
tail -2 $O/profile.log
timeout -k 10 400 python tools/animate.py --frames 0:300:1 --per-frame > $O/c5_full.json 2> $O/c5_full_frames.log
tail -1 $O/c5_full.json | cut -c1-300
echo all done
