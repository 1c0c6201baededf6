# round 6 final check (zo): GPU suite with the parity log, smoke, the default bench line, C2/C4
# lines, torchrun at world 1, rocprofv3 kernel trace + PMC passes of C3 (tools/profile_gpu.sh),
# C5 over all 300 frames, C2 A/B of the 4-wave build against the previous library, kernel-side rank
# balance of C3 and C4 at N = 1, 2, 4, 8
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06zo; rm -rf $O; mkdir -p $O
cd $R
export DT_PARITY_LOG=$O/parity.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
unset DT_PARITY_LOG
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
tail -1 $O/bench.json | cut -c1-200
timeout -k 10 300 python bench.py --config c2 --steps 40 --warmup 2 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err
tail -1 $O/bench_c2.json | cut -c1-200
timeout -k 10 300 python bench.py --config c4 --steps 4 --warmup 1 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err
tail -1 $O/bench_c4.json | cut -c1-200
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline > $O/torchrun_n1.json 2> $O/torchrun_n1.err
tail -1 $O/torchrun_n1.json | cut -c1-200
bash tools/profile_gpu.sh r06zo c3 > $O/profile.log 2>&1
tail -1 $O/profile.log
timeout -k 10 400 python tools/animate.py --frames 0:300:1 --per-frame > $O/c5_full.json 2> $O/c5_full_frames.log
tail -1 $O/c5_full.json | cut -c1-300
bash tools/archive/r06/r06zn.sh > $O/ab_c2.txt 2>&1; grep "^c[23]" $O/ab_c2.txt
INFLIGHT=2 WORLDS=1,2,4,8 timeout -k 10 500 python tools/rank_balance.py c3 2 > $O/rank_balance_c3.log 2>&1
grep -o '"world": [0-9]*\|"max_ms": [0-9.]*\|"kernel_efficiency": [0-9.]*' $O/rank_balance_c3.log | paste -sd' '
INFLIGHT=2 WORLDS=1,2,4,8 timeout -k 10 600 python tools/rank_balance.py c4 2 > $O/rank_balance_c4.log 2>&1
grep -o '"world": [0-9]*\|"max_ms": [0-9.]*\|"kernel_efficiency": [0-9.]*' $O/rank_balance_c4.log | paste -sd' '
echo all done
