# round 6 end (b): the default bench line (10 steps), rocprofv3 kernel trace + PMC passes of C3
# (tools/profile_gpu.sh), C5 over all 300 frames
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06fb; rm -rf $O; mkdir -p $O
cd $R
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
tail -1 $O/bench.json | cut -c1-200
bash tools/profile_gpu.sh r06fb c3 > $O/profile.log 2>&1
tail -2 $O/profile.log
timeout -k 10 400 python tools/animate.py --frames 0:300:1 --per-frame > $O/c5_full.json 2> $O/c5_full_frames.log
tail -1 $O/c5_full.json
echo all done
