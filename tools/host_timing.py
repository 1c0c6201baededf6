import sys, time, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
import distraytracer_amd as dt
torch.cuda.init()
for frame in (240, 960, 1200):
    for rep in range(2):
        t0 = time.perf_counter()
        g = dt.globals_default(); g.use_model = 0
        b = dt.build_scene("final", frame, g)
        t1 = time.perf_counter()
        s = dt.Scene(b, g)
        t2 = time.perf_counter()
        print("frame", frame, "build_scene %.1f ms  Scene %.1f ms" % ((t1 - t0) * 1e3, (t2 - t1) * 1e3), file=sys.stderr, flush=True)
        s.close()
