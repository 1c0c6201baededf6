"""Host time of dt.render_async per call for the plain (image layout, 32x32 tiles) and the
tile-split (FrameSplit at world 1, 8x8 tiles, slab layout) C3 render, and the wall time per frame of
six back-to-back renders: is the split path's per-frame overhead host work?

    python tools/host_time_probe.py        (on the GPU box)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import time, torch, distraytracer_amd as dt
from distraytracer_amd.multigpu import FrameSplit
import bench
g, built = bench.build_globals(dt, "c3")
dev = torch.device("cuda", 0)
scene = dt.Scene(built, g)
img = torch.zeros(3 * g.xRes * g.yRes, dtype=torch.float32, device=dev)
s = torch.cuda.current_stream(dev).cuda_stream
cases = [("plain", img, dt.tiles())]
for side in (8, 16, 32):   # FrameSplit's tile side (default 8)
    split = FrameSplit(g, 1, 0, tile_w=side, tile_h=side)
    cases.append(("split %dx%d" % (side, side), torch.zeros(split.slab_floats, dtype=torch.float32, device=dev),
                  split.tile))
for name, out, tile in cases:
    dt.render(scene, g, 240, out, tile); torch.cuda.synchronize()
    ts = []
    t0 = time.perf_counter()
    for k in range(6):
        a = time.perf_counter(); dt.render_async(scene, g, 240, out, tile, stream=s); ts.append((time.perf_counter() - a) * 1e3)
    torch.cuda.synchronize()
    print(name, "host ms per render_async", [round(x, 2) for x in ts], "wall ms per frame", round((time.perf_counter() - t0) * 1e3 / 6, 2), flush=True)
