"""Bit-identity check of an A/B kernel variant: render a few shares with the library DT_LIB names
(default: this tree's libdt.so) and write their floats to OUT.npz; with --compare A.npz B.npz,
report whether every share is bit-identical (and the rays / shadow rays traced).

    DT_LIB=distraytracer_amd/variants/libdt_x.so python tools/variant_check.py gpurun_out/x.npz
    python tools/variant_check.py gpurun_out/base.npz
    python tools/variant_check.py --compare gpurun_out/base.npz gpurun_out/x.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CASES = [  # (name, builder, frame, models, W, H, spp, depth, world)
    ("c3_1of64", "final", 240, 0, 1920, 1080, 64, 8, 64),
    ("c2_1of16", "final", 240, 0, 800, 600, 16, 4, 16),
    ("c4_1of256", "final", 240, 1, 1920, 1080, 256, 8, 256),
    ("c5_1088_1of512", "final", 1088, 0, 3840, 2160, 64, 10, 512),
    ("c5_1920_1of512", "final", 1920, 0, 3840, 2160, 64, 10, 512),
    ("c5_2200_cloud_1of64", "final", 2200, 0, 3840, 2160, 1, 10, 64),
]


def render_all(out):
    import torch
    import distraytracer_amd as dt
    res = {}
    only = os.environ.get("VC_CASES")   # comma-separated case names (default: all)
    for name, b, frame, models, W, H, spp, depth, world in CASES:
        if only and name not in only.split(","):
            continue
        g = dt.globals_default()
        g.use_model = models
        built = dt.build_scene(b, frame, g)
        g.xRes, g.yRes, g.antialias_samples, g.max_depth = W, H, spp, depth
        tile = dt.tiles(rank=1 % world, world=world, layout=dt.DT_OUT_SLAB)
        scene = dt.Scene(built, g)
        o = torch.zeros(dt.slab_floats(g, tile), dtype=torch.float32, device="cuda")
        st = dt.render(scene, g, frame, o, tile)
        scene.close()
        res[name] = o.cpu().numpy()
        res[name + "_rays"] = np.array([st.rays, st.shadow_rays], dtype=np.int64)
        print("%s: %.2f ms, rays %d shadow %d, donate_overflow %d" % (
            name, st.trace_kernel_ms, st.rays, st.shadow_rays, st.donate_overflow), flush=True)
    # renderImageCloud (dt_sky_kernel: one cloudColor per lane, 256-thread blocks)
    for frame in ((1, 2) if not only or "sky" in only else ()):
        g = dt.globals_default()
        g.xRes, g.yRes = 640, 480
        o = torch.zeros(3 * g.xRes * g.yRes, dtype=torch.float32, device="cuda")
        dt.render_sky(g, frame, o, dt.tiles())
        res["sky_640_f%d" % frame] = o.cpu().numpy()
        print("sky_640_f%d done" % frame, flush=True)
    np.savez(out, **res)


def compare(a, b):
    A, B = np.load(a), np.load(b)
    ok = True
    for k in A.files:
        same = np.array_equal(A[k].view(np.uint32) if A[k].dtype == np.float32 else A[k],
                              B[k].view(np.uint32) if B[k].dtype == np.float32 else B[k])
        ok &= same
        print("%-20s %s" % (k, "identical" if same else "DIFFERENT"))
    print("ALL IDENTICAL" if ok else "MISMATCH")
    return ok


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(0 if compare(sys.argv[2], sys.argv[3]) else 1)
    render_all(sys.argv[1])
