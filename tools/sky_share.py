"""Diagnostic: how much of a C5 frame's render time is the per-pixel cloud sky.

Renders buildFinal(frame) with the sky on (perlin_cloud as the scene sets it) and off
(default colour for misses) and prints both kernel times.

    python tools/sky_share.py 1200 1920x1080 64
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import distraytracer_amd as dt  # noqa: E402


def run(frame, W, H, spp, sky):
    g = dt.globals_default()
    g.use_model = 0
    g.xRes, g.yRes, g.antialias_samples, g.max_depth = W, H, spp, 10
    b = dt.build_scene("final", frame, g)
    if not sky:
        g.perlin_cloud = 0
    s = dt.Scene(b, g)
    out = torch.zeros(3 * W * H, dtype=torch.float32, device="cuda")
    dt.render(s, g, frame, out)   # warm-up
    st = dt.render(s, g, frame, out)
    s.close()
    return st


def main():
    frames = [int(f) for f in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1200]
    W, H = (int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "1920x1080").split("x"))
    spp = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    for f in frames:
        on, off = run(f, W, H, spp, True), run(f, W, H, spp, False)
        print(json.dumps({"frame": f, "res": "%dx%d" % (W, H), "spp": on.samples // max(on.pixels, 1),
                          "kernel_ms_sky": round(on.kernel_ms, 2), "kernel_ms_nosky": round(off.kernel_ms, 2),
                          "sky_pixels": on.sky_pixels}), flush=True)


if __name__ == "__main__":
    main()
