"""Diagnostic: colours of a few C5 cloud-frame pixels through the deferred per-lane sky and (with
DT_SKY_DEFER=0) the cooperative march; SKY2000=1 also compares renderImageCloud at frame 2000 with
the oracle. Written while finding why a called (not inlined) cloud_color_lane returned wrong colours
(DESIGN.md §4)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import distraytracer_amd as dt  # noqa: E402


def main():
    g = dt.globals_default()
    g.use_model = 0
    built = dt.build_scene("final", 2000, g)
    g.xRes, g.yRes = 320, 180
    tile = dt.tiles(x0=128, y0=60, x1=176, y1=92)
    s = dt.Scene(built, g)
    out = torch.zeros(3 * g.xRes * g.yRes, dtype=torch.float32, device="cuda")
    st = dt.render(s, g, 2000, out, tile)
    img = out.cpu().numpy().reshape(g.yRes, g.xRes, 3)[::-1]
    print("sky_pixels", st.sky_pixels, "pixels", st.pixels)
    for (x, y) in [(128, 60), (150, 70), (175, 91)]:
        print((x, y), img[y, x])
    print("frame_f-ish globals: eye", list(g.eye), "lookingAt", list(g.lookingAt), "perlin", g.perlin_cloud)


if __name__ == "__main__":
    main()


def sky2000():
    """renderImageCloud at frame 2000 (dt_sky_kernel) on a few rows vs the oracle"""
    import oracle
    g = dt.globals_default()
    g.xRes, g.yRes = 320, 180
    tile = dt.tiles(x0=0, y0=60, x1=320, y1=62)
    out = torch.zeros(3 * g.xRes * g.yRes, dtype=torch.float32, device="cuda")
    dt.render_sky(g, 2000, out, tile)
    gpu = out.cpu().numpy()
    ref = np.zeros_like(gpu)
    oracle.render_sky(g, 2000, tile, ref)
    print("render_sky frame 2000 max|diff| %.4g" % float(np.abs(gpu - ref).max()))


if __name__ == "__main__" and os.environ.get("SKY2000"):
    sky2000()
