"""renderImageCloud throughput (SURVEY 8d sky micro-benchmark): 1920x1080, frames 1..8,
one pixel per lane (dt_sky_kernel). Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import distraytracer_amd as dt  # noqa: E402


def main():
    g = dt.globals_default()
    g.xRes, g.yRes = 1920, 1080
    out = torch.zeros(3 * g.xRes * g.yRes, dtype=torch.float32, device="cuda")
    dt.render_sky(g, 1, out)   # warm-up
    ms = []
    for frame in range(1, 9):
        st = dt.render_sky(g, frame, out)
        ms.append(st.kernel_ms)
    px = g.xRes * g.yRes
    print(json.dumps({"kernel": "dt_sky_kernel", "res": "1920x1080", "frames": "1..8",
                      "ms_per_frame": round(sum(ms) / len(ms), 3),
                      "mpixels_per_s": round(px / (sum(ms) / len(ms) / 1e3) / 1e6, 2)}))


if __name__ == "__main__":
    main()
