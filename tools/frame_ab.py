"""Diagnostic: kernel time of one buildFinal(frame) render under global overrides.

    python tools/frame_ab.py 1200 960x540 64 "" "blur_samples=0" "perlin_cloud=0"

Each quoted argument after spp is one variant: comma-separated name=value overrides applied to
the globals after the scene builder ran ("" = as built). Prints one JSON line per variant.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import distraytracer_amd as dt  # noqa: E402


def main():
    frame = int(sys.argv[1])
    W, H = (int(v) for v in sys.argv[2].split("x"))
    spp = int(sys.argv[3])
    for var in sys.argv[4:] or [""]:
        g = dt.globals_default()
        g.use_model = 0
        g.xRes, g.yRes, g.antialias_samples, g.max_depth = W, H, spp, 10
        b = dt.build_scene("final", frame, g)
        for kv in filter(None, var.split(",")):
            k, v = kv.split("=")
            setattr(g, k, type(getattr(g, k))(float(v)) if not isinstance(getattr(g, k), int) else int(v))
        s = dt.Scene(b, g)
        out = torch.zeros(3 * W * H, dtype=torch.float32, device="cuda")
        dt.render(s, g, frame, out)
        st = dt.render(s, g, frame, out)
        print(json.dumps({"frame": frame, "variant": var, "kernel_ms": round(st.kernel_ms, 2),
                          "rays_per_sample": round(st.rays / max(st.samples, 1), 3),
                          "shadow_per_sample": round(st.shadow_rays / max(st.samples, 1), 3),
                          "wave_node_visits_per_px": round(st.wave_node_visits / max(st.pixels, 1), 1),
                          "box_tests_per_sample": round(st.box_tests / max(st.samples, 1), 1)
                          if hasattr(st, "box_tests") else None}), flush=True)
        s.close()


if __name__ == "__main__":
    main()
