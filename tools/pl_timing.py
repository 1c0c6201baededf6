"""Diagnostic: host time of dt_scene_create (primary lists included) and of the first render,
per C5 frame at a given resolution (DT_TIMING=1 adds the stage times on stderr)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import distraytracer_amd as dt  # noqa: E402


def main():
    W, H = (int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "3840x2160").split("x"))
    for n in [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "30,270").split(",")]:
        g = dt.globals_default()
        g.use_model = 0
        g.xRes, g.yRes, g.antialias_samples, g.max_depth = W, H, 64, 10
        t0 = time.perf_counter()
        b = dt.build_scene("final", n * 8, g)
        t1 = time.perf_counter()
        s = dt.Scene(b, g)
        t2 = time.perf_counter()
        out = torch.zeros(3 * W * H, dtype=torch.float32, device="cuda")
        st = dt.render(s, g, n * 8, out)
        t3 = time.perf_counter()
        print("n %d: build %.1f ms, scene create %.1f ms, first render %.1f ms (kernel %.1f ms)" %
              (n, (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, st.kernel_ms), flush=True)
        s.close()


if __name__ == "__main__":
    main()
