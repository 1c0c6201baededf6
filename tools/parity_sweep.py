"""Parity across the C5 animation: every `step`-th frame n of buildFinal(n*8) (frames 0..299, the
room, the transition, the tunnel with its motion blur, the cloud frames), rendered at a small
resolution by libdt (the build each frame selects, the work-sharing kernel where tools/animate.py
would use it) and by the oracle on the same inputs, compared channel by channel (max|diff|, bit
identity, equal ray counts). C5's own settings except the resolution: 64 spp, depth 10 (the
builder's 1 spp for the cloud frames). One line per frame; a final summary line.

    python tools/parity_sweep.py [WxH] [step] [start] [stop]     (default 96x54, 5, 0, 300)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import distraytracer_amd as dt  # noqa: E402
import oracle  # noqa: E402


def main():
    W, H = (int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "96x54").split("x"))
    step = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    start = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    stop = int(sys.argv[4]) if len(sys.argv) > 4 else 300
    worst, n_bad, n_frames = 0.0, 0, 0
    for n in range(start, stop, step):
        t0 = time.time()
        g = dt.globals_default()
        g.use_model = 0
        g.xRes, g.yRes, g.antialias_samples, g.max_depth = W, H, 64, 10
        built = dt.build_scene("final", n * 8, g)   # the builder may force 1 spp (cloud frames)
        s = dt.Scene(built, g)
        out = torch.zeros(3 * W * H, dtype=torch.float32, device="cuda")
        st = dt.render(s, g, n * 8, out)
        gpu = out.cpu().numpy()
        name = dt.trace_build(built, g, n * 8)[0]
        # the work-sharing kernel too where tools/animate.py --donate auto may take it (deep cascades)
        gpu_dn = None
        if 120 <= n <= 140 and g.antialias_samples > 1:
            s.set_kernel(dt.DT_KERNEL_DONATE)
            out.zero_()
            st_dn = dt.render(s, g, n * 8, out)
            gpu_dn = out.cpu().numpy()
        s.close()
        ref, rst = oracle.render(built, g, n * 8, dt.tiles(), nthreads=16)
        ok = ~(np.isnan(gpu) | np.isnan(ref))
        diff = float(np.abs(gpu[ok].astype(np.float64) - ref[ok]).max()) if ok.any() else 0.0
        same = bool(np.array_equal(gpu, ref, equal_nan=True))
        rays_equal = int(st.rays) == int(rst.rays)
        if gpu_dn is not None:
            same = same and bool(np.array_equal(gpu_dn, ref, equal_nan=True))
            rays_equal = rays_equal and int(st_dn.rays) == int(rst.rays)
            name += "+dn"
        worst = max(worst, diff)
        n_bad += 0 if (same and rays_equal) else 1
        n_frames += 1
        print(json.dumps({"n": n, "frame": n * 8, "build": name, "spp": g.antialias_samples, "max_abs": diff,
                          "bit_identical": same, "rays": int(st.rays), "rays_equal": rays_equal,
                          "sky_pixels": int(st.sky_pixels), "s": round(time.time() - t0, 2)}), flush=True)
    print(json.dumps({"frames": n_frames, "resolution": "%dx%d" % (W, H), "worst_max_abs": worst,
                      "frames_not_identical": n_bad}), flush=True)


if __name__ == "__main__":
    main()
