"""Bit-identity of start-side culling (host_shadowgrid.cpp header): every case is rendered twice on
the GPU, from a scene whose shadow-grid lists were built as before round 6 (DT_SG_START=0,
DT_SG_QUAD=0: no start-side culling, no hull culling of sphere and cylinder leaves) and one built
with both (DT_SG_START=2: start-side culling on every frame, the overflowing transition frames included;
SG_START_MODE=1 checks the default, which skips those), and the two images, ray counts and
shadow-ray counts must agree exactly. The lists are host data, so any difference in what the device
tests would show up here.

    python tools/sg_start_check.py [case ...]      (default: all; prints one line per case)
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CASES = {  # name: (frame, models, W, H, spp, depth)
    "c3": (240, 0, 1920, 1080, 64, 8),
    "c2": (240, 0, 800, 600, 16, 4),
    "c5_0000": (0, 0, 1920, 1080, 16, 10),
    "c5_0320": (320, 0, 1920, 1080, 16, 10),
    "c5_0640": (640, 0, 1920, 1080, 16, 10),
    "c5_0952": (952, 0, 1920, 1080, 16, 10),
    "c5_1040": (1040, 0, 960, 540, 16, 10),
    "c5_1088": (1088, 0, 960, 540, 16, 10),
    "c5_1200": (1200, 0, 1920, 1080, 16, 10),
    "c5_1600": (1600, 0, 1920, 1080, 16, 10),
    "c5_1920": (1920, 0, 1920, 1080, 16, 10),
}


def main():
    import torch
    import distraytracer_amd as dt
    names = sys.argv[1:] or list(CASES)
    bad = 0
    for name in names:
        frame, models, W, H, spp, depth = CASES[name]
        g = dt.globals_default()
        g.use_model = models
        built = dt.build_scene("final", frame, g)
        g.xRes, g.yRes, g.antialias_samples, g.max_depth = W, H, spp, depth
        res = []
        for env in ("0", os.environ.get("SG_START_MODE", "2")):
            os.environ["DT_SG_START"] = env
            os.environ["DT_SG_QUAD"] = "0" if env == "0" else "1"   # the baseline: lists before round 6
            info = dt.accel_info(built, g)
            scene = dt.Scene(built, g)
            out = torch.zeros(3 * W * H, dtype=torch.float32, device="cuda")
            st = dt.render(scene, g, frame, out)
            res.append((out.cpu().numpy(), st, info["sg_list_entries"]))
            scene.close()
        os.environ.pop("DT_SG_START", None)
        os.environ.pop("DT_SG_QUAD", None)
        (a, sa, ea), (b, sb, eb) = res
        same = np.array_equal(a.view(np.uint32), b.view(np.uint32)) and sa.rays == sb.rays and sa.shadow_rays == sb.shadow_rays
        bad += not same
        print("%s: %s  list entries %d -> %d  rays %d/%d shadow %d/%d  kernel ms %.2f -> %.2f" %
              (name, "bit-identical" if same else "DIFFERENT", ea, eb, sa.rays, sb.rays, sa.shadow_rays, sb.shadow_rays,
               sa.kernel_ms, sb.kernel_ms), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
