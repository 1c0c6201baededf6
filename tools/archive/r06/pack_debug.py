"""round 6: light packing mismatch hunt on C5 frame 0 (64x36, 64 spp, depth 10)"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))
import numpy as np, torch
import distraytracer_amd as dt, oracle
g = dt.globals_default(); g.use_model = 0
b = dt.build_scene("final", 0, g)
g.xRes, g.yRes, g.antialias_samples, g.max_depth = 64, 36, 64, 10
ref, rst = oracle.render(b, g, 0, dt.tiles())
def run(env):
    for k in ("DT_PACK_LANES", "DT_SG_UMBRA", "DT_SG_HULL"):
        os.environ.pop(k, None)
    os.environ.update(env)
    s = dt.Scene(b, g)
    out = torch.zeros(3 * 64 * 36, dtype=torch.float32, device="cuda")
    st = dt.render(s, g, 0, out)
    s.close()
    img = out.cpu().numpy()
    d = np.nonzero(img != ref)[0]
    px = sorted(set(int(i) // 3 for i in d))
    print(env, "rays", st.rays, rst.rays, "differing pixels", [(p % 64, 35 - p // 64) for p in px][:10],
          "max", float(np.abs(img - ref).max()), flush=True)
run({"DT_PACK_LANES": "0"})
run({"DT_PACK_LANES": "64"})
run({"DT_PACK_LANES": "64", "DT_SG_UMBRA": "0"})
run({"DT_PACK_LANES": "64", "DT_SG_HULL": "0"})
run({"DT_PACK_LANES": "8"})
