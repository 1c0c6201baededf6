"""Diagnostic: per-pixel wave cycles of one C3 frame from a -DDT_ITEM_TIMES build (DT_LIB=...):
the slowest items, where they are, and the share of the frame they hold."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import distraytracer_amd as dt  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    g, built = bench.build_globals(dt, cfg)
    s = dt.Scene(built, g)
    out = torch.zeros(3 * g.xRes * g.yRes, dtype=torch.float32, device="cuda")
    dt.render(s, g, 240, out)
    st = dt.render(s, g, 240, out)
    cyc = out.view(g.yRes, g.xRes, 3)[:, :, 0].cpu().numpy()[::-1] * 1e4   # y up
    flat = cyc.ravel()
    order = np.argsort(flat)[::-1]
    print("kernel ms %.2f  items %d  mean %.3g  median %.3g  p99 %.3g  p99.99 %.3g  max %.3g cycles" %
          (st.kernel_ms, flat.size, flat.mean(), np.median(flat), np.percentile(flat, 99), np.percentile(flat, 99.99), flat.max()))
    for k in order[:25]:
        y, x = divmod(int(k), g.xRes)
        print("  pixel (%d, %d): %.4g cycles (%.1fx mean)" % (x, y, flat[k], flat[k] / flat.mean()))
    np.save(os.path.join(os.environ.get("OUT", "."), "item_cycles_%s.npy" % cfg), cyc.astype(np.float32))


if __name__ == "__main__":
    main()
