"""Diagnostic: where does the device differ from the oracle on a C5 tunnel window?"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distraytracer_amd as dt  # noqa: E402
import oracle  # noqa: E402


def run(frame, blur, spp=4, depth=3, win=(128, 60, 192, 108)):
    g = dt.globals_default()
    g.use_model = 0
    b = dt.build_scene("final", frame, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth = 320, 180, spp, depth
    if blur is not None:
        g.blur_samples = blur
    x0, y0, x1, y1 = win
    tile = dt.tiles(x0=x0, y0=y0, x1=x1, y1=y1)
    s = dt.Scene(b, g)
    out = torch.zeros(3 * 320 * 180, dtype=torch.float32, device="cuda")
    dt.render(s, g, frame, out, tile)
    gpu = out.cpu().numpy().reshape(180, 320, 3)[::-1]
    ref = oracle.render(b, g, frame, tile)[0].reshape(180, 320, 3)[::-1]
    d = np.abs(gpu.astype(np.float64) - ref)
    bad = np.argwhere(d > 1e-4)
    print("frame %d blur %s spp %d depth %d: %d bad channels, max %.3g" % (frame, blur, spp, depth, len(bad), d.max()))
    for y, x, c in bad[:8]:
        print("  px (%d,%d) c%d gpu %.4f ref %.4f" % (x, y, c, gpu[y, x, c], ref[y, x, c]))
    s.close()


if __name__ == "__main__":
    torch.cuda.set_device(0)
    run(1680, None)
    run(1680, 0)
    run(1680, None, spp=1)
    run(1680, None, depth=1)
    run(1200, None)
    run(1200, 0)
