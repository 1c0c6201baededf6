"""Start-side culling of the shadow-grid lists (host_shadowgrid.cpp header) on the GPU. The lists
are host data that decide which leaves the device tests; the images must not change:

  * C3's room (full 1920x1080 frame, 8 spp, depth 8) and C5's frames 640 (room), 1200 and 1920
    (tunnel, blur-padded lists): scenes built with DT_SG_START=0 and with the default, bit for bit,
    with the same rays and shadow rays;
  * a camera outside the box of ray origins the lists assumed (the root box and the build camera's
    eye region): prepare_render drops the lists (the trees are walked) and the image is the
    oracle's.
"""
import numpy as np
import pytest
import torch

import distraytracer_amd as dt
import oracle

pytestmark = pytest.mark.gpu

from parity_check import assert_parity


def _render(scene, g, frame):
    out = torch.zeros(3 * g.xRes * g.yRes, dtype=torch.float32, device="cuda")
    st = dt.render(scene, g, frame, out)
    return out.cpu().numpy(), st


@pytest.mark.parametrize("frame,W,H,spp,depth", [(240, 1920, 1080, 8, 8), (640, 960, 540, 8, 10),
                                                 (1200, 960, 540, 8, 10), (1920, 960, 540, 8, 10)])
def test_start_side_lists_bit_identical(cuda, monkeypatch, frame, W, H, spp, depth):
    g = dt.globals_default()
    g.use_model = 0
    built = dt.build_scene("final", frame, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth = W, H, spp, depth
    res = []
    for env in ("0", "1"):
        monkeypatch.setenv("DT_SG_START", env)
        entries = dt.accel_info(built, g)["sg_list_entries"]
        scene = dt.Scene(built, g)
        try:
            img, st = _render(scene, g, frame)
        finally:
            scene.close()
        res.append((img, st, entries))
    (a, sa, ea), (b, sb, eb) = res
    print("frame %d: list entries %d -> %d, kernel %.2f -> %.2f ms" % (frame, ea, eb, sa.kernel_ms, sb.kernel_ms))
    assert eb < ea
    assert sa.rays == sb.rays and sa.shadow_rays == sb.shadow_rays
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_camera_outside_origin_box(cuda):
    """The scene's lists are built for C3's camera; a render from a camera 3000 units above the
    room (outside the root box: the giant window-frame prisms end at y = 1004) must not use them.
    Small frame, against the oracle."""
    g = dt.globals_default()
    g.use_model = 0
    built = dt.build_scene("final", 240, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth = 48, 32, 4, 4
    scene = dt.Scene(built, g)
    try:
        g2 = dt.globals_default()
        g2.use_model = 0
        g2.xRes, g2.yRes, g2.antialias_samples, g2.max_depth = 48, 32, 4, 4
        g2.eye[1] = g.eye[1] + 3000.0
        img, st = _render(scene, g2, 240)
        ref, rst = oracle.render(built, g2, 240, dt.tiles())
        assert st.rays == rst.rays and st.shadow_rays == rst.shadow_rays
        assert_parity("C3 scene, camera outside the origin box", img, ref)
        img1, _ = _render(scene, g, 240)   # the build camera again: the lists are used
        ref1, _ = oracle.render(built, g, 240, dt.tiles())
        assert_parity("C3 scene, build camera", img1, ref1)
    finally:
        scene.close()
