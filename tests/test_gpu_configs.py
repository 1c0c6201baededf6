"""GPU parity at the BASELINE configs' real settings (BASELINE.json configs[1..4]): the HIP path
against the CPU oracle on the same inputs and seeds, at the full resolution, spp and depth of
each config. test_gpu_parity.py covers the features on small windows; this file covers the
configurations themselves:

  C2  buildFinal(240), 800x600, 16 spp, depth 4: the whole frame
  C3  buildFinal(240), 1920x1080, 64 spp, depth 8 (north_star's target): the whole frame
  C4  buildFinal(240) with the models, 1920x1080, 256 spp, depth 8: a 1/64 tile share spread
      over the frame. spp > 64 runs the chunked path (4 chunks of 64 samples per pixel, the
      per-pixel sums carried across chunks, dt_kernels.hip dt_trace_kernel)
  C5  buildFinal(n*8) at 3840x2160, 64 spp, depth 10: 1/512 tile shares of a room frame, the
      room-to-tunnel transition (deep glossy cascades), two tunnel frames with motion blur and
      a cloud frame (1 spp, forced by the builder)

Shares are the multi-GPU tile split's own (rank 0 of `world`, slab layout), so they also run the
slab store path bench.py and multigpu.py use at N > 1. Tolerance (north_star): 1e-4 per
channel, asserted on the largest channel difference (tests/parity_check.py); the images are
bit-identical today (max|diff| = 0, logged per case).
Oracle time on the GPU box's 16 host threads: C3 ~20 s, the others 1-4 s each.
"""
import numpy as np
import pytest
import torch

import distraytracer_amd as dt
import oracle

pytestmark = pytest.mark.gpu

from parity_check import assert_parity


def _globals(builder, frame, models, W, H, spp, depth, brdf=2):
    g = dt.globals_default()
    g.use_model = models
    built = dt.build_scene(builder, frame, g)
    g.xRes, g.yRes = W, H
    if spp:   # 0: keep the builder's settings (cloud frames force 1 spp)
        g.antialias_samples, g.max_depth = spp, depth
    g.brdf_samples = brdf
    return g, built


def _check(label, g, built, frame, tile):
    scene = dt.Scene(built, g)
    if tile.layout == dt.DT_OUT_SLAB:
        n = dt.slab_floats(g, tile)
    else:
        n = 3 * g.xRes * g.yRes
    out = torch.zeros(n, dtype=torch.float32, device="cuda")
    st = dt.render(scene, g, frame, out, tile)
    scene.close()
    gpu = out.cpu().numpy()
    ref, rst = oracle.render(built, g, frame, tile, out=np.zeros(n, dtype=np.float32))
    print("%s: pixels=%d samples=%d rays=%d" % (label, st.pixels, st.samples, st.rays))
    # identical work: the same rays and shadow rays as the reference loop restated by the oracle
    assert st.pixels == rst.pixels and st.samples == rst.samples
    assert st.rays == rst.rays and st.shadow_rays == rst.shadow_rays
    # the conditions the reference aborts on, and the device's own limits, stay at zero
    assert st.stack_overflows == 0 and st.nan_pixels == rst.nan_pixels == 0
    assert st.uv_out_of_range == rst.uv_out_of_range
    assert st.glossy_exhausted == rst.glossy_exhausted
    assert_parity(label, gpu, ref)
    return st


def test_c3_full_frame(cuda):
    """C3, the whole 1920x1080 frame at 64 spp, depth 8 (BASELINE.json configs[2])."""
    g, built = _globals("final", 240, 0, 1920, 1080, 64, 8)
    st = _check("C3 full frame", g, built, 240, dt.tiles())
    assert st.samples == 1920 * 1080 * 64


def test_c2_full_frame(cuda):
    """C2, the whole 800x600 frame at 16 spp, depth 4 (BASELINE.json configs[1])."""
    g, built = _globals("final", 240, 0, 800, 600, 16, 4)
    st = _check("C2 full frame", g, built, 240, dt.tiles())
    assert st.samples == 800 * 600 * 16


def test_c4_256spp_share(cuda):
    """C4 at its real settings: 256 spp (4 chunks of 64 samples per pixel), depth 8, with the
    substitute OBJ models; rank 0's share of a 64-way tile split (~32k pixels spread over the
    frame, the model columns included)."""
    g, built = _globals("final", 240, 1, 1920, 1080, 256, 8)
    tile = dt.tiles(rank=0, world=64, layout=dt.DT_OUT_SLAB)
    st = _check("C4 256 spp 1/64", g, built, 240, tile)
    assert st.samples == st.pixels * 256 and st.tex_fetches > 0


C5_FRAMES = [  # n (frame n*8): what it exercises
    (30, "room, glossy floor/doors, area lights"),
    (136, "room-to-tunnel transition: deep glossy cascades (8 rays per sample)"),
    (150, "tunnel, ads in motion, linear blur shift"),
    (240, "tunnel, cubic blur shift up to ~80 units (bump tree overflow, tree walks)"),
    (250, "cloud frame: the builder forces 1 spp, aperture 0 (scene.h:795-796)"),
]


@pytest.mark.parametrize("n,what", C5_FRAMES, ids=[str(n) for n, _ in C5_FRAMES])
def test_c5_4k_frame_share(cuda, n, what):
    """C5 at its real settings: buildFinal(n*8) from fresh globals at 3840x2160, 64 spp, depth 10
    (cloud frames: the builder's 1 spp); rank 0's share of a 512-way tile split."""
    cloud = n >= 244
    g, built = _globals("final", n * 8, 0, 3840, 2160, 0 if cloud else 64, 10)
    if not cloud:
        assert g.antialias_samples == 64 and g.max_depth == 10
    tile = dt.tiles(rank=0, world=512, layout=dt.DT_OUT_SLAB)
    st = _check("C5 frame %d (%s) 1/512" % (n * 8, what), g, built, n * 8, tile)
    if cloud:
        assert st.samples == st.pixels and st.sky_pixels > 0
    else:
        assert st.samples == st.pixels * 64
    if n in (150, 240):
        assert st.rays > st.samples   # motion-blur re-traces ran
