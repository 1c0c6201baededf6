"""Chunk items (spp > 64): every 64-sample chunk of a pixel is a queue item of its own, so a pixel's
chunks run on different waves; each chunk stores its sample colours, and dt_chunk_sum_kernel, launched
after the trace (and sky-item) launches, adds each pixel's colours in sample order (dt_kernels.hip item
loop and dt_chunk_sum_kernel, dt_api.cpp enqueue_render). The reference sums a pixel's
samples in order (render_final_project.cpp:1062-1213: `color += tmp_color` per sample, then
`/= sampled_n`), so the images must be bit-identical to the per-pixel items (DT_CHUNK_ITEMS=0, one
wave running the chunks in turn) and to the oracle, for:

  * C4's settings (256 spp, depth 8, the OBJ models) on a tile share, pixel-major (the default) and
    chunk-major (DT_CHUNK_ITEMS=2: a pixel's chunks sit n_items queue positions apart, so they run
    on different waves and, at any grid, in different phases of the launch);
  * spp that leave a partial last chunk (81, 100, 144 spp: 17, 36, 16 samples);
  * the sky-item launch (still builds list a chunk with a missed sample; the *_sky build renders the
    listed chunks again, storing their colours over the first launch's): the spheres scene with clouds;
  * a motion-blur build (tunnel frame), and renders repeated on one scene (the colour buffer is
    reused from launch to launch; every chunk overwrites its own slots, so nothing carries over).
"""
import numpy as np
import pytest
import torch

import distraytracer_amd as dt
import oracle

pytestmark = pytest.mark.gpu

from parity_check import assert_parity, log_equal


def _render(scene, g, frame, tile):
    n = dt.slab_floats(g, tile) if tile.layout == dt.DT_OUT_SLAB else 3 * g.xRes * g.yRes
    out = torch.zeros(max(n, 1), dtype=torch.float32, device="cuda")
    st = dt.render(scene, g, frame, out, tile)
    return out.cpu().numpy()[:n], st


def _oracle(built, g, frame, tile):
    n = dt.slab_floats(g, tile) if tile.layout == dt.DT_OUT_SLAB else 3 * g.xRes * g.yRes
    ref, rst = oracle.render(built, g, frame, tile, out=np.zeros(max(n, 1), dtype=np.float32))
    return ref[:n], rst


def _modes(monkeypatch, built, g, frame, tile, label, modes=("1", "2", "0"), repeat=1):
    """Render under each DT_CHUNK_ITEMS mode (one scene, `repeat` renders per mode); the first
    image against the oracle, every other bit for bit against it."""
    scene = dt.Scene(built, g)
    ref, rst = _oracle(built, g, frame, tile)
    first = None
    try:
        for m in modes:
            monkeypatch.setenv("DT_CHUNK_ITEMS", m)
            for k in range(repeat):
                img, st = _render(scene, g, frame, tile)
                print("%s DT_CHUNK_ITEMS=%s #%d: pixels=%d rays=%d" % (label, m, k, st.pixels, st.rays))
                assert st.pixels == rst.pixels and st.samples == rst.samples
                assert st.rays == rst.rays and st.shadow_rays == rst.shadow_rays
                assert st.stack_overflows == 0 and st.nan_pixels == rst.nan_pixels
                assert st.sky_pixels == (first[1].sky_pixels if first is not None else st.sky_pixels)
                if first is None:
                    assert_parity("%s (chunk items %s)" % (label, m), img, ref)
                    first = (img, st)
                else:
                    log_equal("%s: chunk items %s vs %s" % (label, m, modes[0]), img, first[0])
    finally:
        scene.close()
    return first[1], rst


def test_c4_chunk_items(cuda, monkeypatch):
    """C4 (buildFinal(240) with the models, 1920x1080, 256 spp, depth 8), rank 5's share of a
    256-way split in 16x16 tiles: chunk items pixel-major
    and chunk-major, and per-pixel items, bit-identical to each other and to the oracle."""
    g = dt.globals_default()
    g.use_model = 1
    built = dt.build_scene("final", 240, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth = 1920, 1080, 256, 8
    tile = dt.tiles(tile_w=16, tile_h=16, rank=5, world=256, layout=dt.DT_OUT_SLAB)
    st, rst = _modes(monkeypatch, built, g, 240, tile, "C4 256 spp 1/256")
    assert st.samples == st.pixels * 256 and st.tex_fetches > 0


@pytest.mark.parametrize("aa,depth", [(81, 4), (100, 3), (144, 2)])
def test_partial_last_chunk(cuda, monkeypatch, aa, depth):
    """spp = 81, 100, 144: the last chunk holds 17, 36, 16 samples. The C4 scene (mesh build) and the C3
    scene (room build); both builds carry the chunk code."""
    for models in (0, 1):
        g = dt.globals_default()
        g.use_model = models
        built = dt.build_scene("final", 240, g)
        g.xRes, g.yRes, g.antialias_samples, g.max_depth = 1920, 1080, aa, depth
        tile = dt.tiles(tile_w=16, tile_h=16, rank=1, world=1024, layout=dt.DT_OUT_SLAB)
        _modes(monkeypatch, built, g, 240, tile, "final models=%d aa=%d" % (models, aa))


@pytest.mark.parametrize("aa,world", [(100, 1), (256, 3)])
def test_chunk_items_sky_launch(cuda, monkeypatch, aa, world):
    """The spheres scene with perlin_cloud (sky around the spheres) at spp > 64: the still build
    lists every chunk with a missed sample, the *_sky build renders those chunks again, and the
    sum kernel adds the colours after both launches. Whole image and a slab split, each mode
    rendered twice on one scene."""
    g = dt.globals_default()
    built = dt.build_scene("spheres", 0, g)
    g.perlin_cloud = 1
    g.xRes, g.yRes, g.antialias_samples, g.max_depth = 40, 24, aa, 3
    tile = (dt.tiles(tile_w=8, tile_h=8, rank=world - 1, world=world, layout=dt.DT_OUT_SLAB) if world > 1
            else dt.tiles())
    st, rst = _modes(monkeypatch, built, g, 0, tile, "spheres sky aa=%d world=%d" % (aa, world), repeat=2)
    assert rst.sky_pixels > 0 and st.sky_pixels > 0


def test_chunk_items_blur_build(cuda, monkeypatch):
    """A C5 tunnel frame (buildFinal(1200): motion blur, ads in motion; the tunnel build) at 100
    spp, depth 4, on a 1/256 share of a 960x540 frame."""
    g = dt.globals_default()
    g.use_model = 0
    built = dt.build_scene("final", 1200, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth = 960, 540, 100, 4
    tile = dt.tiles(tile_w=16, tile_h=16, rank=2, world=256, layout=dt.DT_OUT_SLAB)
    st, rst = _modes(monkeypatch, built, g, 1200, tile, "tunnel 1200 aa=100", repeat=2)
    assert st.rays > st.samples
