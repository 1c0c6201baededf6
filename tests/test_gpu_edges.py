"""GPU parity at the edges of the render loop's input space: image sizes that are
not multiples of the tile (ragged right and top tiles), single-pixel and single-row images,
antialias_samples that are not perfect squares (the reference takes int(sqrt(n))^2 samples,
render_final_project.cpp:1040-1046), depth 1 and the configs' depths, and a tile split with more
ranks than tiles (ranks whose slab holds no pixel). Every case is compared with the CPU oracle
bit for bit on the same seeds (max|diff| = 0; north_star's 1e-4 tolerance is the bound written
in the assertion), and the work counters must match the reference loop's.
"""
import numpy as np
import pytest
import torch

import distraytracer_amd as dt
import oracle

pytestmark = pytest.mark.gpu

from parity_check import assert_parity, log_equal


def _render_both(built, g, frame, tile):
    n = dt.slab_floats(g, tile) if tile.layout == dt.DT_OUT_SLAB else 3 * g.xRes * g.yRes
    scene = dt.Scene(built, g)
    out = torch.zeros(max(n, 1), dtype=torch.float32, device="cuda")
    st = dt.render(scene, g, frame, out, tile)
    scene.close()
    gpu = out.cpu().numpy()[:n]
    ref, rst = oracle.render(built, g, frame, tile, out=np.zeros(max(n, 1), dtype=np.float32))
    return gpu, ref[:n], st, rst


def _assert_same(label, gpu, ref, st, rst):
    print("%s: pixels=%d samples=%d rays=%d" % (label, st.pixels, st.samples, st.rays))
    assert st.pixels == rst.pixels and st.samples == rst.samples
    assert st.rays == rst.rays and st.shadow_rays == rst.shadow_rays
    assert st.stack_overflows == 0 and st.nan_pixels == rst.nan_pixels
    assert_parity(label, gpu, ref)


# (W, H, antialias_samples, depth): spp = int(sqrt(aa))^2
SIZES = [(1, 1, 4, 2), (7, 5, 10, 3), (33, 17, 2, 1), (97, 3, 16, 4), (2, 41, 9, 8)]


@pytest.mark.parametrize("W,H,aa,depth", SIZES)
def test_ragged_sizes_spheres(cuda, W, H, aa, depth):
    """buildSceneSpheres(0) (C1's scene, motion-blurred spheres) at sizes that leave partial
    tiles, in the image layout with 32x32 tiles."""
    g = dt.globals_default()
    built = dt.build_scene("spheres", 0, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth = W, H, aa, depth
    gpu, ref, st, rst = _render_both(built, g, 0, dt.tiles())
    assert st.pixels == W * H
    assert st.samples == W * H * int(int(aa ** 0.5) ** 2)
    _assert_same("spheres %dx%d aa=%d depth=%d" % (W, H, aa, depth), gpu, ref, st, rst)


@pytest.mark.parametrize("W,H,aa,depth", [(13, 9, 4, 8), (70, 1, 2, 4)])
def test_ragged_sizes_final(cuda, W, H, aa, depth):
    """buildFinal(240) (the C2/C3 scene: glossy cascades, area lights, textures) at ragged sizes."""
    g = dt.globals_default()
    g.use_model = 0
    built = dt.build_scene("final", 240, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth = W, H, aa, depth
    gpu, ref, st, rst = _render_both(built, g, 240, dt.tiles(tile_w=8, tile_h=8))
    _assert_same("final %dx%d aa=%d depth=%d" % (W, H, aa, depth), gpu, ref, st, rst)


def test_more_ranks_than_tiles(cuda):
    """20x12 in 8x8 tiles is 3x2 = 6 tiles (ragged on both axes); split over 8 ranks, two ranks own
    no tile. Every rank's slab matches the oracle's, the empty ranks render nothing, and the
    unpacked slabs give the single-GPU image."""
    g = dt.globals_default()
    g.use_model = 0
    built = dt.build_scene("final", 240, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth = 20, 12, 4, 4
    world = 8
    base = dt.tiles(tile_w=8, tile_h=8, rank=0, world=world, layout=dt.DT_OUT_SLAB)
    slab_n = dt.slab_floats_max(g, base)
    slabs = np.zeros(world * slab_n, dtype=np.float32)
    empty = 0
    for r in range(world):
        tile = dt.tiles(tile_w=8, tile_h=8, rank=r, world=world, layout=dt.DT_OUT_SLAB)
        gpu, ref, st, rst = _render_both(built, g, 240, tile)
        _assert_same("rank %d of %d" % (r, world), gpu, ref, st, rst)
        empty += st.pixels == 0
        slabs[r * slab_n:r * slab_n + gpu.size] = gpu
    assert empty == 2
    image = torch.zeros(3 * 20 * 12, dtype=torch.float32, device="cuda")
    dt.unpack_slabs(g, base, world, torch.from_numpy(slabs).cuda(), image)
    torch.cuda.synchronize()
    whole, ref, st, rst = _render_both(built, g, 240, dt.tiles())
    log_equal("8 ranks' slabs unpacked vs single-GPU image", image.cpu().numpy(), whole)


@pytest.mark.parametrize("aa,depth", [(64, 8), (16, 4)])
def test_five_wave_kernel_matches(cuda, monkeypatch, aa, depth):
    """dt_trace_kernel_w5 (5 waves per SIMD, DT_W5; the default at spp >= 64) and the 4-wave
    dt_trace_kernel render the same bits, at one and at four pixels per wave; checked against the
    oracle as well."""
    g = dt.globals_default()
    g.use_model = 0
    built = dt.build_scene("final", 240, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth = 1920, 1080, aa, depth
    tile = dt.tiles(tile_w=8, tile_h=8, rank=3, world=256, layout=dt.DT_OUT_SLAB)
    imgs = []
    for w5 in ("0", "1"):
        monkeypatch.setenv("DT_W5", w5)
        gpu, ref, st, rst = _render_both(built, g, 240, tile)
        _assert_same("DT_W5=%s aa=%d" % (w5, aa), gpu, ref, st, rst)
        imgs.append(gpu)
    log_equal("dt_trace_kernel_w5 vs dt_trace_kernel aa=%d" % aa, imgs[1], imgs[0])


@pytest.mark.parametrize("aa,depth,builder,frame", [(64, 3, "final", 240), (16, 3, "final", 240),
                                                    (1, 10, "final", 2000)],
                         ids=["64spp_w5", "16spp", "1spp_sky_defer"])
def test_host_output_buffer_fully_written(cuda, aa, depth, builder, frame):
    """dt_render into a HOST buffer covering the whole image skips the host-to-device copy of the
    old contents (dt_api.cpp `covers`), so the kernels must write every float: a NaN-filled numpy
    buffer comes back without a NaN and equal to the oracle, through the 5-wave kernel (64 spp), the
    4-wave kernel (16 spp) and the deferred per-lane sky (cloud frame 2000: the builder's 1 spp)."""
    g = dt.globals_default()
    g.use_model = 0
    built = dt.build_scene(builder, frame, g)
    g.xRes, g.yRes = 96, 54
    if builder == "final" and frame < 1952:
        g.antialias_samples, g.max_depth = aa, depth
    assert g.antialias_samples == aa
    out = np.full(3 * g.xRes * g.yRes, np.nan, dtype=np.float32)
    scene = dt.Scene(built, g)
    st = dt.render(scene, g, frame, out)
    scene.close()
    ref, rst = oracle.render(built, g, frame, dt.tiles())
    assert st.pixels == g.xRes * g.yRes and st.rays == rst.rays
    if aa == 1:
        assert st.sky_pixels > 0
    assert_parity("host output buffer %dx%d aa=%d frame %d" % (g.xRes, g.yRes, aa, frame), out, ref)


@pytest.mark.parametrize("W,H,aa,depth,world", [(48, 32, 4, 2, 1), (40, 24, 64, 3, 1), (64, 48, 16, 2, 3)])
def test_sky_items_rendered_again(cuda, W, H, aa, depth, world):
    """Still-frame builds carry no sky march (dt_kernels.hip DT_SKY_AGAIN): a multi-sample item with
    a missed sample is listed and rendered again by the *_sky build in a second launch. The spheres
    scene with perlin_cloud on has sky around the spheres: 4-wave (4, 16 spp) and 5-wave (64 spp)
    builds, whole image and a slab split, against the oracle (rays and shadow rays counted once:
    the second launch keeps counters of its own and adds only its sky and NaN pixels)."""
    g = dt.globals_default()
    built = dt.build_scene("spheres", 0, g)
    g.perlin_cloud = 1
    g.xRes, g.yRes, g.antialias_samples, g.max_depth = W, H, aa, depth
    tile = dt.tiles(rank=world - 1, world=world, layout=dt.DT_OUT_SLAB) if world > 1 else dt.tiles()
    gpu, ref, st, rst = _render_both(built, g, 0, tile)
    assert rst.sky_pixels > 0 and st.sky_pixels > 0   # oracle: missed samples; GPU: pixels with one
    _assert_same("spheres sky items %dx%d aa=%d world=%d" % (W, H, aa, world), gpu, ref, st, rst)
