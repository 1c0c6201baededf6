"""GPU parity: libdt's HIP kernels vs the CPU oracle on identical inputs and seeds.

Tolerance (north_star): 1e-4 per channel on the float ppmOut values, asserted on the LARGEST
channel difference (tests/parity_check.py assert_parity), with NaN masks equal. The device
repeats the reference's operation sequence in IEEE FP64/FP32 without contraction, and evaluates
the reference's float libm calls (cosf/sinf/tanf/acosf) correctly rounded on both sides
(DESIGN.md §5), so every case below is bit-identical today (max|diff| = 0, logged per case).
"""
import ctypes

import numpy as np
import pytest
import torch

import distraytracer_amd as dt
import oracle

pytestmark = pytest.mark.gpu

from parity_check import assert_parity, log_equal


def _render_gpu(built, g, frame, tile):
    scene = dt.Scene(built, g)
    out = torch.zeros(3 * g.xRes * g.yRes, dtype=torch.float32, device="cuda")
    st = dt.render(scene, g, frame, out, tile)
    scene.close()
    return out.cpu().numpy(), st


def test_sky_render_image_cloud(cuda):
    """renderImageCloud (the reference's `perlin` mode, cpp:1685-1698) 640x480, frames 1..2."""
    g = dt.globals_default()
    g.xRes, g.yRes = 640, 480
    tile = dt.tiles(x0=0, y0=0, x1=640, y1=480)
    for frame in (1, 2):
        out = torch.zeros(3 * g.xRes * g.yRes, dtype=torch.float32, device="cuda")
        dt.render_sky(g, frame, out, tile)
        gpu = out.cpu().numpy()
        # oracle on a strided subset of rows (full frame takes minutes on CPU)
        ref = np.zeros_like(gpu)
        for y0 in range(0, 480, 40):
            oracle.render_sky(g, frame, dt.tiles(x0=0, y0=y0, x1=640, y1=y0 + 2), ref)
        rows = np.zeros((480, 640, 3), dtype=bool)
        for y0 in range(0, 480, 40):
            rows[479 - y0 - 1:479 - y0 + 1] = True
        m = rows.reshape(-1)
        assert_parity("sky frame %d" % frame, gpu[m], ref[m])


def test_spheres_c1_deterministic(cuda):
    """C1: buildSceneSpheres(0), 256x256, 1 spp, depth 1, aperture 0 (deterministic; includes
    the motion-blur re-traces of the moving spheres)."""
    g = dt.globals_default()
    built = dt.build_scene("spheres", 0, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth, g.aperture = 256, 256, 1, 1, 0.0
    tile = dt.tiles()
    gpu, st = _render_gpu(built, g, 0, tile)
    ref, _ = oracle.render(built, g, 0, tile)
    assert st.pixels == 256 * 256
    assert_parity("spheres C1", gpu, ref)


def test_spheres_c1_dof(cuda):
    """C1 with its default aperture 0.2 (DoF through the shared counter RNG)."""
    g = dt.globals_default()
    built = dt.build_scene("spheres", 0, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth = 256, 256, 4, 1
    tile = dt.tiles()
    gpu, _ = _render_gpu(built, g, 0, tile)
    ref, _ = oracle.render(built, g, 0, tile)
    assert_parity("spheres C1 dof", gpu, ref)


def test_spheres_motion_blur_shift(cuda):
    """Motion-blur re-traces with a non-zero shift: buildSceneSpheres(0) rendered at frame 1700
    (>= frame_blur, so val = move_per_frame*dt + accel_t*dt^3, Q19): every leaf box is bumped by
    +-val in y (bumpBVH, helpers.h:530-552), which runs the device's general traversal path."""
    g = dt.globals_default()
    built = dt.build_scene("spheres", 0, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth = 128, 128, 4, 2
    assert g.blur_samples > 0
    tile = dt.tiles()
    gpu, st = _render_gpu(built, g, 1700, tile)
    ref, _ = oracle.render(built, g, 1700, tile)
    assert st.rays > st.samples   # the re-traces ran
    assert_parity("spheres motion blur frame 1700", gpu, ref)


@pytest.mark.parametrize("window", [(380, 250, 420, 280), (100, 400, 140, 430), (700, 100, 740, 130),
                                   (560, 420, 600, 450)])
def test_final_c2_windows(cuda, window):
    """C2: buildFinal(240) without models, 800x600, 16 spp, depth 4, brdf 2, DoF 0.2 —
    Cook-Torrance doors, glossy floor/cylinder, 4 area lights; pixel windows."""
    g = dt.globals_default()
    g.use_model = 0
    built = dt.build_scene("final", 240, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth, g.brdf_samples = 800, 600, 16, 4, 2
    x0, y0, x1, y1 = window
    tile = dt.tiles(x0=x0, y0=y0, x1=x1, y1=y1)
    gpu, st = _render_gpu(built, g, 240, tile)
    ref, rst = oracle.render(built, g, 240, tile)
    m = np.zeros((600, 800), dtype=bool)
    m[600 - y1:600 - y0, x0:x1] = True
    m = np.repeat(m.reshape(-1), 3)
    assert st.pixels == (x1 - x0) * (y1 - y0)
    assert_parity("final C2 %s" % (window,), gpu[m], ref[m])


def test_final_models_window(cuda):
    """buildFinal(480) with use_model=true (substitute column/bust meshes, tools/gen_models.py):
    ~2400 UV-mapped triangles, textured Oren-Nayar marble, roughness from the map; the window
    covers a column and its bust."""
    g = dt.globals_default()
    g.use_model = 1
    built = dt.build_scene("final", 480, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth, g.brdf_samples = 320, 180, 16, 4, 2
    x0, y0, x1, y1 = 24, 20, 72, 100
    tile = dt.tiles(x0=x0, y0=y0, x1=x1, y1=y1)
    gpu, st = _render_gpu(built, g, 480, tile)
    ref, _ = oracle.render(built, g, 480, tile)
    m = np.zeros((180, 320), dtype=bool)
    m[180 - y1:180 - y0, x0:x1] = True
    m = np.repeat(m.reshape(-1), 3)
    assert st.tex_fetches > 0
    assert_parity("final models window", gpu[m], ref[m])


@pytest.mark.parametrize("n", [150, 210])
def test_final_c5_tunnel_motion_blur(cuda, n):
    """C5 animation frames buildFinal(n*8) (scene.h:605-1100): the ad tunnel (substitute ./ads
    frames, generateTrianglePrismMesh) with every "rectangle" in motion. Frame 1200 blurs with
    the linear shift, frame 1680 (>= frame_blur) with the cubic acceleration term; both shift
    the tunnel rectangles and bump the BVH leaves (general traversal path)."""
    g = dt.globals_default()
    g.use_model = 0
    built = dt.build_scene("final", n * 8, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth = 320, 180, 4, 3
    x0, y0, x1, y1 = 128, 60, 192, 108
    tile = dt.tiles(x0=x0, y0=y0, x1=x1, y1=y1)
    gpu, st = _render_gpu(built, g, n * 8, tile)
    ref, rst = oracle.render(built, g, n * 8, tile)
    m = np.zeros((180, 320), dtype=bool)
    m[180 - y1:180 - y0, x0:x1] = True
    m = np.repeat(m.reshape(-1), 3)
    assert st.rays > st.samples and st.rays == rst.rays   # blur re-traces, same count as the oracle
    assert_parity("final C5 frame %d" % (n * 8), gpu[m], ref[m])


@pytest.mark.parametrize("spp,res,build", [(4, (160, 90), "dt_trace_kernel_tunnel"),
                                           (64, (48, 27), "dt_trace_kernel_w5_tunnel")])
def test_called_sky_march_tunnel_builds(cuda, spp, res, build):
    """The tunnel and blur builds march the sky in a called function (dt_kernels.hip DT_SKY_CALL,
    csrc/Makefile SKYCALL). Under -disable-machine-cse that function returned wrong colours (its
    1.5 constants encoded as 0): a whole C5 tunnel frame with sky pixels, n = 180
    (buildFinal(1440), the C5 blur share's frames), on the 4-wave and the 5-wave build, against the
    oracle."""
    g = dt.globals_default()
    g.use_model = 0
    built = dt.build_scene("final", 1440, g)
    g.xRes, g.yRes = res
    g.antialias_samples, g.max_depth = spp, 3
    assert dt.trace_build(built, g, 1440)[0] == build
    gpu, st = _render_gpu(built, g, 1440, dt.tiles())
    ref, rst = oracle.render(built, g, 1440, dt.tiles())
    # (the two count the sky differently: the device once per pixel it marches, the oracle per sample)
    assert st.sky_pixels > 0 and rst.sky_pixels > 0 and st.rays == rst.rays
    assert_parity("C5 frame 1440 sky, %s" % build, gpu, ref)


@pytest.mark.parametrize("defer", ["1", "0"])
def test_final_c5_cloud_frame(cuda, monkeypatch, defer):
    """C5 cloud frame buildFinal(2000) (n = 250 >= 244): the builder forces 1 spp and no aperture
    (scene.h:795-796); 64 pixels per wave. The missed pixels' sky is marched per lane by
    dt_sky_miss_kernel (default), or cooperatively by the wave (DT_SKY_DEFER=0)."""
    monkeypatch.setenv("DT_SKY_DEFER", defer)
    g = dt.globals_default()
    g.use_model = 0
    built = dt.build_scene("final", 2000, g)
    assert g.antialias_samples == 1
    g.xRes, g.yRes = 320, 180
    x0, y0, x1, y1 = 128, 60, 176, 92
    tile = dt.tiles(x0=x0, y0=y0, x1=x1, y1=y1)
    gpu, st = _render_gpu(built, g, 2000, tile)
    ref, rst = oracle.render(built, g, 2000, tile)
    m = np.zeros((180, 320), dtype=bool)
    m[180 - y1:180 - y0, x0:x1] = True
    m = np.repeat(m.reshape(-1), 3)
    assert st.samples == st.pixels == (x1 - x0) * (y1 - y0) and st.sky_pixels > 0
    assert_parity("final C5 cloud frame 2000", gpu[m], ref[m])


def test_final_c3_window(cuda):
    """C3 settings (1920x1080, 64 spp, depth 8) on a window around the window/sky region."""
    g = dt.globals_default()
    g.use_model = 0
    built = dt.build_scene("final", 240, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth, g.brdf_samples = 1920, 1080, 64, 8, 2
    tile = dt.tiles(x0=900, y0=500, x1=916, y1=512)
    gpu, st = _render_gpu(built, g, 240, tile)
    ref, _ = oracle.render(built, g, 240, tile)
    m = np.zeros((1080, 1920), dtype=bool)
    m[1080 - 512:1080 - 500, 900:916] = True
    m = np.repeat(m.reshape(-1), 3)
    assert_parity("final C3 window", gpu[m], ref[m])


def test_slab_layout_matches_image(cuda):
    """tile-split + slab output + unpack reproduces the single-GPU image bit for bit."""
    g = dt.globals_default()
    g.use_model = 0
    built = dt.build_scene("final", 240, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth = 200, 120, 4, 3
    scene = dt.Scene(built, g)
    full = torch.zeros(3 * g.xRes * g.yRes, dtype=torch.float32, device="cuda")
    dt.render(scene, g, 240, full, dt.tiles(tile_w=16, tile_h=16))
    world = 3
    base = dt.tiles(tile_w=16, tile_h=16, world=world, layout=dt.DT_OUT_SLAB)
    per = dt.slab_floats_max(g, base)
    slabs = torch.zeros(world * per, dtype=torch.float32, device="cuda")
    for r in range(world):
        t = dt.tiles(tile_w=16, tile_h=16, rank=r, world=world, layout=dt.DT_OUT_SLAB)
        dt.render(scene, g, 240, slabs[r * per:(r + 1) * per], t)
    img = torch.zeros_like(full)
    dt.unpack_slabs(g, base, world, slabs, img)
    torch.cuda.synchronize()
    log_equal("slab layout (3 ranks) vs image layout", img.cpu().numpy(), full.cpu().numpy())
    scene.close()


def test_fast_tree_gathers_the_reference_leaves(cuda, monkeypatch):
    """The alternative traversal tree (host_fasttree.cpp, same leaves under SAH inner nodes) must
    give the reference-tree image bit for bit (monotone slab test + rank tie-break), whichever
    walks use it: DT_FAST_TREE=0 (none), c (closest hit), s (shadow), 1 (both, the default).
    C2 window with glossy floor, doors and area-light shadows."""
    g = dt.globals_default()
    g.use_model = 0
    built = dt.build_scene("final", 240, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth, g.brdf_samples = 800, 600, 16, 4, 2
    tile = dt.tiles(x0=380, y0=250, x1=420, y1=280)
    monkeypatch.setenv("DT_FAST_TREE", "0")
    ref_img, _ = _render_gpu(built, g, 240, tile)
    for mode in ("c", "s", "1"):
        monkeypatch.setenv("DT_FAST_TREE", mode)
        fast_img, _ = _render_gpu(built, g, 240, tile)
        log_equal("fast tree DT_FAST_TREE=%s vs reference tree" % mode, fast_img, ref_img)


def test_shadow_grid_matches_tree_walks(cuda, monkeypatch):
    """The shadow grid (host_shadowgrid.cpp: per-light candidate-occluder lists per cell) must
    answer every shadow ray as the tree walk does: C3-like window (64 spp, depth 8, DoF, glossy
    floor, 4 area lights + the window point light) with and without it, bit for bit."""
    g = dt.globals_default()
    g.use_model = 0
    built = dt.build_scene("final", 240, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth, g.brdf_samples = 1920, 1080, 64, 8, 2
    tile = dt.tiles(x0=900, y0=500, x1=964, y1=548)
    monkeypatch.setenv("DT_SHADOW_GRID", "0")
    ref_img, ref_st = _render_gpu(built, g, 240, tile)
    # grid size/reach, the block-test sizes of the host build (tests/test_host.py checks the lists
    # themselves) and the likely-occluder list order (any-hit: the image must not change)
    variants = [{"DT_SG_CELLS": "32768", "DT_SG_REACH": "0.5"}, {"DT_SG_CELLS": "4096", "DT_SG_REACH": "2"}]
    variants += [{"DT_SG_BLOCK": b, "DT_SG_ORDER": o} for b in ("0", "4x2", "32x8") for o in ("0", "1")]
    variants += [{"DT_SG_ORDER": "1"}, {"DT_SG_HULL": "0"}, {"DT_SG_HULL": "2"}, {"DT_SG_UMBRA": "0"}, {"DT_SG_UMBRA": "2"}]
    for env in variants:
        for k in ("DT_SG_CELLS", "DT_SG_REACH", "DT_SG_BLOCK", "DT_SG_ORDER", "DT_SG_HULL", "DT_SG_UMBRA"):
            monkeypatch.delenv(k, raising=False)
        monkeypatch.setenv("DT_SHADOW_GRID", "1")
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        img, st = _render_gpu(built, g, 240, tile)
        assert st.shadow_rays == ref_st.shadow_rays, env
        log_equal("shadow grid %s vs tree walks" % env, img, ref_img)


@pytest.mark.parametrize("frame", [1200, 1680])
def test_shadow_grid_hull_culling_tunnel(cuda, monkeypatch, frame):
    """Hull culling (host_shadowgrid.cpp) drops the tunnel's slanted panels from the cells whose
    segments to the light cannot reach them: C5 tunnel windows (ads in motion, blur passes on the
    padded lists) must match tree walks bit for bit with it off, on blocks, and on blocks + cells."""
    g = dt.globals_default()
    g.use_model = 0
    built = dt.build_scene("final", frame, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth = 480, 270, 16, 10
    tile = dt.tiles(x0=160, y0=80, x1=320, y1=176)
    for k in ("DT_SG_CELLS", "DT_SG_REACH", "DT_SG_BLOCK", "DT_SG_ORDER", "DT_SG_HULL"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("DT_SHADOW_GRID", "0")
    ref_img, ref_st = _render_gpu(built, g, frame, tile)
    monkeypatch.setenv("DT_SHADOW_GRID", "1")
    for mode in ("0", "1", "2"):
        monkeypatch.setenv("DT_SG_HULL", mode)
        img, st = _render_gpu(built, g, frame, tile)
        assert st.shadow_rays == ref_st.shadow_rays, mode
        log_equal("frame %d DT_SG_HULL=%s vs tree walks" % (frame, mode), img, ref_img)


@pytest.mark.parametrize("frame", [1680, 1920])
def test_shadow_grid_pass0_lists(cuda, monkeypatch, frame):
    """Large blur shifts: an unpadded second grid serves the pass-0 rays while the blur passes
    keep the padded lists or walk (host_accel.cpp, DT_SG_PASS0). Tunnel windows at frames 1680
    (shift <= 5) and 1920 (<= 81) with it forced on and off must match tree walks bit for bit."""
    g = dt.globals_default()
    g.use_model = 0
    built = dt.build_scene("final", frame, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth = 480, 270, 16, 10
    tile = dt.tiles(x0=160, y0=80, x1=320, y1=176)
    for k in ("DT_SG_CELLS", "DT_SG_REACH", "DT_SG_BLOCK", "DT_SG_ORDER", "DT_SG_HULL", "DT_SG_PASS0"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("DT_SHADOW_GRID", "0")
    ref_img, ref_st = _render_gpu(built, g, frame, tile)
    monkeypatch.setenv("DT_SHADOW_GRID", "1")
    for mode in ("0", "1"):
        monkeypatch.setenv("DT_SG_PASS0", mode)
        img, st = _render_gpu(built, g, frame, tile)
        assert st.shadow_rays == ref_st.shadow_rays, mode
        log_equal("frame %d DT_SG_PASS0=%s vs tree walks" % (frame, mode), img, ref_img)


def test_scene_prepare_then_upload(cuda):
    """dt_scene_prepare (host only) + dt_scene_upload, or a render of a prepared scene (which
    uploads it first), give dt_scene_create's image: C2 window."""
    g = dt.globals_default()
    g.use_model = 0
    built = dt.build_scene("final", 240, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth, g.brdf_samples = 800, 600, 16, 4, 2
    tile = dt.tiles(x0=380, y0=250, x1=420, y1=280)
    ref, ref_st = _render_gpu(built, g, 240, tile)
    for explicit in (True, False):
        scene = dt.Scene(built, g, upload=False)
        if explicit:
            scene.upload()
        out = torch.zeros(3 * g.xRes * g.yRes, dtype=torch.float32, device="cuda")
        st = dt.render(scene, g, 240, out, tile)
        scene.close()
        assert st.rays == ref_st.rays
        log_equal("prepared scene (explicit upload %s) vs dt_scene_create" % explicit, out.cpu().numpy(), ref)


PL_CASES = [  # (name, builder, frame, models, W, H, spp, depth, window)
    ("c3", "final", 240, 0, 1920, 1080, 64, 8, (880, 480, 1008, 560)),
    ("c4-models", "final", 240, 1, 1920, 1080, 16, 3, (1200, 500, 1296, 580)),
    ("c1-dof", "spheres", 0, 0, 256, 256, 16, 2, (64, 64, 192, 192)),
    ("c5-tunnel", "final", 1200, 0, 320, 180, 16, 3, (96, 40, 224, 136)),
    ("c5-tunnel-1680", "final", 1680, 0, 320, 180, 16, 3, (96, 40, 224, 136)),
    ("c2-full", "final", 240, 0, 200, 150, 4, 4, (0, 0, 200, 150)),
]


@pytest.mark.parametrize("case", PL_CASES, ids=[c[0] for c in PL_CASES])
def test_primary_lists_match_tree_walks(cuda, monkeypatch, case):
    """Primary rays over their pixel block's candidate leaves (host_primlists.cpp: camera-space
    frustum of the block's DoF rays, leaves sorted by reach, early exit) must give the image of
    fast-tree walks bit for bit, for any block size (a ragged last block included), super-block
    size, with and without hull culling, and with the blur passes (C5 tunnel frames) on the bump
    tree's lists or on bump-tree walks."""
    name, builder, frame, models, W, H, spp, depth, win = case
    g = dt.globals_default()
    g.use_model = models
    built = dt.build_scene(builder, frame, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth = W, H, spp, depth
    tile = dt.tiles(x0=win[0], y0=win[1], x1=win[2], y1=win[3])
    monkeypatch.setenv("DT_PRIM_LISTS", "0")
    ref_img, ref_st = _render_gpu(built, g, frame, tile)
    monkeypatch.delenv("DT_PRIM_LISTS")
    variants = [{"DT_PL_BLOCK": b} for b in ("8", "3", "16")]
    variants += [{"DT_PL_HULL": "0"}, {"DT_PL_SUPER": "1"}, {"DT_PL_SUPER": "3", "DT_PL_BLOCK": "5"}, {"DT_PL_BUMP": "0"}]
    for env in variants:
        for k in ("DT_PL_BLOCK", "DT_PL_HULL", "DT_PL_SUPER", "DT_PL_BUMP"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        img, st = _render_gpu(built, g, frame, tile)
        assert st.rays == ref_st.rays and st.shadow_rays == ref_st.shadow_rays, env
        log_equal("primary lists %s %s vs fast-tree walks" % (name, env), img, ref_img)


@pytest.mark.parametrize("n", [150, 210, 240])
def test_bump_tree_matches_reference_walks(cuda, monkeypatch, n):
    """Motion-blur passes on the bump tree (host_fasttree.cpp: padded leaves, exact per-leaf
    bumped gather with the ancestor chain) and on the blur-padded shadow-grid lists must give the
    image of reference-tree walks bit for bit. Frame 1200 shifts by < 0.04, frame 1680 by up to 5
    (bumped leaf boxes outgrow their parents: the ancestor-chain test). DT_BUMP_PAD_SCALE=0.5
    pads for half the largest shift, so lanes beyond it send their waves to the reference walk.
    Children order (DT_EYE_ORDER) must not matter either, nor the planar leaves' one-sided padding
    (DT_BUMP_UP=0: +-pad on every leaf). Frame 1920 shifts by up to 81."""
    g = dt.globals_default()
    g.use_model = 0
    built = dt.build_scene("final", n * 8, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth = 320, 180, 16, 3
    tile = dt.tiles(x0=96, y0=40, x1=224, y1=136)
    monkeypatch.setenv("DT_BUMP_TREE", "0")
    monkeypatch.setenv("DT_SHADOW_GRID", "0")
    monkeypatch.setenv("DT_FAST_TREE", "0")
    ref_img, ref_st = _render_gpu(built, g, n * 8, tile)
    assert ref_st.rays > ref_st.samples   # blur passes ran
    for env in ({}, {"DT_BUMP_PAD_SCALE": "0.5"}, {"DT_EYE_ORDER": "0"}, {"DT_BUMP_UP": "0"}):
        for k in ("DT_BUMP_TREE", "DT_SHADOW_GRID", "DT_FAST_TREE", "DT_BUMP_PAD_SCALE", "DT_EYE_ORDER", "DT_BUMP_UP"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        img, st = _render_gpu(built, g, n * 8, tile)
        assert st.rays == ref_st.rays and st.shadow_rays == ref_st.shadow_rays, env
        log_equal("bump tree frame %d %s vs reference-tree walks" % (n * 8, env), img, ref_img)


def _feature_scene():
    """A synthetic scene for the shading paths the shipped builders never use: a glass sphere
    (refraction + Fresnel, Q5), a steel mirror sphere, an Oren-Nayar sphere, a raw triangle, a
    plain Checkerboard floor (geometry.cpp:2248-2341), a sphere light with a bounding axis
    (rejection sampling, Q11), a rectangle light and a point light. Built through the ABI's
    descriptor structs, as a caller of dt_scene_create would."""
    import ctypes
    from distraytracer_amd import _lib
    shapes = []

    def shape(t, **kw):
        s = _lib.ShapeDesc()
        s.type = t
        s.tex_frame = -1
        for k, v in kw.items():
            if k == "v":
                for i, p in enumerate(v):
                    for a in range(3):
                        s.v[i][a] = p[a]
            elif isinstance(v, (list, tuple)):
                for a in range(len(v)):
                    getattr(s, k)[a] = v[a]
            else:
                setattr(s, k, v)
        shapes.append(s)
        return len(shapes) - 1

    A, B, C, D = (-5, 0, 5), (5, 0, 5), (5, 0, -5), (-5, 0, -5)
    shape(6, v=[A, B, C, D], color=(0.5, 0.5, 0.5), color1=(0.9, 0.9, 0.9), color2=(0.1, 0.1, 0.3), S=1.0,
          length=10.0, width=10.0, center=(0, 0, 0))
    shape(1, v=[(0.5, 1.0, 0.0)], radius=0.6, color=(0.9, 0.9, 1.0), material=1, center=(0.5, 1.0, 0.0))
    shape(1, v=[(-1.2, 0.7, 0.5)], radius=0.5, color=(0.8, 0.8, 0.8), material=2, center=(-1.2, 0.7, 0.5))
    shape(1, v=[(1.8, 0.5, -0.8)], radius=0.5, color=(0.9, 0.4, 0.2), model=1, roughness=0.3,
          center=(1.8, 0.5, -0.8))
    shape(3, v=[(-2, 0, -2), (-1, 2, -2), (0, 0, -2)], color=(0.2, 0.8, 0.3), model=3, center=(-1, 2 / 3, -2))
    sl = shape(1, v=[(0, 3.5, 1)], radius=0.3, color=(1, 1, 0.9), emit=1, flags=1, center=(0, 3.5, 1))
    ra, rb, rc, rd = (-1, 4, -1), (1, 4, -1), (1, 4, 1), (-1, 4, 1)
    rl = shape(4, v=[ra, rb, rc, rd], color=(0.8, 0.8, 0.8), emit=2, flags=1, length=1.0, width=1.0,
               center=(0, 4, 0))
    lights = (_lib.LightDesc * 3)()
    lights[0].type, lights[0].shape_index, lights[0].radius = 2, sl, 0.3
    for a in range(3):
        lights[0].center[a] = (0, 3.5, 1)[a]
        lights[0].color[a] = (1, 1, 0.9)[a]
        lights[0].baxis[a] = (0, -1, 0)[a]
        lights[1].center[a] = (0, 4, 0)[a]
        lights[1].color[a] = 0.8
        lights[1].A[a], lights[1].B[a], lights[1].D[a] = ra[a], rb[a], rd[a]
        lights[2].center[a] = (3, 3, 3)[a]
        lights[2].color[a] = 0.6
    lights[1].type, lights[1].shape_index = 3, rl
    lights[2].type, lights[2].shape_index = 1, -1
    arr = (_lib.ShapeDesc * len(shapes))(*shapes)
    desc = _lib.SceneDesc(len(shapes), 3, 0, 0, arr, lights, None)
    g = dt.globals_default()
    g.use_model = 0
    g.eye[0], g.eye[1], g.eye[2] = -4.0, 2.5, 4.0
    g.lookingAt[0], g.lookingAt[1], g.lookingAt[2] = 0.3, 0.8, -0.2
    g.xRes, g.yRes, g.antialias_samples, g.max_depth, g.brdf_samples = 160, 120, 9, 5, 2
    g.aperture, g.focal_length = 0.1, 6.0
    keep = (arr, lights)
    return desc, g, keep


def test_feature_scene_glass_spherelight_checkerboard(cuda):
    desc, g, keep = _feature_scene()
    import ctypes
    h = ctypes.c_void_p()
    dt.check(dt.lib.dt_scene_create(ctypes.byref(desc), ctypes.byref(g), ctypes.byref(h)), "dt_scene_create")
    out = torch.zeros(3 * g.xRes * g.yRes, dtype=torch.float32, device="cuda")
    st = _lib_stats()
    dt.check(dt.lib.dt_render(h, ctypes.byref(g), 0, None, ctypes.c_void_p(out.data_ptr()), 1, None,
                              ctypes.byref(st)), "dt_render")
    dt.lib.dt_scene_destroy(h)
    gpu = out.cpu().numpy()
    ref, rst = oracle.render(desc, g, 0, dt.tiles())
    assert st.rays == rst.rays and st.shadow_rays == rst.shadow_rays
    assert st.rays > st.samples    # reflection and refraction children ran
    # Q25: a glancing ray entering the glass sphere takes cos_phi = sqrt(<0) (the outgoing-ray
    # formula, render_final_project.cpp:619) and its whole pixel goes NaN in the reference too.
    # The NaN pixels must coincide (nan_ok: this scene is built to produce them); every other
    # channel within 1e-4.
    assert rst.nan_pixels > 0 and st.nan_pixels == rst.nan_pixels
    assert_parity("feature scene", gpu, ref, nan_ok=True)


def _lib_stats():
    from distraytracer_amd import _lib
    return _lib.Stats()


def _shape(shapes, t, **kw):
    from distraytracer_amd import _lib
    s = _lib.ShapeDesc()
    s.type = t
    s.tex_frame = -1
    for k, v in kw.items():
        if k == "v":
            for i, p in enumerate(v):
                for a in range(3):
                    s.v[i][a] = p[a]
        elif isinstance(v, (list, tuple)):
            for a in range(len(v)):
                getattr(s, k)[a] = v[a]
        else:
            setattr(s, k, v)
    shapes.append(s)
    return len(shapes) - 1


def _rpc_scene():
    """RectPrismWithCylinder (geometry.cpp:1467-1821) in every role the shipped prismcyl scene
    never gives it: an axis-aligned wall with a hole (textured front face: RectPrism::getUV), a
    tilted box with two holes (the box test uses the vertices' AABB), a steel mirror sphere inside
    the first hole (its reflected rays start between the cap planes: the hole-body branch, boxes
    entered from inside), a glass sphere, a floor, a back wall seen through the hole, a point light
    behind the wall (shadow rays through the hole and past the light: the box test ignores t_max),
    a point light in front and a rectangle light."""
    import math
    from distraytracer_amd import _lib
    shapes, holes = [], []

    def box(c, hx, hy, hz, rot):
        """8 vertices A..H of a box rotated by `rot` about y: A B C D the x = -hx face, E..H = +x"""
        cr, sr = math.cos(rot), math.sin(rot)
        pts = [(-hx, -hy, -hz), (-hx, -hy, hz), (-hx, hy, hz), (-hx, hy, -hz)]
        pts += [(hx, p[1], p[2]) for p in pts]
        return [(c[0] + p[0] * cr + p[2] * sr, c[1] + p[1], c[2] - p[0] * sr + p[2] * cr) for p in pts]

    def cyl(c1, c2, r, col):
        h = _lib.ShapeDesc()
        h.type, h.radius, h.tex_frame = 2, r, -1
        for a in range(3):
            h.v[0][a], h.v[1][a], h.color[a] = c1[a], c2[a], col[a]
        holes.append(h)

    wall = box((0.5, 0, 0), 0.5, 2, 2, 0.0)
    _shape(shapes, 9, v=wall, color=(0.8, 0.2, 0.2), center=(0.5, 0, 0), hole_first=0, n_holes=1,
           flags=4, tex_frame=0)
    cyl((0, 0, 0), (1, 0, 0), 1.0, (0.2, 0.2, 0.9))
    tilt = box((2.2, -1.2, 2.6), 0.4, 0.6, 0.7, 0.5)
    _shape(shapes, 9, v=tilt, color=(0.2, 0.8, 0.3), center=(2.2, -1.2, 2.6), hole_first=1, n_holes=2)
    cyl(tilt[0], tilt[4], 0.25, (0.9, 0.9, 0.1))
    cyl(tilt[2], tilt[6], 0.2, (0.1, 0.9, 0.9))
    _shape(shapes, 1, v=[(0.5, 0.1, -0.2)], radius=0.45, color=(0.9, 0.9, 0.9), material=2, center=(0.5, 0.1, -0.2))
    _shape(shapes, 1, v=[(-1.6, -0.9, 1.4)], radius=0.5, color=(0.9, 0.9, 1.0), material=1, center=(-1.6, -0.9, 1.4))
    _shape(shapes, 6, v=[(-8, -2.5, 6), (8, -2.5, 6), (8, -2.5, -6), (-8, -2.5, -6)], color=(0.5, 0.5, 0.5),
           color1=(0.9, 0.9, 0.9), color2=(0.2, 0.2, 0.4), S=1.0, length=16.0, width=12.0, center=(0, -2.5, 0))
    _shape(shapes, 4, v=[(6, -3, -6), (6, -3, 6), (6, 4, 6), (6, 4, -6)], color=(0.3, 0.6, 0.9), length=12.0,
           width=7.0, center=(6, 0.5, 0))
    ra, rb, rc, rd = (-2, 5, -1), (0, 5, -1), (0, 5, 1), (-2, 5, 1)
    rl = _shape(shapes, 4, v=[ra, rb, rc, rd], color=(0.8, 0.8, 0.8), emit=2, flags=1, length=2.0, width=2.0,
                center=(-1, 5, 0))
    lights = (_lib.LightDesc * 3)()
    for a in range(3):
        lights[0].center[a] = (4.0, 0.2, 0.1)[a]
        lights[0].color[a] = 0.9
        lights[1].center[a] = (-4.0, 3.0, 3.0)[a]
        lights[1].color[a] = 0.5
        lights[2].center[a] = (-1, 5, 0)[a]
        lights[2].color[a] = 0.7
        lights[2].A[a], lights[2].B[a], lights[2].D[a] = ra[a], rb[a], rd[a]
    lights[0].type, lights[0].shape_index = 1, -1
    lights[1].type, lights[1].shape_index = 1, -1
    lights[2].type, lights[2].shape_index = 3, rl
    tex = bytes((i * 37 + 11) % 256 for i in range(8 * 8 * 3))
    texbuf = (ctypes.c_uint8 * len(tex)).from_buffer_copy(tex)
    textures = (_lib.TextureDesc * 1)()
    textures[0].width, textures[0].height, textures[0].channels = 8, 8, 3
    textures[0].pixels = ctypes.cast(texbuf, ctypes.POINTER(ctypes.c_uint8))
    arr = (_lib.ShapeDesc * len(shapes))(*shapes)
    harr = (_lib.ShapeDesc * len(holes))(*holes)
    desc = _lib.SceneDesc(len(shapes), 3, 1, 0, arr, lights, textures, len(holes), 0, harr)
    g = dt.globals_default()
    g.use_model = 0
    g.eye[0], g.eye[1], g.eye[2] = -5.0, 1.2, 2.8
    g.lookingAt[0], g.lookingAt[1], g.lookingAt[2] = 0.6, -0.2, 0.3
    g.xRes, g.yRes, g.antialias_samples, g.max_depth, g.brdf_samples = 200, 150, 9, 5, 2
    g.aperture, g.focal_length = 0.08, 6.0
    return desc, g, (arr, harr, lights, textures, texbuf)


def _render_desc(desc, g, frame=0):
    h = ctypes.c_void_p()
    dt.check(dt.lib.dt_scene_create(ctypes.byref(desc), ctypes.byref(g), ctypes.byref(h)), "dt_scene_create")
    out = torch.zeros(3 * g.xRes * g.yRes, dtype=torch.float32, device="cuda")
    st = _lib_stats()
    dt.check(dt.lib.dt_render(h, ctypes.byref(g), frame, None, ctypes.c_void_p(out.data_ptr()), 1, None,
                              ctypes.byref(st)), "dt_render")
    dt.lib.dt_scene_destroy(h)
    return out.cpu().numpy(), st


def test_rectprism_cylinder_scene(cuda):
    """RectPrismWithCylinder on the device (dt_trace_kernel_rpc) against the oracle: every hit,
    shadow, normal and texel of the scene above, bit for bit, the same rays and shadow rays and
    the same count of getNorm's off-prism points (the reference throws there)."""
    desc, g, keep = _rpc_scene()
    gpu, st = _render_desc(desc, g)
    ref, rst = oracle.render(desc, g, 0, dt.tiles())
    print("rpc scene: rays %d shadow %d prism_norm_fallback %d/%d uv %d tex %d" % (
        st.rays, st.shadow_rays, st.prism_norm_fallback, rst.prism_norm_fallback, st.uv_out_of_range, st.tex_fetches))
    # The wall's texture: RectPrism::getUV is valid only where |(ad x dc).p| <= 1e-5, elsewhere type 0
    # aborts the shading (Q8) at the first unoccluded light. The device skips every shadow ray of
    # such a point up front (it cannot change the colour), the oracle traces them as the reference
    # does: fewer shadow rays on the device, never more.
    assert st.rays == rst.rays and st.shadow_rays <= rst.shadow_rays
    assert st.prism_norm_fallback == rst.prism_norm_fallback > 0   # hole-body hits (the mirror's rays)
    assert st.rays > st.samples and st.nan_pixels == rst.nan_pixels
    # NaN pixels, if the glass sphere makes any (Q25), must coincide
    assert_parity("RectPrismWithCylinder scene", gpu, ref, nan_ok=True)


@pytest.mark.parametrize("frame,oblique", [(0, False), (7, False), (0, True)])
def test_prismcyl_mode(cuda, frame, oblique):
    """The reference's `./render prismcyl <n>` mode (render_final_project.cpp:1711-1723):
    BuildScenePrismCylinder(n) at 640x480 with the globals' defaults (antialias 10 -> 9 spp,
    depth 10, DoF); frame 0's camera looks straight down the hole's axis (a black frame, see
    tests/test_host.py), so an oblique eye is rendered too."""
    g = dt.globals_default()
    built = dt.build_scene("prismcyl", frame, g)
    g.xRes, g.yRes = 640, 480
    if oblique:
        g.eye[0], g.eye[1], g.eye[2] = -5.0, 1.3, 2.2
    gpu, st = _render_gpu(built, g, frame, dt.tiles())
    ref, rst = oracle.render(built, g, frame, dt.tiles())
    assert st.rays == rst.rays and st.shadow_rays == rst.shadow_rays
    assert_parity("prismcyl frame %d%s" % (frame, " oblique" if oblique else ""), gpu, ref)
    if oblique:
        assert ref.max() > 0
