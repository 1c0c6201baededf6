"""DFS work sharing inside a wave (dt_kernels.hip DT_DONATE, dt_trace_kernel_dn; DT_DONATE=1).

Idle lanes run whole pending subtrees of other lanes' rayColor trees and the owners replay the
recorded colours in the reference's accumulation order, so the image must be bit-identical to the
product kernel's (and the oracle's) with the same rays traced. The cases are the ones that donate:
a C3 share of the 8-way tile split (the deep glossy column), C5's room-to-tunnel transition frame
(8 rays per sample), a motion-blur frame (in_motion, Q6, is the last rayColor's: kept as the
value of the largest pre-order path, whoever ran that node) and C2's full frame.

Also the other per-launch kernel choice: still frames' kernels against their motion-blur builds.
"""
import numpy as np
import pytest
import torch

import distraytracer_amd as dt
import oracle
from parity_check import assert_parity, log_equal
from test_gpu_configs import _globals

pytestmark = pytest.mark.gpu


def _render(g, built, frame, tile, donate, monkeypatch, via_env=False):
    """donate through dt_scene_set_kernel (the scene's own choice), or via_env: DT_KERNEL_AUTO and
    the DT_DONATE environment variable"""
    monkeypatch.setenv("DT_DONATE", "1" if donate and via_env else "0")
    scene = dt.Scene(built, g)
    if not via_env:
        scene.set_kernel(dt.DT_KERNEL_DONATE if donate else dt.DT_KERNEL_PRODUCT)
    n = dt.slab_floats(g, tile) if tile.layout == dt.DT_OUT_SLAB else 3 * g.xRes * g.yRes
    out = torch.zeros(n, dtype=torch.float32, device="cuda")
    st = dt.render(scene, g, frame, out, tile)
    scene.close()
    return out.cpu().numpy(), st


CASES = [  # (id, builder args, frame, tile world, oracle check, donates)
    ("c3_rank0_of_8", ("final", 240, 0, 1920, 1080, 64, 8), 240, 8, True, True),
    ("c5_1088_transition", ("final", 1088, 0, 3840, 2160, 64, 10), 1088, 512, True, True),
    ("c5_1920_blur", ("final", 1920, 0, 3840, 2160, 64, 10), 1920, 512, True, False),
    ("c2_full", ("final", 240, 0, 800, 600, 16, 4), 240, 1, False, False),
]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_donate_bit_identical(cuda, monkeypatch, case):
    label, args, frame, world, check_oracle, donates = case
    g, built = _globals(*args)
    tile = dt.tiles(rank=0, world=world, layout=dt.DT_OUT_SLAB) if world > 1 else dt.tiles()
    base, st0 = _render(g, built, frame, tile, False, monkeypatch)
    img, st = _render(g, built, frame, tile, True, monkeypatch)
    print("%s: donations=%d overflow=%d kernel %.2f -> %.2f ms" % (label, st.donations, st.donate_overflow,
                                                                 st0.trace_kernel_ms, st.trace_kernel_ms))
    assert st0.donations == 0
    assert st.donate_overflow == 0 and st.stack_overflows == 0
    assert st.rays == st0.rays and st.shadow_rays == st0.shadow_rays and st.samples == st0.samples
    log_equal("%s work-sharing kernel vs product kernel (bits)" % label, img.view(np.uint32), base.view(np.uint32))
    if donates:
        assert st.donations > 0   # the deep cascades did donate
        img_env, st_env = _render(g, built, frame, tile, True, monkeypatch, via_env=True)
        assert st_env.donations > 0
        log_equal("%s work-sharing kernel via DT_DONATE (bits)" % label, img_env.view(np.uint32), base.view(np.uint32))
    if check_oracle:
        ref, rst = oracle.render(built, g, frame, tile, out=np.zeros(img.size, dtype=np.float32))
        assert st.rays == rst.rays
        assert_parity("%s work-sharing kernel vs oracle" % label, img, ref)


def test_set_kernel_rejects_unknown_choice(cuda):
    g, built = _globals("final", 240, 0, 64, 32, 4, 2)
    scene = dt.Scene(built, g)
    for k in (dt.DT_KERNEL_AUTO, dt.DT_KERNEL_PRODUCT, dt.DT_KERNEL_DONATE):
        scene.set_kernel(k)
    assert dt.lib.dt_scene_set_kernel(scene.handle, 7) == -1
    scene.close()


BLUR_CASES = [  # (id, builder args, frame, tile world): still frames, 5-wave (64 spp) and 4-wave (16 spp)
    ("c3_1of64_w5", ("final", 240, 0, 1920, 1080, 64, 8), 240, 64),
    ("c2_full_w4", ("final", 240, 0, 800, 600, 16, 4), 240, 1),
    ("c5_room_480_1of512_w5", ("final", 480, 0, 3840, 2160, 64, 10), 480, 512),
    ("c4_models_1of256_w5_full", ("final", 240, 1, 1920, 1080, 256, 8), 240, 256),
]


@pytest.mark.parametrize("case", BLUR_CASES, ids=[c[0] for c in BLUR_CASES])
def test_still_kernels_match_blur_builds(cuda, monkeypatch, case):
    """Frames below frame_prism take the product kernels built without the motion-blur shift paths
    (dt_kernels.hip DT_NOSHIFT): the room builds for scenes within DT_ROOM_FEATURES, the *_full
    builds otherwise (C4's meshes: triangles, Oren-Nayar). DT_BLUR_KERNEL=1 renders them with the
    *_blur builds, which every later frame takes. Same rays, same bits."""
    label, args, frame, world = case
    g, built = _globals(*args)
    tile = dt.tiles(rank=0, world=world, layout=dt.DT_OUT_SLAB) if world > 1 else dt.tiles()
    monkeypatch.setenv("DT_BLUR_KERNEL", "0")
    still, st0 = _render(g, built, frame, tile, False, monkeypatch)
    monkeypatch.setenv("DT_BLUR_KERNEL", "1")
    blur, st1 = _render(g, built, frame, tile, False, monkeypatch)
    assert st0.rays == st1.rays and st0.shadow_rays == st1.shadow_rays
    log_equal("%s still kernel vs blur build (bits)" % label, still.view(np.uint32), blur.view(np.uint32))


GENERAL_CASES = [  # (id, builder args, frame, tile world)
    ("c2_full_w4_room", ("final", 240, 0, 800, 600, 16, 4), 240, 1),
    ("c4_16spp_1of64_w4_full", ("final", 240, 1, 1920, 1080, 16, 8), 240, 64),
    ("c3_1of64_w5", ("final", 240, 0, 1920, 1080, 64, 8), 240, 64),
]


@pytest.mark.parametrize("case", GENERAL_CASES, ids=[c[0] for c in GENERAL_CASES])
def test_general_walks_match_product_walks(cuda, monkeypatch, case):
    """DT_GENERAL_WALKS=1 sends every wave down the exact reference-tree walks that only waves with
    an axis-parallel or NaN ray take otherwise (called out of line in the 4-wave still builds,
    dt_kernels.hip DT_GENERAL_OOL). The gathered leaves and tie order are the reference's either
    way, so the image is the same bit for bit with the same rays."""
    label, args, frame, world = case
    g, built = _globals(*args)
    tile = dt.tiles(rank=0, world=world, layout=dt.DT_OUT_SLAB) if world > 1 else dt.tiles()
    monkeypatch.setenv("DT_GENERAL_WALKS", "0")
    base, st0 = _render(g, built, frame, tile, False, monkeypatch)
    monkeypatch.setenv("DT_GENERAL_WALKS", "1")
    gen, st1 = _render(g, built, frame, tile, False, monkeypatch)
    assert st0.rays == st1.rays and st0.shadow_rays == st1.shadow_rays
    log_equal("%s general walks vs product walks (bits)" % label, gen.view(np.uint32), base.view(np.uint32))


FEATURE_CASES = [  # (id, builder args, frame, tile world): the build each scene's features select
    ("c3_room_1of64_w5", ("final", 240, 0, 1920, 1080, 64, 8), 240, 64),
    ("c2_room_full_w4", ("final", 240, 0, 800, 600, 16, 4), 240, 1),
    ("c4_mesh_1of256_w5", ("final", 240, 1, 1920, 1080, 256, 8), 240, 256),
    ("c5_tunnel_1920_1of512_w5", ("final", 1920, 0, 3840, 2160, 64, 10), 1920, 512),
    ("c5_tunnel_1600_16spp_1of64_w4", ("final", 1600, 0, 960, 540, 16, 6), 1600, 64),
]


@pytest.mark.parametrize("case", FEATURE_CASES, ids=[c[0] for c in FEATURE_CASES])
def test_feature_builds_match_full_builds(cuda, monkeypatch, case):
    """Each scene takes the build whose features cover it (dt_api.cpp: room, mesh or full for still
    frames; tunnel or blur for motion-blur frames); DT_FULL_KERNEL=1 renders it with the build that
    has every feature. Same rays, same bits."""
    label, args, frame, world = case
    g, built = _globals(*args)
    tile = dt.tiles(rank=0, world=world, layout=dt.DT_OUT_SLAB) if world > 1 else dt.tiles()
    monkeypatch.setenv("DT_FULL_KERNEL", "0")
    feat, st0 = _render(g, built, frame, tile, False, monkeypatch)
    monkeypatch.setenv("DT_FULL_KERNEL", "1")
    full, st1 = _render(g, built, frame, tile, False, monkeypatch)
    assert st0.rays == st1.rays and st0.shadow_rays == st1.shadow_rays
    log_equal("%s feature build vs full build (bits)" % label, feat.view(np.uint32), full.view(np.uint32))
