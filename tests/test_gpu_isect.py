"""The intersection micro-benchmark (2^24 primary rays of the C3 camera) against the
oracle: dt_intersect_primary (dt_isect_kernel: rayColor's gather + closest hit for the camera's
primary rays, through the primary lists or the fast tree as the trace kernel takes them) and
or_primary_hit (the reference's gather of every leaf whose box the ray passes, then the strict-<
closest hit in gather order) give the same shape and the same float t for every ray.

Ray windows: the first rays, the middle of the frame, and the last rays of the 2^24 (sample indices
8 and up: 2^24 exceeds 8 rays per pixel of 1920x1080). Integer and float results: bit-exact."""
import numpy as np
import pytest
import torch

import distraytracer_amd as dt
import oracle

pytestmark = pytest.mark.gpu

N_BENCH = 1 << 24
WIN = 1 << 15


def _scene(builder, frame, models, W, H):
    g = dt.globals_default()
    g.use_model = models
    built = dt.build_scene(builder, frame, g)
    g.xRes, g.yRes = W, H
    return g, built


def _check(g, built, frame, firsts, n=WIN):
    scene = dt.Scene(built, g)
    try:
        for first in firsts:
            shape = torch.empty(n, dtype=torch.int32, device="cuda")
            t = torch.empty(n, dtype=torch.float32, device="cuda")
            dt.intersect_primary(scene, g, frame, first, shape, t)
            rs, rt = oracle.primary_hit(built, g, frame, first, n)
            gs, gt = shape.cpu().numpy(), t.cpu().numpy()
            bad = np.nonzero((gs != rs) | (gt.view(np.uint32) != rt.view(np.uint32)))[0]
            print("rays %d..%d: hits %.3f, mismatches %d" % (first, first + n, float((gs >= 0).mean()), bad.size))
            assert bad.size == 0, "ray %d: gpu (%d, %r) oracle (%d, %r)" % (
                first + bad[0], gs[bad[0]], gt[bad[0]], rs[bad[0]], rt[bad[0]])
    finally:
        scene.close()


def test_isect_c3_camera():
    g, built = _scene("final", 240, 0, 1920, 1080)
    _check(g, built, 240, [0, N_BENCH // 2, N_BENCH - WIN])


def test_isect_c4_models():
    # the meshes (triangles) in front of the camera
    g, built = _scene("final", 240, 1, 1920, 1080)
    _check(g, built, 240, [N_BENCH // 2 - WIN, N_BENCH // 2 + 3 * WIN])


def test_isect_c5_frames():
    # a room frame and a tunnel frame at 4K
    for n in (60, 150):
        g, built = _scene("final", n * 8, 0, 3840, 2160)
        _check(g, built, n * 8, [(3840 * 2160 * 8) // 3], n=WIN)


def test_isect_host_arrays_and_empty():
    g, built = _scene("final", 240, 0, 1920, 1080)
    scene = dt.Scene(built, g)
    try:
        shape = np.empty(4096, dtype=np.int32)
        t = np.empty(4096, dtype=np.float32)
        dt.intersect_primary(scene, g, 240, 123457, shape, t)
        rs, rt = oracle.primary_hit(built, g, 240, 123457, 4096)
        assert np.array_equal(shape, rs) and np.array_equal(t.view(np.uint32), rt.view(np.uint32))
        assert dt.intersect_primary(scene, g, 240, 0, np.empty(0, np.int32), np.empty(0, np.float32)) == 0
    finally:
        scene.close()


def test_isect_full_bench_size():
    # all 2^24 rays in one call, as tools/isect_bench.py runs them; every t finite for a hit
    g, built = _scene("final", 240, 0, 1920, 1080)
    scene = dt.Scene(built, g)
    try:
        shape = torch.empty(N_BENCH, dtype=torch.int32, device="cuda")
        t = torch.empty(N_BENCH, dtype=torch.float32, device="cuda")
        ms = dt.intersect_primary(scene, g, 240, 0, shape, t)
        hit = shape >= 0
        print("2^24 rays: %.3f ms, hit fraction %.4f" % (ms, float(hit.float().mean())))
        assert ms > 0
        assert bool(torch.isfinite(t[hit]).all()) and bool((t[~hit] == torch.finfo(torch.float32).max).all())
        # the first window again inside the full run: same answers as a separate call
        s2 = torch.empty(WIN, dtype=torch.int32, device="cuda")
        t2 = torch.empty(WIN, dtype=torch.float32, device="cuda")
        dt.intersect_primary(scene, g, 240, 0, s2, t2)
        assert torch.equal(shape[:WIN], s2) and torch.equal(t[:WIN].view(torch.int32), t2.view(torch.int32))
    finally:
        scene.close()
