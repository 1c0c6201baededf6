"""The launch path of round 5 (dt_api.cpp enqueue_render): a scene's launch record has
one device copy per counter parity, uploaded only when its bytes change, the cloud z table likewise,
and each trace launch zeroes the other parity's counters (and the sky-item launch's) from
workgroup 0, so no copy or fill kernel runs between the frames of a still scene. What could go wrong
is stale state: a record or z table not re-uploaded after a change, counters not zeroed, the sky-item
count of an earlier frame. Here one scene renders frames whose records differ (frame number, sky,
resolution, tiles) in an order that revisits each parity with and without a change, and every
image and every counter must equal a fresh scene's render of the same frame."""
import numpy as np
import pytest
import torch

import distraytracer_amd as dt

pytestmark = pytest.mark.gpu

KEYS = ("pixels", "samples", "rays", "shadow_rays", "sky_pixels", "nan_pixels", "tex_fetches",
        "stack_overflows", "uv_out_of_range", "glossy_exhausted", "reflect_errors")


def _globals(frame, res, spp):
    g = dt.globals_default()
    g.use_model = 0
    b = dt.build_scene("final", frame, g)
    g.xRes, g.yRes = res
    g.antialias_samples, g.max_depth = spp, 4
    return g, b


def _fresh(b, g, frame, tile):
    s = dt.Scene(b, g)
    out = torch.zeros(3 * g.xRes * g.yRes if tile is None else max(dt.slab_floats(g, tile), 1),
                      dtype=torch.float32, device="cuda")
    st = dt.render(s, g, frame, out, tile)
    s.close()
    return out.cpu().numpy(), {k: getattr(st, k) for k in KEYS}


@pytest.mark.parametrize("built_frame,spp,sky", [(240, 4, False), (1440, 4, True), (2000, 1, True)])
def test_reused_scene_matches_fresh_renders(cuda, built_frame, spp, sky):
    """buildFinal(240): a still room frame (the still builds, their sky-item launch); 1440: a tunnel
    frame with motion blur and sky (the z table); 2000: a 1-spp cloud frame (the deferred sky, whose
    kernel reads the record's device copy). One scene object renders a sequence that changes the
    frame number, the resolution, the sample count and the tiling and comes back to earlier
    settings; each render must equal a fresh scene's, image and counters."""
    g0, b = _globals(built_frame, (160, 96), spp)
    seq = [(0, (160, 96), spp, None), (0, (160, 96), spp, None), (8, (160, 96), spp, None),
           (0, (160, 96), 4 * spp, None),
           (0, (160, 96), spp, dt.tiles(tile_w=8, tile_h=8, rank=1, world=4, layout=dt.DT_OUT_SLAB)),
           (0, (96, 64), spp, None), (0, (160, 96), spp, None), (8, (160, 96), spp, None)]
    scene = dt.Scene(b, g0)
    for i, (df, res, ns, tile) in enumerate(seq):
        g = dt.globals_default()
        g.use_model = 0
        dt.build_scene("final", built_frame, g)   # the builder's globals (perlin_cloud, ...)
        g.xRes, g.yRes = res
        g.antialias_samples, g.max_depth = ns, 4
        frame = built_frame + df
        n = 3 * g.xRes * g.yRes if tile is None else max(dt.slab_floats(g, tile), 1)
        out = torch.zeros(n, dtype=torch.float32, device="cuda")
        st = dt.render(scene, g, frame, out, tile)
        got = out.cpu().numpy()
        ref, ref_st = _fresh(b, g, frame, tile)
        assert np.array_equal(got, ref), "render %d: image differs from a fresh scene's" % i
        assert {k: getattr(st, k) for k in KEYS} == ref_st, "render %d: counters differ" % i
        assert st.rays > 0
        if sky and tile is None:
            assert st.sky_pixels > 0
    scene.close()


def test_two_scenes_alternating_streams(cuda):
    """bench.py's two frames in flight: two scene objects on two streams, frames enqueued without
    waiting; every frame's image equals the first, and each scene's counters those of one frame."""
    g, b = _globals(240, (160, 96), 4)
    ref, ref_st = _fresh(b, g, 240, None)
    scenes = [dt.Scene(b, g), dt.Scene(b, g)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [torch.zeros(3 * g.xRes * g.yRes, dtype=torch.float32, device="cuda") for _ in range(6)]
    for k in range(6):
        dt.render_async(scenes[k % 2], g, 240, outs[k], None, stream=streams[k % 2].cuda_stream)
    torch.cuda.synchronize()
    for k in range(6):
        assert np.array_equal(outs[k].cpu().numpy(), ref), "frame %d" % k
    for s in scenes:
        st = dt.collect_stats(s)
        assert {k: getattr(st, k) for k in KEYS} == ref_st
        s.close()
