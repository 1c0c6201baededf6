"""The drop-in boundary exercised the ways a caller of the reference's renderImage would use it,
on the GPU, against the CPU oracle:

  * from C: the `dtrender` CLI (csrc/dtrender.cpp, the reference's ./render modes over
    include/dt.h) writes a PPM whose bytes equal writePPM of the oracle's image;
  * multi-GPU plumbing over the real RCCL backend: GatherPipeline (tile split, async gather,
    unpack on the render stream) at world size 1 gives the plain single-render image;
  * render-time globals the scene was not built for: blur shifts of the other sign than the
    bump tree's one-sided padding assumed fall back to exact walks.
"""
import os
import subprocess

import numpy as np
import pytest
import torch

import distraytracer_amd as dt
import oracle
from parity_check import assert_parity, log_equal

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DTRENDER = os.path.join(ROOT, "distraytracer_amd", "dtrender")


def _read_ppm(path):
    data = open(path, "rb").read()
    parts = data.split(b"\n", 3)
    assert parts[0] == b"P6" and parts[2] == b"255"
    w, h = (int(v) for v in parts[1].split())
    px = np.frombuffer(parts[3], dtype=np.uint8)
    assert px.size == 3 * w * h
    return w, h, px


@pytest.mark.parametrize("mode,args,builder,frame,settings", [
    ("spheres", [], "spheres", 0, dict(xRes=256, yRes=256, antialias_samples=1, max_depth=1)),
    ("final", ["30", "--res", "192x108", "--spp", "4", "--depth", "3"], "final", 240,
     dict(xRes=192, yRes=108, antialias_samples=4, max_depth=3)),
    ("prismcyl", ["7"], "prismcyl", 7, dict(xRes=640, yRes=480)),
], ids=["spheres", "final30", "prismcyl7"])
def test_dtrender_cli_matches_oracle(cuda, tmp_path, mode, args, builder, frame, settings):
    """A non-Python caller of include/dt.h: dtrender builds, renders on the GPU and writes the PPM
    (helpers.h:174-195 truncation); its bytes must be the oracle image's truncated bytes."""
    assert os.path.exists(DTRENDER), "dtrender not built (make -C distraytracer_amd/csrc)"
    out = tmp_path / ("%s.ppm" % mode)
    r = subprocess.run([DTRENDER, mode] + args + ["--out", str(out)], capture_output=True, text=True, timeout=120)
    print(r.stdout, r.stderr)
    assert r.returncode == 0
    w, h, px = _read_ppm(out)
    g = dt.globals_default()
    g.use_model = 0
    built = dt.build_scene(builder, frame, g)
    for k, v in settings.items():
        setattr(g, k, v)
    assert (w, h) == (g.xRes, g.yRes)
    ref, _ = oracle.render(built, g, frame, dt.tiles())
    ref_px = ref.astype(np.uint8)   # (unsigned char)float, as writePPM
    log_equal("dtrender %s PPM bytes vs writePPM(oracle)" % mode, px, ref_px)


def test_gather_pipeline_over_rccl(cuda, tmp_path):
    """bench.py's N > 1 path at world size 1 over the real NCCL (= RCCL) backend: frames render
    into double-buffered slabs on torch's stream, GatherPipeline gathers them asynchronously and
    scatters on rank 0 with dt_unpack_slabs on the same stream. The assembled image equals a plain
    full-frame render of the same frame, for every frame of the pipeline."""
    import torch.distributed as dist
    from distraytracer_amd.multigpu import FrameSplit, GatherPipeline
    # a file rendezvous (a port probed free beforehand can be lost to another process)
    dist.init_process_group("nccl", init_method="file://" + str(tmp_path / "rdv"), rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        g = dt.globals_default()
        g.use_model = 0
        built = dt.build_scene("final", 240, g)
        g.xRes, g.yRes, g.antialias_samples, g.max_depth = 240, 136, 4, 3
        scene = dt.Scene(built, g)
        split = FrameSplit(g, 1, 0)
        dev = torch.device("cuda", 0)
        z = lambda n: torch.zeros(n, dtype=torch.float32, device=dev)
        pipe = GatherPipeline(split, [z(split.slab_floats), z(split.slab_floats)],
                              [z(split.slab_floats), z(split.slab_floats)], z(3 * g.xRes * g.yRes))
        sh = torch.cuda.current_stream(dev).cuda_stream
        images = []
        for k in range(3):
            g.seed = k
            dt.render_async(scene, g, 240, pipe.slab(k), split.tile, stream=sh)
            pipe.submit(k)   # completes frame k-1 into the image
            if k > 0:
                images.append(pipe.image.clone())
        pipe.finish()
        images.append(pipe.image.clone())
        torch.cuda.synchronize()
        for k, img in enumerate(images):
            g.seed = k
            ref = z(3 * g.xRes * g.yRes)
            dt.render(scene, g, 240, ref, dt.tiles())
            log_equal("GatherPipeline frame %d vs dt_render" % k, img.cpu().numpy(), ref.cpu().numpy())
        scene.close()
    finally:
        dist.destroy_process_group()


def test_gather_pipeline_two_streams_over_rccl(cuda, tmp_path):
    """bench.py's N > 1 path with two frames in flight (its default): frame k renders on
    streams[k % 2] with a scene object of its own, GatherPipeline orders the gather after the render
    by an event and the next render into a slab after that slab's gather. Every assembled image
    equals a plain full-frame render of its frame."""
    import torch.distributed as dist
    from distraytracer_amd.multigpu import FrameSplit, GatherPipeline
    # a file rendezvous (a port probed free beforehand can be lost to another process)
    dist.init_process_group("nccl", init_method="file://" + str(tmp_path / "rdv"), rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        g = dt.globals_default()
        g.use_model = 0
        built = dt.build_scene("final", 240, g)
        g.xRes, g.yRes, g.antialias_samples, g.max_depth = 240, 136, 4, 3
        scenes = [dt.Scene(built, g), dt.Scene(built, g)]
        split = FrameSplit(g, 1, 0)
        dev = torch.device("cuda", 0)
        z = lambda n: torch.zeros(n, dtype=torch.float32, device=dev)
        streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
        pipe = GatherPipeline(split, [z(split.slab_floats), z(split.slab_floats)],
                              [z(split.slab_floats), z(split.slab_floats)], z(3 * g.xRes * g.yRes), streams=streams)
        images = []
        n = 5
        for k in range(n):
            g.seed = k
            pipe.begin(k)
            dt.render_async(scenes[k % 2], g, 240, pipe.slab(k), split.tile, stream=pipe.stream(k).cuda_stream)
            pipe.submit(k)   # completes frame k-1 into the image
            if k > 0:
                images.append(pipe.image.clone())
        pipe.finish()
        images.append(pipe.image.clone())
        torch.cuda.synchronize()
        assert len(images) == n
        for k, img in enumerate(images):
            g.seed = k
            ref = z(3 * g.xRes * g.yRes)
            dt.render(scenes[0], g, 240, ref, dt.tiles())
            log_equal("GatherPipeline (2 streams) frame %d vs dt_render" % k, img.cpu().numpy(), ref.cpu().numpy())
        for sc in scenes:
            sc.close()
    finally:
        dist.destroy_process_group()


def test_negative_blur_shift_at_render_time(cuda):
    """The bump tree and the blur-padded shadow-grid lists of a tunnel frame are padded for
    non-negative shifts only (the build globals' move_per_frame, accel_t >= 0: host_accel.cpp
    up_only). dt_render takes its own globals: rendering the same scene with the motion negated
    draws negative shifts, which must send those waves to the reference-tree walk (DParams
    bump_up_only), not to leaves that were never padded below. Against the oracle."""
    g = dt.globals_default()
    g.use_model = 0
    frame = 1680
    built = dt.build_scene("final", frame, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth = 320, 180, 16, 3
    scene = dt.Scene(built, g)   # built for shifts >= 0
    g.move_per_frame = -g.move_per_frame
    g.accel_t = -g.accel_t
    tile = dt.tiles(x0=96, y0=40, x1=224, y1=136)
    out = torch.zeros(3 * g.xRes * g.yRes, dtype=torch.float32, device="cuda")
    st = dt.render(scene, g, frame, out, tile)
    scene.close()
    ref, rst = oracle.render(built, g, frame, tile)
    assert st.rays == rst.rays and st.shadow_rays == rst.shadow_rays and st.rays > st.samples
    assert_parity("negative blur shifts at render time", out.cpu().numpy(), ref)
