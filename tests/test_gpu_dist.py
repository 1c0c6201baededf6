"""The product path at world size 2 in separate processes.

Two spawned ranks share the one GPU of the box. Each builds the scene, renders its FrameSplit share
of every frame with libdt.so (dt.render into its slab: the HIP trace kernel, then one D2H copy), and
GatherPipeline gathers the slabs to rank 0 over gloo (RCCL refuses two ranks on one device, and gloo
gathers host tensors), where dt_unpack_slabs' host twin (FrameSplit.assemble) scatters them into the
ppmOut image. The assembled frames must be bit-identical to single-process dt.render images of the
same frames (sample RNG is keyed on the global pixel, render_final_project.cpp:1031-1218, so the
split cannot change a pixel), and rank 1's slab must equal the oracle's render of the same share:
the ppmOut layout the slabs reassemble into is the reference's (render_final_project.cpp:1213-1217).
Scaling across GPUs stays unmeasured on hardware (no 8-GPU node); this is the correctness of the
multi-process product path. test_shipped_device_path_world2 runs bench.py's N > 1 step itself (two
frames in flight on two streams, device slabs, the device scatter), with the gather's transport
swapped for a host hop over gloo.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import distraytracer_amd as dt
import oracle
from parity_check import assert_parity, log_equal

pytestmark = pytest.mark.gpu

FRAMES = 2   # seeds 0 and 1: two frames through the double-buffered pipeline


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _globals(spp=16, W=400, H=300):
    g = dt.globals_default()
    g.use_model = 0
    built = dt.build_scene("final", 240, g)
    # C2's settings (Cook-Torrance doors, area-light soft shadows, glossy) at a quarter of its pixels
    g.xRes, g.yRes, g.antialias_samples, g.max_depth = W, H, spp, 4
    return g, built


def _rank(rank, world, port, outdir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    # a file rendezvous in the test's own directory: a TCP store on a port probed free beforehand
    # can lose it to another process (EADDRINUSE seen on a GPU box)
    dist.init_process_group("gloo", init_method="file://" + os.path.join(outdir, "rdv"), rank=rank,
                            world_size=world)
    try:
        from distraytracer_amd.multigpu import FrameSplit, GatherPipeline
        torch.cuda.set_device(0)
        g, built = _globals()
        scene = dt.Scene(built, g)
        split = FrameSplit(g, world, rank)
        z = lambda n: torch.zeros(n, dtype=torch.float32)
        pipe = GatherPipeline(split, [z(split.slab_floats), z(split.slab_floats)],
                              [z(world * split.slab_floats), z(world * split.slab_floats)],
                              z(3 * g.xRes * g.yRes))
        images, slabs, rays = [], [], []
        for k in range(FRAMES):
            g.seed = k
            st = dt.render(scene, g, 240, pipe.slab(k).numpy(), split.tile)   # libdt, host slab
            slabs.append(pipe.slab(k).numpy().copy())
            rays.append((st.rays, st.shadow_rays, st.pixels))
            pipe.submit(k)   # completes frame k-1 into the image, starts frame k's gather
            if rank == 0 and k > 0:
                images.append(pipe.image.numpy().copy())
        pipe.finish()
        if rank == 0:
            images.append(pipe.image.numpy().copy())
            np.save(os.path.join(outdir, "images.npy"), np.stack(images))
        np.save(os.path.join(outdir, "slabs_%d.npy" % rank), np.stack(slabs))
        np.save(os.path.join(outdir, "rays_%d.npy" % rank), np.array(rays, dtype=np.int64))
        scene.close()
    finally:
        dist.destroy_process_group()


def test_product_path_world2_processes(cuda, tmp_path):
    world = 2
    mp.start_processes(_rank, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    got = np.load(tmp_path / "images.npy")
    g, built = _globals()
    scene = dt.Scene(built, g)
    single_rays = []
    for k in range(FRAMES):
        g.seed = k
        out = torch.zeros(3 * g.xRes * g.yRes, dtype=torch.float32, device=cuda)
        st = dt.render(scene, g, 240, out, dt.tiles())
        single_rays.append(st.rays)
        log_equal("world-2 processes frame %d = single-process render" % k, got[k], out.cpu().numpy())
    scene.close()
    # every pixel rendered once: the ranks' rays add up to the single render's
    r0, r1 = np.load(tmp_path / "rays_0.npy"), np.load(tmp_path / "rays_1.npy")
    assert [int(a + b) for a, b in zip(r0[:, 0], r1[:, 0])] == single_rays
    assert int(r0[0, 2] + r1[0, 2]) == g.xRes * g.yRes
    # rank 1's slab of frame 0 against the oracle's render of rank 1's share
    from distraytracer_amd.multigpu import FrameSplit
    g.seed = 0
    split = FrameSplit(g, world, 1)
    ref = np.zeros(split.slab_floats, dtype=np.float32)
    _, rst = oracle.render(built, g, 240, split.tile, out=ref)
    slab1 = np.load(tmp_path / "slabs_1.npy")[0]
    assert_parity("world-2 processes rank 1 slab vs oracle", slab1, ref)
    assert int(r1[0, 0]) == rst.rays and int(r1[0, 1]) == rst.shadow_rays


class _HostHopSplit:
    """FrameSplit with the gather's transport swapped for gloo over host copies (RCCL refuses two
    ranks on one device): the device slab goes to the host on torch's current stream, gloo gathers,
    and rank 0's gathered slabs go back into the DEVICE buffer the pipeline hands it. Everything else
    (tile split, slab layout, the device scatter dt_unpack_slabs) is FrameSplit's own."""

    def __init__(self, split):
        self.s = split
        self.rank, self.world, self.tile, self.slab_floats = split.rank, split.world, split.tile, split.slab_floats

    def gather(self, slab, gathered, group=None, async_op=False):
        import torch.distributed as dist
        host = slab.cpu()   # on torch's current stream, which GatherPipeline.submit ordered after the render
        parts = [torch.zeros_like(host) for _ in range(self.world)] if self.rank == 0 else None
        dist.gather(host, gather_list=parts, dst=0, group=group)
        if self.rank == 0:
            gathered.copy_(torch.cat(parts).to(gathered.device))
        return None

    def assemble(self, gathered, image, stream=None):
        self.s.assemble(gathered, image, stream)


def _rank_device_path(rank, world, port, outdir, shape=(16, 400, 300)):
    """bench.py's N > 1 step (bench.py step(): render_async on streams[k % 2] with a scene object per
    stream into device slabs, GatherPipeline.begin / submit / finish, the device scatter on rank 0)."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    # a file rendezvous in the test's own directory: a TCP store on a port probed free beforehand
    # can lose it to another process (EADDRINUSE seen on a GPU box)
    dist.init_process_group("gloo", init_method="file://" + os.path.join(outdir, "rdv"), rank=rank,
                            world_size=world)
    try:
        from distraytracer_amd.multigpu import FrameSplit, GatherPipeline
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        g, built = _globals(*shape)
        scenes = [dt.Scene(built, g), dt.Scene(built, g)]
        split = _HostHopSplit(FrameSplit(g, world, rank))
        zd = lambda n: torch.zeros(n, dtype=torch.float32, device=dev)
        streams = [torch.cuda.Stream(dev) for _ in range(2)]
        pipe = GatherPipeline(split, [zd(split.slab_floats), zd(split.slab_floats)],
                              [zd(world * split.slab_floats) if rank == 0 else zd(1) for _ in range(2)],
                              zd(3 * g.xRes * g.yRes) if rank == 0 else zd(1), streams=streams)
        images, slabs = [], []
        for k in range(FRAMES + 1):   # frames with seeds 0, 1, 2: both slabs and streams reused
            g.seed = k
            pipe.begin(k)
            dt.render_async(scenes[k % 2], g, 240, pipe.slab(k), split.tile, stream=pipe.stream(k).cuda_stream)
            pipe.submit(k)   # completes frame k-1 on the device image, starts frame k's gather
            if rank == 0 and k > 0:
                torch.cuda.synchronize()
                images.append(pipe.image.cpu().numpy())
            torch.cuda.synchronize()
            slabs.append(pipe.slab(k).cpu().numpy())
        pipe.finish()
        torch.cuda.synchronize()
        if rank == 0:
            images.append(pipe.image.cpu().numpy())
            np.save(os.path.join(outdir, "dev_images.npy"), np.stack(images))
        np.save(os.path.join(outdir, "dev_slabs_%d.npy" % rank), np.stack(slabs))
        for sc in scenes:
            sc.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("shape", [(16, 400, 300), (81, 160, 96)], ids=["16spp-8x8", "81spp-2x2-chunks"])
def test_shipped_device_path_world2(cuda, tmp_path, shape):
    """The N > 1 path as bench.py ships it: two frames in flight per rank on two
    streams with a scene object each, device slabs, GatherPipeline's event ordering, and the device
    scatter (dt_unpack_slabs) on rank 0; only the collective's transport is a host hop over gloo.
    Every assembled frame is bit-identical to a single-process render of that frame, and rank 1's
    slab of frame 0 equals the oracle's render of its share. At 16 spp the split takes 8x8 tiles; at
    81 spp (two 64-sample chunks a pixel) 2x2 tiles and chunk items, as C4 does at N > 1."""
    world = 2
    mp.start_processes(_rank_device_path, args=(world, _free_port(), str(tmp_path), shape), nprocs=world, join=True,
                       start_method="spawn")
    got = np.load(tmp_path / "dev_images.npy")
    assert got.shape[0] == FRAMES + 1
    g, built = _globals(*shape)
    scene = dt.Scene(built, g)
    for k in range(FRAMES + 1):
        g.seed = k
        out = torch.zeros(3 * g.xRes * g.yRes, dtype=torch.float32, device=cuda)
        dt.render(scene, g, 240, out, dt.tiles())
        log_equal("shipped device path, world 2, frame %d = single-process render" % k, got[k], out.cpu().numpy())
    scene.close()
    from distraytracer_amd.multigpu import FrameSplit
    g.seed = 0
    split = FrameSplit(g, world, 1)
    ref = np.zeros(split.slab_floats, dtype=np.float32)
    oracle.render(built, g, 240, split.tile, out=ref)
    assert_parity("shipped device path rank 1 slab vs oracle", np.load(tmp_path / "dev_slabs_1.npy")[0], ref)
