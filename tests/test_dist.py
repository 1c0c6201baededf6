"""Multi-rank frame split on CPU (gloo): every rank renders its interleaved 32x32 tiles into a
packed slab, FrameSplit gathers the slabs to rank 0 and scatters them into the ppmOut image
(SURVEY §8e). The per-rank renderer here is the oracle (the GPU path is covered by the -m gpu
tests); what this checks is the N>1 plumbing bench.py runs over RCCL: tile ownership, equal
slab sizes for a plain gather, the gather itself and the unpack, against the oracle's
full-frame render. Sample RNG is keyed on the global pixel, so the assembled frame must be
bit-identical to the single-rank one."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scene(cfg):
    import distraytracer_amd as dt
    g = dt.globals_default()
    g.use_model = 0
    if cfg == "final":
        b = dt.build_scene("final", 240, g)
        g.xRes, g.yRes, g.antialias_samples, g.max_depth = 72, 40, 4, 3
    elif cfg == "final64":   # one pixel per wave: 2x2 split tiles from world 4 on (tile_side)
        b = dt.build_scene("final", 240, g)
        g.xRes, g.yRes, g.antialias_samples, g.max_depth = 38, 22, 64, 2
    else:
        b = dt.build_scene("spheres", 0, g)
        g.xRes, g.yRes, g.antialias_samples, g.max_depth = 70, 45, 1, 1
    return g, b


def _worker(rank, world, port, cfg, result_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from distraytracer_amd.multigpu import FrameSplit
        g, b = _scene(cfg)
        split = FrameSplit(g, world, rank)
        slab = np.zeros(split.slab_floats, dtype=np.float32)
        oracle.render(b, g, 240, split.tile, out=slab, nthreads=2)
        slab_t = torch.from_numpy(slab)
        gathered = torch.zeros(world * split.slab_floats if rank == 0 else 1, dtype=torch.float32)
        split.gather(slab_t, gathered if rank == 0 else None)
        if rank == 0:
            image = torch.zeros(3 * g.xRes * g.yRes, dtype=torch.float32)
            split.assemble(gathered, image)
            np.save(result_path, image.numpy())
    finally:
        dist.destroy_process_group()


def _pipe_worker(rank, world, port, result_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from distraytracer_amd.multigpu import FrameSplit, GatherPipeline
        g, b = _scene("spheres")
        split = FrameSplit(g, world, rank)
        z = lambda n: torch.zeros(n, dtype=torch.float32)
        pipe = GatherPipeline(split, [z(split.slab_floats), z(split.slab_floats)],
                              [z(world * split.slab_floats), z(world * split.slab_floats)],
                              z(3 * g.xRes * g.yRes))
        images = []
        for k in range(3):   # frame k renders with seed k, as bench.py's steps render frames
            g.seed = k
            slab = pipe.slab(k).numpy()
            slab[:] = 0
            oracle.render(b, g, 240, split.tile, out=slab, nthreads=2)
            pipe.submit(k)   # completes frame k-1 into the image, starts frame k's gather
            if rank == 0 and k > 0:
                images.append(pipe.image.numpy().copy())
        pipe.finish()
        if rank == 0:
            images.append(pipe.image.numpy().copy())
            np.save(result_path, np.stack(images))
    finally:
        dist.destroy_process_group()


def test_gather_pipeline_double_buffer(tmp_path):
    """bench.py's pipelined gather (frame k's gather beside frame k+1's render, two slab
    buffers): after every submit the image holds exactly the previous frame."""
    import distraytracer_amd as dt
    import oracle
    out = str(tmp_path / "imgs.npy")
    mp.start_processes(_pipe_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    got = np.load(out)
    g, b = _scene("spheres")
    for k in range(3):
        g.seed = k
        ref, _ = oracle.render(b, g, 240, dt.tiles(), nthreads=4)
        assert np.array_equal(got[k], ref), k


@pytest.mark.parametrize("world,cfg", [(2, "final"), (3, "spheres"), (4, "final64")])
def test_tile_split_gather_equals_single_rank(tmp_path, world, cfg):
    import distraytracer_amd as dt
    import oracle
    out = str(tmp_path / "img.npy")
    mp.start_processes(_worker, args=(world, _free_port(), cfg, out), nprocs=world, join=True,
                       start_method="spawn")
    got = np.load(out)
    g, b = _scene(cfg)
    ref, _ = oracle.render(b, g, 240, dt.tiles(), nthreads=4)
    assert np.array_equal(got, ref)   # bit-identical for any world size


def _queue_worker(rank, world, port, result_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import time
        from distraytracer_amd.multigpu import FrameQueue
        store = dist.distributed_c10d._get_default_store()
        frames = list(range(0, 40, 2))
        cost = {n: float(n % 7 + (50 if n == 24 else 0)) for n in frames}
        q = FrameQueue(frames, cost, store, epoch=0, rank=rank, world=world)
        got = []
        for n in q:
            got.append(n)
            time.sleep(0.002 * cost[n])   # "render": a rank holding a costly frame takes fewer
        # a second queue in the same process group (a second animation pass) starts afresh
        q2 = FrameQueue(list(range(5)), None, store, epoch=1, rank=rank, world=world)
        got2 = list(q2)
        everyone = [None] * world
        dist.all_gather_object(everyone, [got, got2])
        # ranks whose cost data disagree must fail loudly, not duplicate or skip frames
        bad_cost = {n: float(n if rank == 1 else -n) for n in frames}
        dist.barrier()
        try:
            FrameQueue(frames, bad_cost, store, epoch=2)   # rank / world from torch.distributed
            mismatch = False
        except RuntimeError:
            mismatch = True
        flags = [None] * world
        dist.all_gather_object(flags, mismatch)
        # a queue built again on a used epoch is refused on every rank (its counter is past the end:
        # it would hand out nothing), and a store without an epoch is refused outright
        dist.barrier()
        try:
            FrameQueue(frames, cost, store, epoch=0, rank=rank, world=world)
            reused = False
        except RuntimeError:
            reused = True
        try:
            FrameQueue(frames, cost, store, rank=rank, world=world)
            no_epoch = False
        except ValueError:
            no_epoch = True
        refused = [None] * world
        dist.all_gather_object(refused, [reused, no_epoch])
        if rank == 0:
            with open(result_path, "w") as f:
                import json
                json.dump({"per_rank": [e[0] for e in everyone], "second": [e[1] for e in everyone],
                           "order": q.order, "mismatch": flags, "refused": refused}, f)
    finally:
        dist.destroy_process_group()


def test_frame_queue_hands_out_every_frame_once(tmp_path):
    """C5 frame-parallel (tools/animate.py --split frames): the store counter hands every frame to
    exactly one rank, most expensive first (LPT); each rank sees its frames in queue order. A second
    queue in the same group hands out its frames afresh, and ranks whose frame orders differ raise."""
    import json
    out = str(tmp_path / "q.json")
    mp.start_processes(_queue_worker, args=(3, _free_port(), out), nprocs=3, join=True, start_method="spawn")
    r = json.load(open(out))
    flat = sorted(n for lst in r["per_rank"] for n in lst)
    assert flat == list(range(0, 40, 2))
    order = r["order"]
    assert order[0] == 24                      # the costliest frame goes out first
    for lst in r["per_rank"]:
        pos = [order.index(n) for n in lst]
        assert pos == sorted(pos)
    assert sorted(n for lst in r["second"] for n in lst) == list(range(5))
    # rank 1's order is the reverse of ranks 0 and 2's: every rank sees the disagreement and raises
    assert all(r["mismatch"])
    assert all(a and b for a, b in r["refused"])   # a reused epoch, and a store without an epoch


def test_frame_queue_single_process():
    from distraytracer_amd.multigpu import FrameQueue
    q = FrameQueue([5, 1, 3, 9], {5: 1.0, 1: 10.0, 9: 10.0})   # 3 unknown: the mean (7)
    assert list(q) == [1, 9, 3, 5]


def test_tile_side_rule():
    """multigpu.tile_side: 32 for a whole frame, 2x2 for multi-chunk pixels at N > 1 (keyed on the
    samples the kernel takes, int(sqrt(aa))^2: aa = 80 is one chunk), 2x2 for one-wave pixels from
    N = 4 on, 8x8 for several pixels per wave (profiles/r06s_*, r06i_*, r06h_*)."""
    from distraytracer_amd.multigpu import tile_side
    assert tile_side(1, 64) == 32 and tile_side(1, 256) == 32
    assert [tile_side(n, 256) for n in (2, 4, 8)] == [2, 2, 2]
    assert [tile_side(n, 64) for n in (2, 4, 8)] == [8, 2, 2]
    assert [tile_side(n, 80) for n in (2, 8)] == [8, 2]      # 64 samples taken: one chunk
    assert [tile_side(n, 81) for n in (2, 8)] == [2, 2]      # 81: two chunks
    assert [tile_side(n, 16) for n in (2, 4, 8)] == [8, 8, 8]
