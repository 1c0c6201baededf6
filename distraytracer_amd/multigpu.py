"""Image-space tile split across ranks + gather of finished tiles.

Every rank holds the whole (tiny) scene and renders one tile of every group of `world`
consecutive tiles (raster order), the ranks rotated by a hash of the group (dt_scene_dev.h
tile_of), into a packed slab: the expensive sky/glossy regions spread over all GPUs, and unlike a
plain t % world interleave no rank is tied to a fixed set of tile columns. The tile side follows
the world size and the samples per pixel (tile_side): 2x2 for pixels of several 64-sample chunks
(spp > 64, C4) at every N > 1 and for one-wave pixels (C3) from N = 4 on, 8x8 (the primary lists'
block) otherwise; many tiles per rank even out the ranks' work. Rank-balance kernel times of C3 (profiles/r04zs_rank_balance_tiles.log,
slowest share 8x8 against 16x16): N=2 17.60 against 17.75 ms, N=4 9.09 against 9.12, N=8 4.73
against 4.87 (round 3: slowest rank 6.29 -> 5.96 ms from 32x32, profiles/r03z_rank_balance_tiles.log).
32x32 at N = 1, where the waves that run at once cover a compact part of the image: at world 1 the
8x8 split renders C3 in 36.6 ms against 35.0 (16x16) and 34.9 (32x32, the plain path's 34.8;
profiles/r04zs_split_tiles.log).
The only exchange step is one gather of the finished slabs to rank 0 (torch.distributed:
RCCL over xGMI on the GPU box, gloo in the CPU tests), after which rank 0 scatters the slabs
into the ppmOut image (dt_unpack_slabs). Sample RNG is keyed on the global pixel index, so the
image is bit-identical for any world size.
"""
from . import DT_OUT_SLAB, slab_floats_max, tiles, unpack_slabs


def tile_side(world, spp=64):
    """the split's tile side for a world size and samples per pixel (module docstring). Pixels of
    several 64-sample chunks (spp > 64: C4) take 2x2 at N > 1, where each chunk is a queue item of
    its own (chunk items, dt_api.cpp): C4's kernel-side bound 0.988 / 0.982 / 0.969 at N = 2 / 4 / 8
    (every world-8 share within 39.2-39.6 ms; profiles/r06h_rb_c4_t2.log, r06i_rb_c4_t2.log), against
    0.985 / 0.978 / 0.930 with 4x4, 0.986 / 0.956 / 0.915 with 8x8 and 0.974 / 0.980 / 0.871 with
    16x16 (profiles/r06g_rb_t4.log, r06g_rb_t8.log, r06g_rb_t16.log). The cost is concentrated: the
    longest 1% of C4's chunk items hold ~47% of the wave time, in a few clusters of mesh pixels
    (profiles/r06e_costs_c4_w8.log), and small tiles spread each cluster over every rank.
    Pixels of one wave each (33..64 samples: C3) take 2x2 from N = 4 on and 8x8 at N = 2 (two runs
    of each, C3, two frames in flight, profiles/r06s_rb_c3_t8a/b.log, r06s_rb_c3_t2a/b.log): the
    slowest share at N = 8 4.431 / 4.417 ms with 2x2 against 4.440 / 4.457 with 8x8, at N = 4
    8.632 / 8.597 against 8.632 / 8.624, at N = 2 16.988 / 17.003 against 16.915 / 16.944. Several
    pixels per wave (spp <= 32: C2) keep 8x8 (profiles/r06i_rb_c2_t4.log, r06i_rb_c2_t8.log)."""
    if world <= 1:
        return 32
    # the samples the kernel takes: int(sqrt(aa))^2 (host_flatten.cpp; aa = 65..80 is one chunk)
    import math
    s = int(math.isqrt(max(int(spp), 1))) ** 2
    if s > 64:
        return 2
    return 2 if s > 32 and world >= 4 else 8


class FrameSplit:
    def __init__(self, g, world, rank, tile_w=None, tile_h=None):
        spp = getattr(g, "antialias_samples", 64)
        tile_w = tile_w or tile_side(world, spp)
        tile_h = tile_h or tile_side(world, spp)
        self.g = g
        self.world = world
        self.rank = rank
        self.tile = tiles(tile_w=tile_w, tile_h=tile_h, rank=rank, world=world, layout=DT_OUT_SLAB)
        self.base = tiles(tile_w=tile_w, tile_h=tile_h, rank=0, world=world, layout=DT_OUT_SLAB)
        # equal-size slabs (rank 0 owns the most tiles) so a plain gather works
        self.slab_floats = slab_floats_max(g, self.base)

    def gather(self, slab, gathered, group=None, async_op=False):
        """gather the per-rank slabs into `gathered` (world*slab_floats) on rank 0. With
        async_op the collective's Work is returned (wait() before reading `gathered`)."""
        import torch.distributed as dist
        if self.world == 1 and not (dist.is_available() and dist.is_initialized()):
            gathered.copy_(slab)
            return None
        parts = list(gathered.view(self.world, self.slab_floats).unbind(0)) if self.rank == 0 else None
        return dist.gather(slab, gather_list=parts, dst=0, group=group, async_op=async_op)

    def assemble(self, gathered, image, stream=None):
        """scatter the gathered slabs into the ppmOut image; on the GPU the unpack kernel runs on
        `stream` (default: torch's current stream, the one the gather's wait() ordered)"""
        if stream is None and getattr(gathered, "is_cuda", False):
            import torch
            stream = torch.cuda.current_stream(gathered.device).cuda_stream
        unpack_slabs(self.g, self.base, self.world, gathered, image, stream=stream)


class GatherPipeline:
    """Double-buffered frame gather: frame k renders into slab k%2; submit(k) starts its gather
    (async collective) and first completes frame k-1's (wait + scatter into the image on rank
    0), so one frame's gather runs beside the next frame's render. finish() drains.

    streams (optional, two torch.cuda.Streams): frame k renders on streams[k%2] (call begin(k)
    first, and render with a scene object of its own per stream: a scene's launches share one
    launch record), so frame k+1's waves start on the CUs frame k's last waves leave idle. The
    collective and the scatter stay on torch's current stream, ordered after the render by an
    event; a slab is rendered into again only after its gather and scatter (ev_free). Without
    streams, frames render on the current stream."""

    def __init__(self, split, slabs, gathered, image, streams=None):
        self.split = split
        self.slabs = slabs          # two per-rank slab buffers
        self.gathered = gathered    # two world*slab_floats buffers on rank 0 (ignored elsewhere)
        self.image = image
        self.streams = streams
        self.ev_free = [None, None]
        self.pending = None

    def slab(self, k):
        return self.slabs[k % 2]

    def stream(self, k):
        """the stream frame k renders on (None: torch's current stream)"""
        return self.streams[k % 2] if self.streams else None

    def begin(self, k):
        """before frame k's render: its stream waits until slab k%2's previous gather is done"""
        if self.streams and self.ev_free[k % 2] is not None:
            self.streams[k % 2].wait_event(self.ev_free[k % 2])

    def submit(self, k):
        b = k % 2
        rendered = None
        if self.streams:
            import torch
            rendered = torch.cuda.Event()
            rendered.record(self.streams[b])
        self.finish()
        if rendered is not None:
            import torch
            torch.cuda.current_stream(self.slabs[b].device).wait_event(rendered)
        work = self.split.gather(self.slabs[b], self.gathered[b] if self.split.rank == 0 else None, async_op=True)
        self.pending = (work, b)

    def finish(self):
        if self.pending is None:
            return
        work, b = self.pending
        self.pending = None
        if work is not None:
            work.wait()   # orders torch's current stream after the collective
        if self.split.rank == 0:
            self.split.assemble(self.gathered[b], self.image)   # on that same stream
        if self.streams:
            import torch
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.slabs[b].device))
            self.ev_free[b] = ev


class FrameQueue:
    """Frame-parallel animation (C5): frames handed out one at a time from a shared
    counter in the process group's store, in descending order of their estimated cost (longest
    processing time first: the room-to-tunnel transition frames, up to ~50x the mean, go out first
    and the cheap ones fill the tails). A rank asks for its next frame when it starts preparing it,
    so a rank that drew an expensive frame simply takes fewer. No collective on the data path: the
    store counter is a host-side atomic add.

    frames: the frame ids to render; cost: {frame id: estimated cost} (missing ids: the mean);
    store: a torch.distributed Store (None: a single process, plain iteration); key, epoch: the
    store keys of this queue, the same on every rank. With a store the epoch is required: a second
    queue in the same process group must pass another one, so that its counter starts at 0 (a queue
    whose keys are already in the store is refused, on every rank); rank, world: this process's
    place in the group (default: torch.distributed's)."""

    def __init__(self, frames, cost=None, store=None, key="dt_frame_queue", epoch=None, rank=None, world=None):
        cost = cost or {}
        known = [cost[n] for n in frames if n in cost]
        mean = sum(known) / len(known) if known else 1.0
        # stable: equal costs keep the frames' own order
        self.order = sorted(frames, key=lambda n: -cost.get(n, mean))
        self.store = store
        if store is not None and epoch is None:
            raise ValueError("FrameQueue: pass an epoch with a store (one per queue in the process group)")
        self.key = "%s/%d" % (key, epoch or 0)
        self._local = 0
        if store is not None:
            if rank is None or world is None:
                import torch.distributed as dist
                rank = dist.get_rank() if rank is None else rank
                world = dist.get_world_size() if world is None else world
            # every rank must hand out the same order, or frames would be rendered twice or never:
            # each rank publishes a hash of its order, waits for every rank's and compares them all,
            # so on a mismatch every rank raises (none goes on rendering)
            import hashlib
            h = hashlib.sha1(repr(self.order).encode()).hexdigest()
            # a reused epoch: its counter is already past frames, or a rank's order hash is stale. The
            # check comes before this rank publishes its own hash, and no rank hands out a frame
            # before every hash is published, so no rank of this queue can have created these keys
            used = store.check([self.key]) or store.check(["%s/order/%d" % (self.key, rank)])
            store.set("%s/order/%d" % (self.key, rank), "used" if used else h)
            if used:
                raise RuntimeError("FrameQueue %s: the store already holds this queue's keys (pass a new epoch)" % self.key)
            keys = ["%s/order/%d" % (self.key, r) for r in range(world)]
            store.wait(keys)
            hashes = [store.get(k) for k in keys]
            hashes = [x.decode() if isinstance(x, bytes) else x for x in hashes]
            bad = [r for r, x in enumerate(hashes) if x != h]
            if bad:
                raise RuntimeError("FrameQueue %s: rank %d's frame order differs from rank(s) %s "
                                   "(different frame lists or cost data)" % (self.key, rank, bad))

    def next(self):
        """the next frame id, or None when every frame has been handed out"""
        if self.store is None:
            i = self._local
            self._local += 1
        else:
            i = int(self.store.add(self.key, 1)) - 1
        return self.order[i] if i < len(self.order) else None

    def __iter__(self):
        while True:
            n = self.next()
            if n is None:
                return
            yield n
