"""Image-space tile split across ranks + gather of finished tiles.

Every rank holds the whole (tiny) scene and renders the 32x32 tiles t with t % world == rank
(interleaved, so the expensive sky/glossy regions spread over all GPUs) into a packed slab.
The only exchange step is one gather of the finished slabs to rank 0 (torch.distributed:
RCCL over xGMI on the GPU box, gloo in the CPU tests), after which rank 0 scatters the slabs
into the ppmOut image (dt_unpack_slabs). Sample RNG is keyed on the global pixel index, so the
image is bit-identical for any world size.
"""
from . import DT_OUT_SLAB, slab_floats_max, tiles, unpack_slabs


class FrameSplit:
    def __init__(self, g, world, rank, tile_w=32, tile_h=32):
        self.g = g
        self.world = world
        self.rank = rank
        self.tile = tiles(tile_w=tile_w, tile_h=tile_h, rank=rank, world=world, layout=DT_OUT_SLAB)
        self.base = tiles(tile_w=tile_w, tile_h=tile_h, rank=0, world=world, layout=DT_OUT_SLAB)
        # equal-size slabs (rank 0 owns the most tiles) so a plain gather works
        self.slab_floats = slab_floats_max(g, self.base)

    def gather(self, slab, gathered, group=None):
        """gather the per-rank slabs into `gathered` (world*slab_floats) on rank 0."""
        import torch.distributed as dist
        if self.world == 1:
            gathered.copy_(slab)
            return
        parts = list(gathered.view(self.world, self.slab_floats).unbind(0)) if self.rank == 0 else None
        dist.gather(slab, gather_list=parts, dst=0, group=group)

    def assemble(self, gathered, image):
        unpack_slabs(self.g, self.base, self.world, gathered, image)
