"""Experiment: per-slot costs of a config's rank shares from a -DDT_ITEM_TIMES=2 build (DT_LIB=...,
tools/tail.py's item start/end times), written as slot orders by decreasing cost for
DT_TILE_ORDER=dir:<out> (dt_api.cpp): the longest tiles first, so that a launch's drain is made of
its cheapest tiles (longest-processing-time order).

    DT_LIB=distraytracer_amd/variants/libdt_itemrt.so python tools/lpt_order.py c3 <out dir> [worlds]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import distraytracer_amd as dt  # noqa: E402
from distraytracer_amd.multigpu import tile_side  # noqa: E402
from tail import intervals  # noqa: E402


def main():
    cfg, out_dir = sys.argv[1], sys.argv[2]
    worlds = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "1,8").split(",")]
    os.makedirs(out_dir, exist_ok=True)
    g, built = bench.build_globals(dt, cfg)
    s = dt.Scene(built, g)
    for world in worlds:
        ts = tile_side(world)
        for rank in range(world):
            tile = dt.tiles(rank=rank, world=world, layout=dt.DT_OUT_SLAB, tile_w=ts, tile_h=ts)
            nf = max(dt.slab_floats(g, tile), 1)
            out = torch.zeros(nf, dtype=torch.float32, device="cuda")
            dt.render(s, g, 240, out, tile)
            dt.render(s, g, 240, out, tile)
            n = nf // 3
            start, end = intervals(out, n)
            dur = np.where((start > 0) & (end > 0), end - start, 0).astype(np.float64)
            cost = dur.reshape(-1, ts * ts).sum(axis=1)            # per slot, slab order
            order = np.argsort(-cost, kind="stable").astype(np.uint32)
            order.tofile(os.path.join(out_dir, "order_w%d_r%d_t%d.bin" % (world, rank, ts)))
            top = cost[order[:3]] / 1e5
            print("world %d rank %d: %d slots, top tile costs %s ms, median %.3f ms"
                  % (world, rank, cost.size, np.round(top, 3).tolist(), np.median(cost) / 1e5), flush=True)
    s.close()


if __name__ == "__main__":
    main()
