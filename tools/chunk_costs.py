"""Diagnostic: per-item durations of one rank's share (chunk items for spp > 64) from a
-DDT_ITEM_TIMES=2 build with DT_ITEM_COSTS=1 (dt_debug_item_costs), and what a different queue order
would give the persistent grid's drain (list scheduling of the measured durations over the grid's
wave slots, one item per dequeue).

    DT_LIB=distraytracer_amd/variants/libdt_itemrt.so python tools/chunk_costs.py [c4] [world] [rank ...]

Prints, per share: the kernel time, the items' summed wave time, the longest items (pixel, chunk,
ms), how much of the wave time the top 0.1% / 1% of items hold, and the replayed makespan for the
queue order, for items above k x the mean first (the rest in queue order) and for longest first."""
import ctypes
import heapq
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import distraytracer_amd as dt  # noqa: E402
from distraytracer_amd.multigpu import tile_side  # noqa: E402


def tile_rot(slot, world):   # dt_scene_dev.h tile_rot
    h = (slot * 2654435761) & 0xFFFFFFFF
    h ^= h >> 15
    h = (h * 0x2C1B3C6D) & 0xFFFFFFFF
    h ^= h >> 12
    return h % world


def pixel_of(q, tw, th, tiles_x, rank, world):
    slot, lp = divmod(q, tw * th)
    t = slot * world + (rank + tile_rot(slot, world)) % world
    ty, tx = divmod(t, tiles_x)
    py, px = divmod(lp, tw)
    return tx * tw + px, ty * th + py


def replay(d, slots):
    """makespan of list scheduling: each item, in order, to the wave slot that frees first"""
    h = [0.0] * slots
    for x in d:
        heapq.heapreplace(h, h[0] + x)
    return max(h)


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
    world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    ranks = [int(v) for v in sys.argv[3:]] or list(range(world))
    os.environ["DT_ITEM_COSTS"] = "1"
    g, built = bench.build_globals(dt, cfg)
    s = dt.Scene(built, g)
    ts = tile_side(world, g.antialias_samples)
    spp = int(int(g.antialias_samples ** 0.5) ** 2)
    chunks = (spp + 63) // 64
    ppw = 64 // spp if spp <= 64 else 1   # pixels per wave item (dt_render: spp < 64 packs pixels)
    tiles_x = (g.xRes + ts - 1) // ts
    slots = int(os.environ.get("SLOTS", "5120"))
    for rank in ranks:
        tile = dt.tiles(rank=rank, world=world, layout=dt.DT_OUT_SLAB, tile_w=ts, tile_h=ts)
        out = torch.zeros(max(dt.slab_floats(g, tile), 1), dtype=torch.float32, device="cuda")
        dt.render(s, g, 240, out, tile)
        st = dt.render(s, g, 240, out, tile)
        n = int(dt.lib.dt_debug_item_costs(s.handle, None, 0))
        if n <= 0:
            raise SystemExit("no item costs: a -DDT_ITEM_TIMES=2 build (DT_LIB) and DT_ITEM_COSTS=1 are needed")
        c = np.zeros(n, dtype=np.uint32)
        dt.lib.dt_debug_item_costs(s.handle, c.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), n)
        ms = c.astype(np.float64) * 1e-5   # 100 MHz ticks -> ms
        per_chunk = chunks > 1 and n % chunks == 0 and n // chunks * ppw >= st.pixels
        order = np.argsort(ms)[::-1]
        top = []
        for code in order[:12]:
            item, ck = divmod(int(code), chunks) if per_chunk else (int(code), -1)
            x, y = pixel_of(item * ppw, ts, ts, tiles_x, rank, world)   # (the item's first pixel)
            top.append({"x": x, "y": y, "chunk": ck, "ms": round(float(ms[code]), 3)})
        tot = ms.sum()
        srt = np.sort(ms)[::-1]
        mean = tot / n
        res = {"config": cfg, "world": world, "rank": rank, "items": n, "chunk_items": per_chunk,
               "kernel_ms": round(st.kernel_ms, 3), "wave_ms_total": round(tot, 1), "mean_ms": round(mean, 4),
               "ideal_ms": round(tot / slots, 3), "top0.1pct_share": round(srt[:max(n // 1000, 1)].sum() / tot, 4),
               "top1pct_share": round(srt[:max(n // 100, 1)].sum() / tot, 4),
               "replay_queue_ms": round(replay(ms, slots), 3)}
        for k in (4, 16, 64):
            hot = ms > k * mean
            res["replay_hot%dx_first_ms" % k] = round(replay(np.concatenate([ms[hot], ms[~hot]]), slots), 3)
            res["hot%dx_items" % k] = int(hot.sum())
        res["replay_longest_first_ms"] = round(replay(srt, slots), 3)
        res["longest"] = top
        print(json.dumps(res), flush=True)
    s.close()


if __name__ == "__main__":
    main()
