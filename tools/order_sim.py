"""Diagnostic: what a different queue order would give the persistent grid's drain. Runs the
-DDT_ITEM_TIMES=2 build (DT_LIB=distraytracer_amd/variants/libdt_itemrt.so, as tools/tail.py) to
get each item's duration in queue order, then replays the queue by list scheduling (each batch of
P.item_batch items to the wave slot that frees first, slots = the measured waves in flight) for the
measured order and for reorderings: items above a cost threshold first (in queue order, the rest
after them in queue order) with the threshold at several multiples of the mean, and full
longest-first. The replay's makespan against the measured span validates the model.
    python tools/order_sim.py [c3|c2|c4] [worlds, default 1,8]"""
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
from tail import intervals  # noqa: E402


def replay(d, slots, batch):
    """makespan of list scheduling: batches of `batch` consecutive items, each to the first free slot"""
    h = [0.0] * slots
    heapq.heapify(h)
    n = len(d)
    cs = np.concatenate([[0.0], np.cumsum(d)])
    for b in range(0, n, batch):
        t = heapq.heappop(h)
        heapq.heappush(h, t + cs[min(b + batch, n)] - cs[b])
    return max(h)


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    worlds = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "1,8").split(",")]
    g, built = bench.build_globals(dt, cfg)
    s = dt.Scene(built, g)
    for world in worlds:
        ts = tile_side(world, g.antialias_samples)   # as FrameSplit
        tile = dt.tiles(rank=0, world=world, layout=dt.DT_OUT_SLAB, tile_w=ts, tile_h=ts)
        nf = max(dt.slab_floats(g, tile), 1)
        out = torch.zeros(nf, dtype=torch.float32, device="cuda")
        dt.render(s, g, 240, out, tile)
        st = dt.render(s, g, 240, out, tile)
        n = nf // 3
        start, end = intervals(out, n)
        ok = (start > 0) & (end > 0)
        d = np.where(ok, (end - start) / 1e5, 0.0)   # ms, queue order
        span = (end[ok].max() - start[ok].min()) / 1e5
        # waves in flight (p99), as tools/tail.py
        ev = np.concatenate([np.stack([start[ok], np.ones(ok.sum(), np.int64)], 1),
                             np.stack([end[ok], -np.ones(ok.sum(), np.int64)], 1)])
        ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
        slots = int(np.percentile(np.cumsum(ev[:, 1]), 99))
        batch = 3 if n >= 256 * 5120 else 2   # dt_api.cpp item_batch (grid 5120 at 5 waves)
        res = {"config": cfg, "world": world, "items": int(n), "kernel_ms": round(st.kernel_ms, 3),
               "span_ms": round(float(span), 3), "slots": slots, "batch": batch,
               "ideal_ms": round(float(d.sum()) / slots, 3), "replay_queue_ms": round(replay(d, slots, batch), 3)}
        mean = float(d[ok].mean())
        for k in (2, 4, 8, 16):
            hot = d > k * mean
            order = np.concatenate([np.nonzero(hot)[0], np.nonzero(~hot)[0]])
            res["replay_hot%dx_first_ms" % k] = round(replay(d[order], slots, batch), 3)
            res["hot%dx_fraction" % k] = round(float(hot.mean()), 5)
        res["replay_longest_first_ms"] = round(replay(np.sort(d)[::-1], slots, batch), 3)
        res["replay_batch1_ms"] = round(replay(d, slots, 1), 3)
        # batches of `batch` items spaced n/batch apart in the queue (item q's batch partner q + n/batch)
        m = -(-n // batch)
        strided = np.concatenate([d, np.zeros(m * batch - n)]).reshape(batch, m).T.reshape(-1)
        res["replay_strided_batch_ms"] = round(replay(strided, slots, batch), 3)
        res["longest_items_ms"] = [round(float(v), 3) for v in np.sort(d)[::-1][:6]]
        res["longest_items_queue_pos"] = [int(v) for v in np.argsort(d)[::-1][:6]]
        if os.environ.get("SAVE"):
            np.savez_compressed("%s_%s_w%d.npz" % (os.environ["SAVE"], cfg, world), d=d.astype(np.float32),
                                slots=slots, batch=batch)
        print(json.dumps(res), flush=True)
    s.close()


if __name__ == "__main__":
    main()
