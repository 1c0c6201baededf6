"""Diagnostic: how busy the persistent trace grid stays over one launch, from a -DDT_ITEM_TIMES=2
build (DT_LIB=...; tools/build_full_variant.sh itemrt EXTRA=-DDT_ITEM_TIMES=2), which stores each
item's start and end on the 100 MHz clock in place of its pixel. For each world size's rank-0 share
(FrameSplit tiles, as bench.py at N ranks): the launch's span, the items in flight over time
against the grid's wave count, the time lost at the start (ramp) and after the queue drains
(tail), and the longest items of the tail.

    python tools/tail.py [c3|c2|c4] [worlds, default 1,8]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import distraytracer_amd as dt  # noqa: E402
from distraytracer_amd.multigpu import tile_side  # noqa: E402


def intervals(out, n):
    a = out[:3 * n].view(n, 3).cpu().numpy().astype(np.int64)
    s_lo, e_lo, e_hi = a[:, 0], a[:, 1], a[:, 2]
    end = (e_hi << 24) | e_lo
    start = (end & ~np.int64(0xFFFFFF)) | s_lo
    start = np.where(start > end, start - (1 << 24), start)   # the start's low bits wrapped
    return start, end


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
        start, end = start[ok], end[ok]
        t0, t1 = start.min(), end.max()
        # items in flight over time: +1 at each start, -1 at each end
        ev = np.concatenate([np.stack([start, np.ones_like(start)], 1), np.stack([end, -np.ones_like(end)], 1)])
        ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
        cur = np.cumsum(ev[:, 1])
        dtk = np.diff(np.append(ev[:, 0], t1))
        peak = int(np.percentile(cur, 99))
        busy = float((np.minimum(cur, peak) * dtk).sum()) / (peak * float(t1 - t0))
        # ramp: until in-flight first reaches 95% of peak; tail: after the last time it was there
        at = np.nonzero(cur >= 0.95 * peak)[0]
        ramp = (ev[at[0], 0] - t0) / 1e5 if at.size else None
        tail_start = ev[at[-1], 0] if at.size else t0
        tail = (t1 - tail_start) / 1e5
        lost_tail = float(((peak - np.minimum(cur, peak)) * dtk)[ev[:, 0] >= tail_start].sum()) / peak / 1e5
        dur = (end - start) / 1e5
        late = np.argsort(end)[::-1][:5]
        print(json.dumps({"config": cfg, "world": world, "items": int(ok.sum()), "kernel_ms": round(st.kernel_ms, 3),
                          "span_ms": round((t1 - t0) / 1e5, 3), "waves_in_flight_p99": peak,
                          "busy_fraction": round(busy, 4), "ramp_ms": round(ramp, 3) if ramp is not None else None,
                          "tail_ms": round(tail, 3), "tail_lost_ms": round(lost_tail, 3),
                          "item_ms_mean": round(float(dur.mean()), 4), "item_ms_p99": round(float(np.percentile(dur, 99)), 4),
                          "item_ms_max": round(float(dur.max()), 3),
                          "last_items_ms": [[round((start[k] - t0) / 1e5, 3), round(float(dur[k]), 3)] for k in late]}),
              flush=True)
    s.close()


if __name__ == "__main__":
    main()
