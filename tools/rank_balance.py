"""Per-rank share of the tile split on ONE GPU: for world N in {1, 2, 4, 8}, render every rank's
slab (its tiles of the hashed split, DT_OUT_SLAB) one after another on this device and report each rank's
trace-kernel time. With one GPU per rank the frame takes max_r T_r plus the gather, so
T_1 / (N * max_r T_r) bounds the kernel-side strong-scaling efficiency of bench.py at N GPUs
(load balance of the interleaved tiles, the persistent grid's tail on 1/N of the pixels).

    python tools/rank_balance.py [c3|c2|c4] [reps]     (TILE=<side>: the split's tile side, default FrameSplit's for the world size;
    TILE_W=<w> TILE_H=<h>: non-square tiles at world > 1)

RES=3840x2160: the config at another resolution. WORLDS=8 (or 1,8 ...): only these world sizes (the efficiency then needs world 1 among them).
INFLIGHT=n (2, 3, ...): each rank's time per frame over 16 frames rendered back to back on n streams with
one scene object each (bench.py renders two in flight at N > 1), instead of one launch's kernel time.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import distraytracer_amd as dt  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    g, built = bench.build_globals(dt, cfg)
    if os.environ.get("RES"):   # RES=WxH: the config at another resolution (more items per launch)
        g.xRes, g.yRes = (int(v) for v in os.environ["RES"].split("x"))
    scene = dt.Scene(built, g)
    inflight = int(os.environ.get("INFLIGHT", "1"))
    scenes = [scene] + [dt.Scene(built, g) for _ in range(max(inflight, 1) - 1)]
    streams = [torch.cuda.Stream() for _ in range(max(inflight, 2))]

    def frame_ms(tile, out):
        """wall time per frame of 16 frames on `inflight` streams (frames in flight), one scene each"""
        import time
        outs = [out] + [torch.zeros_like(out) for _ in range(inflight - 1)]
        for sc in scenes:
            dt.render(sc, g, 240, out, tile)
        best = None
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(16):
                dt.render_async(scenes[k % inflight], g, 240, outs[k % inflight], tile,
                                stream=streams[k % inflight].cuda_stream)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / 16
            best = ms if best is None else min(best, ms)
        return best
    from distraytracer_amd.multigpu import tile_side
    t1 = None
    worlds = [int(v) for v in os.environ.get("WORLDS", "1,2,4,8").split(",")]
    for world in worlds:
        per, work = [], []
        for rank in (range(world) if not os.environ.get("REVERSE") else reversed(range(world))):
            ts = int(os.environ["TILE"]) if "TILE" in os.environ else tile_side(world, g.antialias_samples)   # as FrameSplit
            tw = th = ts
            if world > 1 and "TILE_W" in os.environ:   # TILE_W=w TILE_H=h: non-square tiles for world > 1
                tw, th = int(os.environ["TILE_W"]), int(os.environ["TILE_H"])
            tile = dt.tiles(rank=rank, world=world, layout=dt.DT_OUT_SLAB, tile_w=tw, tile_h=th)
            out = torch.zeros(max(dt.slab_floats(g, tile), 1), dtype=torch.float32, device="cuda")
            st = dt.render(scene, g, 240, out, tile)   # warm-up
            if inflight >= 2:
                best = frame_ms(tile, out)
            else:
                best = min(dt.render(scene, g, 240, out, tile).kernel_ms for _ in range(reps))
            per.append(round(best, 3))
            # work proxies: rays and shadow rays traced, in millions
            work.append((round(st.rays / 1e6, 2), round(st.shadow_rays / 1e6, 2)))
        if os.environ.get("REVERSE"):
            per, work = per[::-1], work[::-1]
        if world == 1:
            t1 = per[0]
        mx = max(per)
        print(json.dumps({"config": cfg, "world": world, "kernel_ms_per_rank": per, "max_ms": mx,
                          "mean_ms": round(sum(per) / world, 3),
                          "kernel_efficiency": round(t1 / (world * mx), 4) if t1 else None,
                          "rays_shadow_M": work}), flush=True)
    for sc in scenes:
        sc.close()


if __name__ == "__main__":
    main()
