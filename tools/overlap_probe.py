"""Probe: does a second frame in flight hide the persistent grid's tail? Renders K frames of a
config (or of one rank's tile share) back to back, either all on one stream, or alternating
between two streams with one scene object each (every scene has its own launch record and queue
word), and reports wall-clock ms per frame for both.

    python tools/overlap_probe.py [c3|c2|c4] [world] [K]      (world > 1: rank 0's share, 8x8 tiles)
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import distraytracer_amd as dt  # noqa: E402


def run(scenes, streams, outs, g, tile, k):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(k):
        j = i % len(scenes)
        dt.render_async(scenes[j], g, 240, outs[j], tile, stream=streams[j].cuda_stream)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / k


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    world = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    g, built = bench.build_globals(dt, cfg)
    tile = dt.tiles(rank=0, world=world, layout=dt.DT_OUT_SLAB, tile_w=8, tile_h=8) if world > 1 else dt.tiles()
    n = dt.slab_floats(g, tile) if world > 1 else 3 * g.xRes * g.yRes
    scenes = [dt.Scene(built, g), dt.Scene(built, g)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [torch.zeros(n, dtype=torch.float32, device="cuda") for _ in range(2)]
    for s in scenes:   # upload + warm-up
        dt.render(s, g, 240, outs[0], tile)
    res = {"config": cfg, "world": world, "frames": k}
    for rep in range(2):
        res["one_stream_ms_%d" % rep] = round(run(scenes[:1], streams[:1], outs[:1], g, tile, k), 3)
        res["two_streams_ms_%d" % rep] = round(run(scenes, streams, outs, g, tile, k), 3)
    same = torch.equal(outs[0], outs[1])
    res["images_equal"] = bool(same)
    print(json.dumps(res), flush=True)
    for s in scenes:
        s.close()


if __name__ == "__main__":
    main()
