"""PMC workload for the N=8 share excess: one launch of the whole C3 frame x COPIES,
then one launch per rank share of the world-WORLD split x COPIES (dt_render_repeat_async), in that
order, so rocprofv3 --pmc dispatches 1 and 2..WORLD+1 (after the warm-ups) can be compared:
    rocprofv3 --pmc SQ_INSTS_VALU ... -- python3 tools/share_pmc.py
tools/share_pmc_cmp.py reads the counter CSVs."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import distraytracer_amd as dt  # noqa: E402
from distraytracer_amd.multigpu import tile_side  # noqa: E402


def main():
    world = int(os.environ.get("WORLD", "8"))
    copies = int(os.environ.get("COPIES", "4"))
    g, built = bench.build_globals(dt, "c3")
    scene = dt.Scene(built, g)
    shares = [None] + [dt.tiles(rank=r, world=world, layout=dt.DT_OUT_SLAB, tile_w=tile_side(world),
                                tile_h=tile_side(world)) for r in range(world)]
    outs = []
    for tile in shares:
        n = max(dt.slab_floats(g, tile), 1) if tile else 3 * g.xRes * g.yRes
        outs.append(torch.zeros(n * copies, dtype=torch.float32, device="cuda"))
    # warm-up: one plain render of the whole frame (not a repeat launch)
    dt.render(scene, g, 240, outs[0][:3 * g.xRes * g.yRes], None)
    torch.cuda.synchronize()
    for i, (tile, out) in enumerate(zip(shares, outs)):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        dt.render_repeat_async(scene, g, 240, out, copies, out.numel() // copies, tile)
        ev1.record()
        torch.cuda.synchronize()
        print("share %s ms/copy %.3f" % ("whole" if tile is None else "r%d" % (i - 1),
                                          ev0.elapsed_time(ev1) / copies), flush=True)


if __name__ == "__main__":
    main()
