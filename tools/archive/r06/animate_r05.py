# round-5 animate.py (one frame at a time), kept for the round-6 A/B of two frames in flight
"""C5 driver: render a range of animation frames of buildFinal(n*8) (scene.h:605-1100), each frame
from fresh globals as the reference's one-process-per-frame runs do (Q23). Reports frames/s and
Mpixel-samples/s, and per frame the conditions the reference aborts on, which must
all stay zero over the run.

  python tools/animate.py --frames 0:300:1 --res 3840x2160 --spp 64 [--out DIR] [--per-frame]
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/animate.py \\
         --split frames|tiles ...

--split frames (default): frame-parallel. Frames are handed out by a shared counter in the process
  group's store, most expensive first (longest-processing-time order from data/c5_frame_cost.json,
  the round-2 per-frame times); no collective on the data path (FrameQueue, multigpu.py).
--split tiles: every frame is tile-split over all ranks and gathered to rank 0 over RCCL, as
  bench.py does for C3 (FrameSplit / GatherPipeline, multigpu.py).
--split static: frame n on rank n % world (round 2's assignment, for comparison).

Frames >= frame_cloud (n >= 244) force 1 spp and no aperture, as buildFinal does
(scene.h:795-796); the reported samples are the ones actually rendered.

--donate auto (default): frames whose rays fan out into deep glossy cascades render with the
  work-sharing trace kernel (DT_DONATE=1), the others with the product kernel. The
  choice comes from a probe render of a 1/256 tile share of the frame itself (~0.5% of the
  frame): more than --donate-rps rays per sample (default 3.1) selects work sharing. Measured over
  all 300 frames (profiles/r03k_c5_full_*.log): frames below ~3.1 rays per sample (C3 1.46, the
  room frames, the tunnel's blur frames at 2.8) lose 1-5% with it, the transition frames from 3.2
  up to 8.1 gain 2-17%. --donate on|off forces one kernel.
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)

# the reference printf+throws / terminates on these (the device counts them), plus the
# device's own DFS stack limit and NaN pixels; all must stay zero. RectPrismV2::getNorm's off-prism
# points (geometry.cpp:890-919) are not among them: the reference prints and returns the nearest face
# normal, and so does the device; they are reported as prism_norm_fallback.
ABORT_COUNTERS = ("stack_overflows", "nan_pixels", "uv_out_of_range", "glossy_exhausted", "reflect_errors",
                  "spherelight_exhausted", "donate_overflow")
REPORTED = ABORT_COUNTERS + ("prism_norm_fallback",)


def parse_range(s):
    a, b, c = (s.split(":") + ["1"])[:3] if s.count(":") >= 1 else (s, str(int(s) + 1), "1")
    return list(range(int(a), int(b), int(c)))


def frame_costs():
    p = os.path.join(ROOT, "data", "c5_frame_cost.json")
    if not os.path.exists(p):
        return {}
    with open(p) as f:
        return {int(k): float(v) for k, v in json.load(f)["render_ms"].items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", default="0:300:37", help="start:stop:step of n (frame = n*8)")
    ap.add_argument("--res", default="3840x2160")
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--depth", type=int, default=10)
    ap.add_argument("--split", default="frames", choices=("frames", "tiles", "static"))
    ap.add_argument("--out", default="", help="directory for frame.NNNN.png (none: keep on the GPU)")
    ap.add_argument("--per-frame", action="store_true", help="print host-build and render ms per frame (stderr)")
    ap.add_argument("--donate", default="auto", choices=("auto", "on", "off"))
    ap.add_argument("--donate-rps", type=float, default=3.1)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import distraytracer_amd as dt
    from distraytracer_amd.multigpu import FrameQueue, FrameSplit, GatherPipeline

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    distributed = "WORLD_SIZE" in os.environ
    if distributed:
        dist.init_process_group("nccl", device_id=dev)
    W, H = (int(v) for v in args.res.split("x"))
    frames = parse_range(args.frames)
    if args.split == "frames":
        store = dist.distributed_c10d._get_default_store() if distributed and world > 1 else None
        mine = iter(FrameQueue(frames, frame_costs(), store, epoch=0, rank=rank, world=world))
    elif args.split == "static":
        mine = iter([n for n in frames if n % world == rank])
    else:
        mine = iter(frames)   # every rank renders its tiles of every frame
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    samples = 0
    aborts = {k: 0 for k in REPORTED}
    done = []

    def prepare(n):
        """host side of frame n: buildFinal(n*8) from fresh globals, BVH, flatten, acceleration"""
        torch.cuda.set_device(local)   # the HIP device is per thread
        f0 = time.perf_counter()
        g = dt.globals_default()   # fresh globals per frame (one process per frame in the reference)
        g.use_model = 0
        g.xRes, g.yRes, g.antialias_samples, g.max_depth = W, H, args.spp, args.depth
        built = dt.build_scene("final", n * 8, g)
        scene = dt.Scene(built, g, upload=False)   # host half only: the GPU is busy with frame n-1
        return n, g, scene, time.perf_counter() - f0

    def next_job(ex):
        n = next(mine, None)
        return ex.submit(prepare, n) if n is not None else None

    img = torch.empty(3 * W * H if (args.split != "tiles" or rank == 0) else 1, dtype=torch.float32, device=dev)
    pipe = None
    if args.split == "tiles":
        g0 = dt.globals_default()
        g0.xRes, g0.yRes = W, H
        split = FrameSplit(g0, world, rank)
        z = lambda k: torch.zeros(k, dtype=torch.float32, device=dev)
        pipe = GatherPipeline(split, [z(split.slab_floats), z(split.slab_floats)],
                              [z(world * split.slab_floats if rank == 0 else 1) for _ in range(2)], img)
    sh = torch.cuda.current_stream(dev).cuda_stream
    g_res = dt.globals_default()
    g_res.xRes, g_res.yRes = W, H
    probe_tile = dt.tiles(rank=0, world=256, layout=dt.DT_OUT_SLAB)
    probe = torch.empty(max(dt.slab_floats(g_res, probe_tile), 1), dtype=torch.float32, device=dev)
    donated = 0

    def choose_kernel(scene, g, n):
        """the trace kernel of frame n's scene (dt_scene_set_kernel, never the process environment:
        the worker thread is building the next scene meanwhile): the probe's rays per sample decide
        (--donate auto)"""
        if args.donate != "auto":
            scene.set_kernel(dt.DT_KERNEL_DONATE if args.donate == "on" else dt.DT_KERNEL_PRODUCT)
            return args.donate == "on", None
        scene.set_kernel(dt.DT_KERNEL_PRODUCT)
        pst = dt.render(scene, g, n * 8, probe, probe_tile)
        rps = pst.rays / max(pst.samples, 1)
        on = rps > args.donate_rps
        scene.set_kernel(dt.DT_KERNEL_DONATE if on else dt.DT_KERNEL_PRODUCT)
        return on, rps
    # frame n+1's host build runs on a worker thread while frame n renders (ctypes releases the
    # GIL inside the library calls)
    with ThreadPoolExecutor(1) as ex:
        fut = next_job(ex)
        k = 0
        while fut is not None:
            n, g, scene, host_s = fut.result()
            fut = next_job(ex)
            f1 = time.perf_counter()
            scene.upload()   # device half (a few ms), between renders
            dn_on, probe_rps = choose_kernel(scene, g, n)
            donated += dn_on
            if pipe is None:
                st = dt.render(scene, g, n * 8, img)
            else:
                dt.render_async(scene, g, n * 8, pipe.slab(k), split.tile, stream=sh)
                pipe.submit(k)   # gathers frame k, completes frame k-1 into the image
                st = dt.collect_stats(scene, sh)
            torch.cuda.synchronize()
            f2 = time.perf_counter()
            samples += st.samples
            for key in REPORTED:
                aborts[key] += getattr(st, key)
            done.append(n)
            if args.per_frame:
                rec = {"n": n, "frame": n * 8, "rank": rank, "host_ms": round(host_s * 1e3, 1),
                       "render_ms": round((f2 - f1) * 1e3, 1), "spp": st.samples // max(st.pixels, 1),
                       "donate": bool(dn_on), "probe_rays_per_sample": probe_rps and round(probe_rps, 3),
                       "donations": st.donations, "donate_overflow": st.donate_overflow,
                       "rays_per_sample": round(st.rays / max(st.samples, 1), 3), "sky_pixels": st.sky_pixels}
                rec.update({key: getattr(st, key) for key in REPORTED})
                print(json.dumps(rec), file=sys.stderr, flush=True)
            if args.out and (pipe is None or rank == 0):
                if pipe is not None:
                    pipe.finish()
                os.makedirs(args.out, exist_ok=True)
                dt.write_png(os.path.join(args.out, "frame.%04d.png" % n), g, img.cpu().numpy())
            scene.close()
            k += 1
    if pipe is not None:
        pipe.finish()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    nframes = len(done) if args.split != "tiles" else len(frames)
    if distributed and world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        c = torch.tensor([float(samples), float(len(done))] + [float(v) for v in aborts.values()],
                         dtype=torch.float64, device=dev)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        samples = c[0].item()
        if args.split != "tiles":
            nframes = int(c[1].item())
        aborts = {key: int(v) for key, v in zip(REPORTED, c[2:].tolist())}
    if rank == 0:
        print(json.dumps({"config": "C5 buildFinal(n*8) frames %s, %dx%d, %d spp, depth %d" % (args.frames, W, H,
                                                                                          args.spp, args.depth),
                          "n_gpus": world, "frames": nframes, "seconds": round(elapsed, 3),
                          "frames_per_s": round(nframes / elapsed, 4),
                          "mpixel_samples_per_s": round(samples / elapsed / 1e6, 3),
                          "parallelism": {"frames": "frame-parallel, dynamic queue in LPT order",
                                          "static": "frame-parallel, frame n on rank n %% %d" % world,
                                          "tiles": "tile-split x%d + RCCL gather per frame" % world}[args.split],
                          "abort_counters": {k: aborts[k] for k in ABORT_COUNTERS},
                          "prism_norm_fallback": aborts["prism_norm_fallback"],
                          "work_sharing": {"mode": args.donate, "rays_per_sample_above": args.donate_rps,
                                           "frames_on_rank0": donated}}), flush=True)
    if distributed:
        dist.destroy_process_group()
    if any(aborts[k] for k in ABORT_COUNTERS):
        raise SystemExit("abort conditions of the reference were hit: %s" % aborts)


if __name__ == "__main__":
    main()
