"""C5 driver: render a range of animation frames of buildFinal(n*8) (scene.h:605-1100), frame-
parallel over ranks (frame f on rank f % world), each frame from fresh globals as the
reference's one-process-per-frame runs do (Q23). Reports frames/s and Mpixel-samples/s.

  python tools/animate.py --frames 0:300:37 --res 3840x2160 --spp 64 [--out DIR]
  python -m torch.distributed.run --nproc-per-node 8 tools/animate.py ...

Frames >= frame_cloud (n >= 244) force 1 spp and no aperture, as buildFinal does
(scene.h:795-796); the reported samples are the ones actually rendered.
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def parse_range(s):
    a, b, c = (s.split(":") + ["1"])[:3] if s.count(":") >= 1 else (s, str(int(s) + 1), "1")
    return list(range(int(a), int(b), int(c)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", default="0:300:37", help="start:stop:step of n (frame = n*8)")
    ap.add_argument("--res", default="3840x2160")
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--depth", type=int, default=10)
    ap.add_argument("--out", default="", help="directory for frame.NNNN.png (none: keep on the GPU)")
    ap.add_argument("--per-frame", action="store_true", help="print host-build and render ms per frame (stderr)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import distraytracer_amd as dt

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    W, H = (int(v) for v in args.res.split("x"))
    mine = [n for n in parse_range(args.frames) if n % world == rank]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    samples = 0

    def prepare(n):
        """host side of frame n: buildFinal(n*8) from fresh globals, BVH, flatten, upload"""
        torch.cuda.set_device(local)   # the HIP device is per thread
        f0 = time.perf_counter()
        g = dt.globals_default()   # fresh globals per frame (one process per frame in the reference)
        g.use_model = 0
        g.xRes, g.yRes, g.antialias_samples, g.max_depth = W, H, args.spp, args.depth
        built = dt.build_scene("final", n * 8, g)
        scene = dt.Scene(built, g, upload=False)   # host half only: the GPU is busy with frame n
        return g, scene, time.perf_counter() - f0

    # frame n+1's host build runs on a worker thread while frame n renders (ctypes releases the
    # GIL inside the library calls)
    img = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
    with ThreadPoolExecutor(1) as ex:
        fut = ex.submit(prepare, mine[0]) if mine else None
        for idx, n in enumerate(mine):
            g, scene, host_s = fut.result()
            if idx + 1 < len(mine):
                fut = ex.submit(prepare, mine[idx + 1])
            f1 = time.perf_counter()
            scene.upload()   # device half (a few ms), between renders
            st = dt.render(scene, g, n * 8, img)
            torch.cuda.synchronize()
            f2 = time.perf_counter()
            samples += st.samples
            if args.per_frame:
                print(json.dumps({"n": n, "frame": n * 8, "host_ms": round(host_s * 1e3, 1),
                                  "render_ms": round((f2 - f1) * 1e3, 1), "spp": st.samples // max(st.pixels, 1),
                                  "rays_per_sample": round(st.rays / max(st.samples, 1), 3),
                                  "sky_pixels": st.sky_pixels}), file=sys.stderr, flush=True)
            if args.out:
                os.makedirs(args.out, exist_ok=True)
                dt.write_png(os.path.join(args.out, "frame.%04d.png" % n), g, img.cpu().numpy())
            scene.close()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed, float(samples), float(len(mine))], dtype=torch.float64, device="cuda")
        tmax = t[:1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed, samples, nframes = float(tmax.item()), float(t[1].item()), int(t[2].item())
    else:
        nframes = len(mine)
    if rank == 0:
        print(json.dumps({"config": "C5 buildFinal(n*8) frames %s, %dx%d, %d spp, depth %d" % (args.frames, W, H,
                                                                                          args.spp, args.depth),
                          "n_gpus": world, "frames": nframes, "seconds": round(elapsed, 3),
                          "frames_per_s": round(nframes / elapsed, 4),
                          "mpixel_samples_per_s": round(samples / elapsed / 1e6, 3),
                          "parallelism": "frame-parallel (frame n on rank n %% %d)" % world}))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
