"""Benchmark: Mpixel-samples/s of the distraytracer render loop on MI355X.

Workload (BASELINE.json configs[2], north_star's target): buildFinal(240) — the repo's default
scene (`./render` = frame 30 -> buildFinal(240)) without the missing OBJ models — at
1920x1080, antialias_samples=64 (64 spp), max_depth=8, brdf_samples=2, aperture 0.2 (DoF),
glossy floor/doors/cylinder, Cook-Torrance doors, 4 rectangle area lights + window point light.
One step = one full frame; two frames are in flight on alternating streams (--inflight). At N>1
the frame is tile-split over the ranks (multigpu.FrameSplit: hashed groups of 8x8 tiles, 2x2 for
pixels of several 64-sample chunks) and the finished slabs are gathered to rank 0 over RCCL (strong
scaling: the total work per step is one frame at every N).

value = W*H*spp*steps / max-over-ranks wall time of the timed region (scene resident on the
GPU, output in HBM; no host transfers inside).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (xRes, yRes, antialias_samples, max_depth, brdf_samples, use_model)
    "c3": (1920, 1080, 64, 8, 2, 0),
    "c2": (800, 600, 16, 4, 2, 0),
    # C4: the full scene incl. the OBJ models (substitute meshes, tools/gen_models.py), 256 spp
    "c4": (1920, 1080, 256, 8, 2, 1),
}


def build_globals(dt, cfg):
    g = dt.globals_default()
    xres, yres, aa, depth, brdf, models = CONFIGS[cfg]
    g.use_model = models
    built = dt.build_scene("final", 240, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth, g.brdf_samples = xres, yres, aa, depth, brdf
    return g, built


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(dt, cfg, frac_world, scene, dev, all_cores=False):
    """The CPU oracle (the reference loop restated in C, same RNG) on a bounded, spatially uniform
    sample of the same frame: rank 0's share of a `frac_world`-way tile split. SURVEY §8(d): the
    host's cores (OpenMP dynamic), median of 3 after 1 warm-up, plus 1 core. The GPU renders the
    same share into a slab beside it, and the two are compared (parity of the timed config), and the
    oracle counts the include/dt_work.h events of the reference's loop on it."""
    import statistics

    import numpy as np
    import torch

    import oracle
    g, built = build_globals(dt, cfg)
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    # the GPU box allots its CPU share through OMP_NUM_THREADS (16 per GPU there, while nproc shows the
    # whole machine); elsewhere every core of the affinity mask
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(omp, affinity) if omp > 0 else affinity
    tile = dt.tiles(rank=0, world=frac_world, layout=dt.DT_OUT_SLAB)
    n = dt.slab_floats(g, tile)
    out = np.zeros(n, dtype=np.float32)
    _, st, work = oracle.render_work(built, g, 240, tile, out=out, nthreads=threads)   # warm-up (+ event counts)
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        _, st = oracle.render(built, g, 240, tile, out=out, nthreads=threads)
        times.append(time.perf_counter() - t0)
    dt_s = statistics.median(times)
    # single core, on a 16x smaller share of the same split
    tile1 = dt.tiles(rank=0, world=frac_world * 16, layout=dt.DT_OUT_SLAB)
    out1 = np.zeros(dt.slab_floats(g, tile1), dtype=np.float32)
    t1 = time.perf_counter()
    _, st1 = oracle.render(built, g, 240, tile1, out=out1, nthreads=1)
    dt1 = time.perf_counter() - t1
    # parity of the timed config: the product path on the same share
    gslab = torch.zeros(n, dtype=torch.float32, device=dev)
    gst = dt.render(scene, g, 240, gslab, tile)
    diff = np.abs(gslab.cpu().numpy().astype(np.float64) - out.astype(np.float64))
    parity = {"pixels": int(st.pixels), "samples": int(st.samples), "max_abs": float(diff.max()),
              "frac_gt_1e-4": float((diff > 1e-4).mean()),
              "same_rays": bool(gst.rays == st.rays and gst.shadow_rays == st.shadow_rays),
              "sample": "rank 0's share of a %d-way tile split of the timed frame, GPU slab vs oracle slab" % frac_world}
    cpu = {"value": round(st.samples / dt_s / 1e6, 4), "unit": "Mpixel-samples/s", "cores": threads,
           "kind": "port", "nproc": os.cpu_count(), "affinity_cpus": affinity, "omp_num_threads": omp or None,
           "cpu_model": _cpu_model(),
           "sample": "oracle/oracle.c (OpenMP, %d threads) on rank 0's share of a %d-way 32x32 tile split "
                     "(%d pixels x %d spp), median of 3 runs after 1 warm-up: %s s"
                     % (threads, frac_world, st.pixels, st.samples // max(st.pixels, 1),
                        "/".join("%.2f" % t for t in times)),
           "single_core": {"value": round(st1.samples / dt1 / 1e6, 4), "cores": 1,
                           "sample": "rank 0's share of a %d-way split, %.1f s" % (frac_world * 16, dt1),
                           "note": "like for like with the reference, whose render loop is single-threaded "
                                   "(render_final_project.cpp:1031-1218)"}}
    if all_cores and affinity > threads:
        # every core of the affinity mask; off by default on the GPU box, whose pool
        # rules give one GPU's job a 16-core share of the node (OMP_NUM_THREADS) even though the
        # affinity mask shows all of the node's cores
        ta = []
        for _ in range(3):
            t0 = time.perf_counter()
            _, sta = oracle.render(built, g, 240, tile, out=out, nthreads=affinity)
            ta.append(time.perf_counter() - t0)
        cpu["all_cores"] = {"value": round(sta.samples / statistics.median(ta) / 1e6, 4), "cores": affinity,
                            "sample": "same share, median of 3: %s s" % "/".join("%.2f" % t for t in ta)}
    else:
        cpu["all_cores"] = {"measured": False, "cores": affinity,
                            "reason": "the job's CPU share is OMP_NUM_THREADS=%s of the %d cores in the affinity "
                                      "mask; bench.py --cpu-all-cores times every core" % (omp or None, affinity)
                            if affinity > threads else "the threads above are every core of the affinity mask"}
    return cpu, parity, work, st.samples


def end_to_end_ms(dt, cfg, dev):
    """One frame end to end as a caller of the ABI sees it: host scene build
    (buildFinal + BVH + flatten), upload, render, D2H of the ppmOut image; file write excluded."""
    import torch
    out = None
    times = []
    for _ in range(3):   # median of 3 (the output buffer is pinned once, outside the timing)
        t0 = time.perf_counter()
        g, built = build_globals(dt, cfg)
        scene = dt.Scene(built, g)
        if out is None:
            t_pin = time.perf_counter()
            out = torch.empty(3 * g.xRes * g.yRes, dtype=torch.float32, pin_memory=True)
            t0 += time.perf_counter() - t_pin
        dt.render(scene, g, 240, out.numpy())
        times.append(time.perf_counter() - t0)
        scene.close()
    return round(sorted(times)[1] * 1e3, 3)


def counter_fp64(pmc, kernel_ms):
    """The FP64 rate the PMC counters give for the trace kernel: the committed
    profile's FP64 VALU instructions per launch (ADD + MUL + TRANS + 2 FMA, wave instructions) x 64
    lanes x the VALU lane utilisation, / this run's kernel time. A cross-check of the dt_work.h weight
    table: the two rates are computed from independent data (event counts x weights, hardware
    counters) and should agree."""
    f = (pmc or {}).get("f64_insts_per_launch") or {}
    lanes = (pmc or {}).get("valu_lane_utilisation")
    if not f or not lanes or not kernel_ms:
        return None
    insts = f.get("add", 0) + f.get("mul", 0) + f.get("trans", 0) + 2 * f.get("fma", 0)
    flops = insts * 64 * lanes
    from distraytracer_amd import work as W
    r = {"achieved": round(flops / (kernel_ms / 1e3) / 1e12, 4), "unit": "TFLOP/s",
         "frac": round(flops / (kernel_ms / 1e3) / 1e12 / W.PEAK_FP64_TFLOPS, 5),
         "flops_per_launch": flops, "profile": "profiles/%s_summary.json" % pmc.get("tag"),
         "formula": "(SQ_INSTS_VALU_ADD_F64 + MUL_F64 + TRANS_F64 + 2 FMA_F64) x 64 x lane utilisation / kernel_ms"}
    if pmc.get("valu_insts_per_launch"):
        r["f64_share_of_valu_insts"] = round((insts - f.get("fma", 0)) / pmc["valu_insts_per_launch"], 4)
    return r


def valu_roofline(cfg, kernel_ms, samples, ref_work=None, ref_samples=0, pmc=None, world=1):
    """the binding roofline is the VALU. achieved = the include/dt_work.h events the
    trace kernel executes for this frame (counted by the diagnostic library in a child process) x
    their weights, / the trace kernel's HIP-event time; against the MI355X FP64 vector peak. Beside
    it: the counter-derived FP64 rate of the committed PMC profile (counter_fp64) and the reference
    loop's count for the same frame (the oracle's, scaled from its sample). At world > 1 the counting
    run renders rank 0's share of the same split, so achieved is rank 0's GPU's rate on its share."""
    from distraytracer_amd import work as W
    dev = W.device_counts(cfg, world=world)
    if dev is None:
        return None
    if world > 1:
        samples = dev["samples"]   # rank 0's share of the timed frame, counted as the timed launch renders it
    ops = dev["ops"] * (samples / max(dev["samples"], 1))   # the counting frame is the timed frame
    achieved = ops / (kernel_ms / 1e3) / 1e12
    r = {"bound": "valu", "achieved": round(achieved, 4), "peak": W.PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
         "frac": achieved / W.PEAK_FP64_TFLOPS,
         "ops_per_launch": ops, "ops_per_sample": round(ops / samples, 2),
         "kernel": None, "kernel_ms": round(kernel_ms, 3),   # named by the caller
         "counts_per_sample": W.breakdown(dev["counts"], dev["samples"]),
         "note": "FP64-equivalent VALU operations of the events the kernel executes (include/dt_work.h "
                 "weights x libdt_work.so counts) / the trace kernel's HIP-event time, against the "
                 "78.6 TFLOP/s FP64 vector peak (an FMA counts 2 there and in counter_fp64)",
         "share": ("rank 0's share of a %d-way tile split (%d pixel-samples per frame)" % (world, samples)
                   if world > 1 else "the whole frame")}
    cf = counter_fp64(pmc, kernel_ms)
    if cf is not None:
        cf["ratio_to_weighted"] = round(cf["achieved"] / achieved, 4) if achieved else None
        r["counter_fp64"] = cf
    if ref_work is not None and ref_samples:
        ref_ops = W.price(ref_work) / ref_samples
        r["reference_loop"] = {"ops_per_sample": round(ref_ops, 2),
                               "equivalent_tflops": round(ref_ops * samples / (kernel_ms / 1e3) / 1e12, 4),
                               "note": "the reference's own loop (every leaf its boxes pass, the sky per "
                                       "missing sample), counted by the oracle on the cpu_baseline sample"}
    return r


def trace_kernel_name(spp, models):
    """the trace kernel dt_render launches for the bench configs (frame 240, a still frame;
    dt_api.cpp enqueue_render): the 5-wave build at one pixel per wave, spp >= 64, unless DT_W5 says
    otherwise; the room build without OBJ models, the *_mesh build with them (C4)"""
    e = os.environ.get("DT_W5")
    ppw = 64 // min(spp, 64)
    name = "dt_trace_kernel_w5" if ppw <= 8 and (e[:1] == "1" if e else spp >= 64) else "dt_trace_kernel"
    return name + "_mesh" if models else name


def load_pmc_traffic():
    """HBM bytes per trace launch from the committed rocprofv3 PMC summary (profiles/), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_trace_summary.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            d = json.load(f)
        return d
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 10 timed frames (0.33 s of C3): with two frames in flight the first launch runs alone, which
    # 3 steps weighed at ~1% of the frame time (profiles/r06fa_bench.json against r06fa_torchrun_n1.json)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-frac", type=int, default=8, help="CPU baseline renders 1/N of the tiles")
    ap.add_argument("--cpu-all-cores", action="store_true",
                    help="also time the CPU baseline on every core of the affinity mask (not the GPU box's default)")
    ap.add_argument("--no-roofline", action="store_true", help="skip the VALU work count (child process)")
    ap.add_argument("--inflight", type=int, default=None, choices=(1, 2),
                    help="frames in flight per rank (2, the default: alternating streams and scene objects, "
                         "DESIGN.md §7)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import distraytracer_amd as dt
    from distraytracer_amd.multigpu import FrameSplit, GatherPipeline

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # one rank per GPU: RCCL refuses two ranks on one device, so a node with fewer GPUs than
    # ranks is an error here, not something to fold onto fewer devices
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    if local >= ndev:
        raise SystemExit("bench.py: LOCAL_RANK %d but only %d visible GPU(s); run one rank per GPU" % (local, ndev))
    torch.cuda.set_device(local)
    # launched by torch.distributed.run (WORLD_SIZE set): the tile split + RCCL gather path runs at
    # every world size, N=1 included (a 1-GPU box rehearses the collective code path that way)
    distributed = "WORLD_SIZE" in os.environ
    if distributed:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    g, built = build_globals(dt, args.config)
    scene = dt.Scene(built, g)
    split = FrameSplit(g, world, rank)
    W, H = g.xRes, g.yRes
    spp = int(int(g.antialias_samples ** 0.5) ** 2)
    dev = torch.device("cuda", local)
    # two frames in flight at every N: frame k+1's waves start on the CUs frame k's longest items leave
    # idle. N = 1: C2 +3.3% (its kernel is bounded by a column of 30x-mean items, a glossy cascade of
    # 6.6 rays per sample), C3 and C4 +-0.1% (profiles/r06j_*)
    inflight = args.inflight or 2
    if not distributed:
        # N = 1: with two frames in flight, frame k renders into images[k % 2] on streams[k % 2]
        images = [torch.zeros(3 * W * H, dtype=torch.float32, device=dev) for _ in range(inflight)]
        image = images[0]
        streams1 = [torch.cuda.Stream(dev) for _ in range(2)] if inflight == 2 else None
        tile = dt.tiles()
    else:
        # double-buffered slabs: frame k's gather (RCCL, async) overlaps frame k+1's render
        # with two frames in flight, frame k renders on streams[k % 2] with a scene object of its own
        # (its own launch record and queue word): frame k+1's waves fill the CUs frame k's tail
        # leaves idle (C3's 1/8 share: -2.1% per frame, profiles/r03ap_philox_mad64_overlap.log)
        streams = [torch.cuda.Stream(dev) for _ in range(2)] if inflight == 2 else None
        pipe = GatherPipeline(split, [torch.zeros(split.slab_floats, dtype=torch.float32, device=dev)
                                      for _ in range(2)],
                              [torch.zeros(world * split.slab_floats if rank == 0 else 1, dtype=torch.float32,
                                           device=dev) for _ in range(2)],
                              torch.zeros(3 * W * H if rank == 0 else 1, dtype=torch.float32, device=dev),
                              streams=streams)
        tile = split.tile
    scenes = [scene, dt.Scene(built, g)] if inflight == 2 else [scene]
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream

    def finish_pending():
        if distributed:
            pipe.finish()

    def step(k, evs=None):
        out = images[k % len(images)] if not distributed else pipe.slab(k)
        rs = (pipe.stream(k) if distributed else (streams1[k % 2] if streams1 else None)) or stream
        if distributed:
            pipe.begin(k)
        if evs is not None:
            evs[0].record(rs)
        dt.render_async(scenes[k % len(scenes)], g, 240, out, tile, stream=rs.cuda_stream)
        if evs is not None:
            evs[1].record(rs)
        if distributed:
            pipe.submit(k)

    for sc in scenes[1:]:   # setup of the second frame-in-flight scene: its first launch, untimed
        dt.render(sc, g, 240, pipe.slab(1) if distributed else images[1], tile)
    for k in range(args.warmup):
        step(k)
    finish_pending()
    torch.cuda.synchronize()
    stats = dt.collect_stats(scene, sh)

    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k, evs[k])
    finish_pending()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if len(scenes) > 1:
        # two frames in flight on alternating streams: a frame's own event pair also spans the time
        # its waves share the GPU with the other stream's frame (the pairs summed exceed the step
        # time), so the kernel time per frame is the span from the first frame's start to the last
        # end, / K: the GPU time the K launches occupy, never above ms_per_step
        start = min(evs[0][0].elapsed_time(a) for a, _ in evs)
        end = max(evs[0][0].elapsed_time(b) for _, b in evs)
        kernel_ms = (end - start) / args.steps
        kernel_basis = "span of the %d launches / %d (two frames in flight on alternating streams)" % (
            args.steps, args.steps)
    else:
        kernel_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
        kernel_basis = "mean of the %d launches' HIP-event durations on the launch stream" % args.steps
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    lib_stats = dt.collect_stats(scene, sh)

    if rank == 0:
        samples = W * H * spp * args.steps
        value = samples / elapsed / 1e6
        # HBM roofline, as north_star asks: algorithmic bytes of one trace launch =
        # framebuffer written once, texels read, scene read
        px = lib_stats.pixels
        alg_bytes = px * 3 * 4 + lib_stats.tex_fetches * 3 + 70 * 1024
        hbm_achieved = alg_bytes / (kernel_ms / 1e3) / 1e9
        pmc = load_pmc_traffic() or {}
        if pmc.get("config", "c3") != args.config:
            pmc = {}   # the committed PMC profile is of another workload
        traffic = pmc.get("hbm_bytes_per_launch")
        hbm = {"bound": "hbm", "achieved": round(hbm_achieved, 4), "peak": 8000.0, "unit": "GB/s",
               "frac": hbm_achieved / 8000.0, "traffic": traffic,
               "traffic_source": ("profiles/%s_summary.json (2*FETCH_SIZE + WRITE_SIZE, fabric requests "
                                  "incl. Infinity-Cache hits: an upper bound on HBM bytes; mostly scratch)"
                                  % pmc.get("tag")) if traffic else None,
               "alg_bytes_per_launch": int(alg_bytes)}
        cpu, parity, ref_work, ref_samples = None, None, None, 0
        e2e = end_to_end_ms(dt, args.config, dev) if world == 1 else None
        if world == 1 and not args.no_cpu_baseline:
            cpu, parity, ref_work, ref_samples = cpu_baseline(dt, args.config, args.cpu_frac, scene, dev,
                                                              args.cpu_all_cores)
        roof = None
        if not args.no_roofline:
            # at N > 1 the work is counted on rank 0's share of the split (the frame this GPU renders);
            # the committed PMC profile is of a whole-frame launch, so counter_fp64 is N = 1 only
            roof = valu_roofline(args.config, kernel_ms, W * H * spp, ref_work, ref_samples,
                                 pmc if world == 1 and pmc.get("kernel") == trace_kernel_name(spp, g.use_model)
                                 else None, world=world)
        if roof is not None:
            roof["kernel"] = trace_kernel_name(spp, g.use_model)
            roof["kernel_ms_basis"] = kernel_basis
        if roof is None:   # no diagnostic library: the HBM line alone
            roof = dict(hbm, kernel=trace_kernel_name(spp, g.use_model), kernel_ms=round(kernel_ms, 3),
                        kernel_ms_basis=kernel_basis)
        else:
            roof["hbm"] = hbm
        if pmc.get("valu_active_per_wave_cycle"):
            roof["pmc"] = {"profile": "profiles/%s_summary.json" % pmc.get("tag"),
                           "valu_active_per_wave_cycle": pmc.get("valu_active_per_wave_cycle"),
                           "simd_busy": round(pmc.get("waves_per_simd", 4) * pmc["valu_active_per_wave_cycle"], 3),
                           "lane_utilisation": pmc.get("valu_lane_utilisation")}
        line = {
            "metric": "Mpixel-samples/s (W×H×spp/s) + wall-clock per frame, 1/2/4/8 GPU",
            "value": round(value, 3),
            "unit": "Mpixel-samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("reference scene buildFinal(240) with substitute OBJ models (tools/gen_models.py)"
                     if g.use_model else "reference scene buildFinal(240), no OBJ models (absent, F6)"),
            "config": {"workload": "buildFinal(240) %dx%d, %d spp, depth %d, brdf_samples %d, DoF aperture 0.2, "
                                   "glossy + Cook-Torrance + 4 area lights" % (W, H, spp, g.max_depth,
                                                                              g.brdf_samples),
                       "name": args.config, "use_model": int(g.use_model),
                       "frame": 240, "xRes": W, "yRes": H, "spp": spp, "max_depth": g.max_depth,
                       "parallelism": ("tile-split x%d + RCCL gather, %d frame(s) in flight" % (world, len(scenes))
                                       if distributed else "single GPU, %d frame(s) in flight" % len(scenes))},
            "roofline": roof,
            "cpu_baseline": cpu,
            "parity": parity,
            "end_to_end_ms_per_frame": e2e,
            "work": {"rays_per_sample": round(lib_stats.rays / max(lib_stats.samples, 1), 3),
                     "shadow_rays_per_sample": round(lib_stats.shadow_rays / max(lib_stats.samples, 1), 3),
                     "stack_overflows": lib_stats.stack_overflows, "nan_pixels": lib_stats.nan_pixels},
        }
        print(json.dumps(line), flush=True)
    for sc in scenes:
        sc.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
