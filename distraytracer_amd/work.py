"""The VALU roofline of the render loop: event counts x the weight table of
include/dt_work.h.

The weights and event names are parsed from the header itself, so bench.py, the diagnostic
library and anyone recomputing `roofline.achieved` use the same numbers. Device counts come from
libdt_work.so (the kernels built with -DDT_WORK_COUNTERS), loaded in a child process so the timed
process only ever loads the product libdt.so:

    python -m distraytracer_amd.work --config c3      # JSON: per-event counts of one frame
"""
import json
import os
import re
import subprocess
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
HEADER = os.path.join(os.path.dirname(_HERE), "include", "dt_work.h")
WORK_LIB = os.path.join(_HERE, "libdt_work.so")


def _parse_header(path=HEADER):
    src = open(path).read()
    enum = re.search(r"enum dt_work_event \{(.*?)\};", src, re.S).group(1)
    base = {m.group(1): int(m.group(2)) for m in re.finditer(r"(DT_WK_\w+)\s*=\s*(\d+)", enum)}
    n = base.pop("DT_WK_N")
    body = re.search(r"dt_work_weight\[DT_WK_N\]\s*=\s*\{(.*?)\};", src, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    weights = [float(v) for v in body.replace("\n", " ").split(",") if v.strip()]
    if len(weights) != n:
        raise ValueError("dt_work.h: %d weights for %d events" % (len(weights), n))
    peak = float(re.search(r"#define DT_PEAK_FP64_VECTOR_TFLOPS ([\d.]+)", src).group(1))
    # event names: the enum's bases, typed offsets spelled out
    names = [None] * n
    order = sorted(base.items(), key=lambda kv: kv[1])
    shape_types = ["", "sphere", "cylinder", "triangle", "rectangle", "rectprism_v2", "checkerboard",
                   "checkerboard_hole", "checker_cylinder", "rectprism_cyl"]
    models = ["phong", "oren_nayar", "cook_torrance", "raw"]
    for i, (name, idx) in enumerate(order):
        end = order[i + 1][1] if i + 1 < len(order) else n
        short = name[len("DT_WK_"):].lower()
        for k in range(idx, end):
            if end - idx == 1:
                names[k] = short
            elif short in ("hit_shape", "shadow_shape"):
                names[k] = "%s.%s" % (short, shape_types[k - idx] or "none")
            elif short == "brdf":
                names[k] = "brdf.%s" % models[k - idx]
            else:
                names[k] = "%s.%d" % (short, k - idx)
    return n, names, weights, peak


N_EVENTS, NAMES, WEIGHTS, PEAK_FP64_TFLOPS = _parse_header()
SKY = NAMES.index("sky")


def price(counts):
    """FP64-equivalent VALU operations of a count vector (len N_EVENTS)"""
    return float(sum(float(c) * w for c, w in zip(counts, WEIGHTS)))


def breakdown(counts, samples):
    """per pixel-sample counts and operations of the events that occur"""
    out = {}
    for name, c, w in zip(NAMES, counts, WEIGHTS):
        if c:
            out[name] = {"per_sample": round(float(c) / max(samples, 1), 4), "ops_per_sample": round(float(c) * w / max(samples, 1), 2)}
    return out


def device_counts(config, timeout=180, world=1):
    """Per-event counts of one frame of `config` executed by the diagnostic kernels (child process
    with DT_LIB=libdt_work.so); world > 1: of rank 0's share of the frame's tile split
    (multigpu.FrameSplit, as bench.py renders it). None when the diagnostic library was not built."""
    if not os.path.exists(WORK_LIB):
        return None
    # the child renders alone on this process's GPU: no torch.distributed rendezvous variables
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "MASTER_ADDR",
                        "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    env["DT_LIB"] = WORK_LIB
    r = subprocess.run([sys.executable, "-m", "distraytracer_amd.work", "--config", config,
                        "--world", str(world)], env=env,
                       cwd=os.path.dirname(_HERE), capture_output=True, text=True, timeout=timeout)
    if r.returncode != 0:
        raise RuntimeError("work counting failed: %s" % r.stderr[-2000:])
    return json.loads(r.stdout.strip().splitlines()[-1])


def _count_main():
    import argparse
    import ctypes

    import numpy as np
    import torch

    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--world", type=int, default=1, help="count rank 0's share of a WORLD-way tile split")
    args = ap.parse_args()
    sys.path.insert(0, os.path.dirname(_HERE))
    import bench
    import distraytracer_amd as dt
    from distraytracer_amd._lib import LIB_PATH
    if os.path.realpath(LIB_PATH) != os.path.realpath(WORK_LIB):
        raise SystemExit("run with DT_LIB=%s" % WORK_LIB)
    torch.cuda.set_device(0)
    g, built = bench.build_globals(dt, args.config)
    scene = dt.Scene(built, g)
    if args.world > 1:
        from distraytracer_amd.multigpu import FrameSplit
        split = FrameSplit(g, args.world, 0)
        out = torch.zeros(split.slab_floats, dtype=torch.float32, device="cuda")
        st = dt.render(scene, g, 240, out, split.tile)
    else:
        out = torch.zeros(3 * g.xRes * g.yRes, dtype=torch.float32, device="cuda")
        st = dt.render(scene, g, 240, out, dt.tiles())
    buf = (ctypes.c_uint64 * N_EVENTS)()
    dt.check(dt.lib.dt_debug_counters(scene.handle, buf, N_EVENTS), "dt_debug_counters")
    counts = np.array(list(buf), dtype=np.float64)
    counts[SKY] = st.sky_pixels   # the sky is marched once per pixel, cooperatively or per lane
    scene.close()
    print(json.dumps({"config": args.config, "world": args.world, "samples": int(st.samples), "pixels": int(st.pixels),
                      "rays": int(st.rays), "shadow_rays": int(st.shadow_rays), "sky_pixels": int(st.sky_pixels),
                      "counts": [int(c) for c in counts], "ops": price(counts),
                      "diagnostic_kernel_ms": round(st.kernel_ms, 3)}))


if __name__ == "__main__":
    _count_main()
