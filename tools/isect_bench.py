"""Intersection micro-benchmark: 2^24 primary rays of the C3 camera, closest hit
(include/dt.h dt_intersect_primary, dt_isect_kernel). Prints one JSON line: kernel ms (HIP events,
median of K launches), Mrays/s, parity of three 2^15-ray windows against the oracle's
or_primary_hit (mismatching rays: shape or float t), and the oracle's own rate on the host's
threads as the CPU reference point.

    python tools/isect_bench.py [K]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import distraytracer_amd as dt  # noqa: E402

N = 1 << 24
WIN = 1 << 15


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    g, built = bench.build_globals(dt, "c3")
    scene = dt.Scene(built, g)
    shape = torch.empty(N, dtype=torch.int32, device="cuda")
    t = torch.empty(N, dtype=torch.float32, device="cuda")
    dt.intersect_primary(scene, g, 240, 0, shape, t)   # warm-up (uploads, primary lists)
    ms = sorted(dt.intersect_primary(scene, g, 240, 0, shape, t) for _ in range(k))
    med = ms[len(ms) // 2]
    hits = float((shape >= 0).float().mean())
    out = {"bench": "isect_primary_c3", "rays": N, "kernel": "dt_isect_kernel", "reps": k,
           "kernel_ms_median": round(med, 4), "kernel_ms_min": round(ms[0], 4),
           "mrays_per_s": round(N / (med / 1e3) / 1e6, 1), "hit_fraction": round(hits, 4)}
    import oracle   # the checker and CPU reference point only
    gs, gt = shape.cpu().numpy(), t.cpu().numpy()
    bad = 0
    for first in (0, N // 2, N - WIN):
        rs, rt = oracle.primary_hit(built, g, 240, first, WIN)
        bad += int(((gs[first:first + WIN] != rs) | (gt[first:first + WIN].view(np.uint32) != rt.view(np.uint32))).sum())
    out["parity"] = {"rays_checked": 3 * WIN, "mismatches": bad}
    threads = min(int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0)),
                  len(os.sched_getaffinity(0)))
    n_cpu = 1 << 21
    oracle.primary_hit(built, g, 240, 0, 1 << 16, nthreads=threads)   # warm-up
    t0 = time.perf_counter()
    oracle.primary_hit(built, g, 240, N // 4, n_cpu, nthreads=threads)
    cpu_s = time.perf_counter() - t0
    out["cpu_oracle"] = {"mrays_per_s": round(n_cpu / cpu_s / 1e6, 2), "threads": threads,
                         "sample": "2^21 rays from ray 2^22"}
    scene.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
