"""Frame-parallel C5 on N GPUs from measured per-frame times: the makespan of the assignments
tools/animate.py offers, replayed on one GPU's per-frame log (a simulation of the N > 1 schedule,
not a multi-GPU measurement; no 8-GPU node has been available to this repo).

  python tools/c5_schedule.py profiles/r03d_c5_full.log [--gpus 1,2,4,8]

static  frame n on rank n % N (round 2)
lpt     a shared queue in descending order of the cost table the run uses (data/c5_frame_cost.json),
        each rank taking the next frame when it finishes one (tools/animate.py --split frames)
The host build of frame n+1 overlaps frame n's render, so a rank's time is its render times plus
its first frame's host build."""
import argparse
import heapq
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(path):
    rows = {}
    for line in open(path):
        if line.startswith('{"n"'):
            r = json.loads(line)
            rows[r["n"]] = (r["host_ms"], r["render_ms"])
    return rows


def makespan(rows, assign_order, n_gpus, dynamic):
    if not dynamic:
        per = [0.0] * n_gpus
        first = [None] * n_gpus
        for n in sorted(rows):
            r = n % n_gpus
            if first[r] is None:
                first[r] = rows[n][0]
            per[r] += rows[n][1]
        return max(p + (f or 0) for p, f in zip(per, first))
    heap = [(0.0, r) for r in range(n_gpus)]
    started = set()
    for n in assign_order:
        t, r = heapq.heappop(heap)
        if r not in started:
            started.add(r)
            t += rows[n][0]
        heapq.heappush(heap, (t + rows[n][1], r))
    return max(t for t, _ in heap)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("log")
    ap.add_argument("--gpus", default="1,2,4,8")
    a = ap.parse_args()
    rows = load(a.log)
    cost = json.load(open(os.path.join(ROOT, "data", "c5_frame_cost.json")))["render_ms"]
    order = sorted(rows, key=lambda n: -float(cost.get(str(n), 0.0)))
    total = sum(r for _, r in rows.values())
    out = {"log": a.log, "frames": len(rows), "render_s_one_gpu": round(total / 1e3, 2),
           "longest_frame_s": round(max(r for _, r in rows.values()) / 1e3, 3), "schedules": {}}
    for n in (int(v) for v in a.gpus.split(",")):
        s = makespan(rows, None, n, False) / 1e3
        d = makespan(rows, order, n, True) / 1e3
        out["schedules"][n] = {"static_s": round(s, 2), "static_frames_per_s": round(len(rows) / s, 2),
                               "lpt_s": round(d, 2), "lpt_frames_per_s": round(len(rows) / d, 2),
                               "lpt_efficiency": round(total / 1e3 / n / d, 3)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
