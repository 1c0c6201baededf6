"""Overlap of trace-kernel dispatches in a rocprofv3 kernel trace (--kernel-trace, CSV output):
with frames in flight on two streams, does frame k+1's kernel start before frame k's ends (the
persistent grid's tail filled by the next frame), or do the dispatches run one after another?

    python tools/overlap.py <dir with *kernel_trace.csv> [kernel-name-substring]

Prints each dispatch's start offset, duration and overlap with the previous one (ms), then the
span of all of them against the sum of their durations."""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "dt_trace_kernel"
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if sub in r.get("Kernel_Name", ""):
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", ""),
                                 r["Kernel_Name"][:40]))
    rows.sort()
    if not rows:
        print("no dispatches of", sub)
        return
    t0 = rows[0][0]
    prev_end = None
    total = 0
    for s, e, q, n in rows:
        ov = (prev_end - s) / 1e6 if prev_end is not None else 0.0
        print("start %9.3f  dur %7.3f  queue %s  overlap-with-previous %7.3f  %s" % ((s - t0) / 1e6, (e - s) / 1e6, q, ov, n))
        prev_end = e if prev_end is None else max(prev_end, e)
        total += e - s
    span = max(e for _, e, _, _ in rows) - t0
    print("dispatches %d  span %.3f ms  sum of durations %.3f ms  mean %.3f ms  span/dispatch %.3f ms" %
          (len(rows), span / 1e6, total / 1e6, total / 1e6 / len(rows), span / 1e6 / len(rows)))


if __name__ == "__main__":
    main()
