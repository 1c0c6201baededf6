"""Per-variant trace-kernel counters from tools/ab_round.sh PMC=1 (gpurun_out/<TAG>/pmc_<v>/):
one row per variant, values per launch of the trace kernel (dispatches averaged)."""
import collections
import csv
import glob
import os
import sys


def read(d, kernel):
    acc = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if not r["Kernel_Name"].startswith(kernel):
                continue
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add(r["Dispatch_Id"])
    return {k: v / max(len(disp[k]), 1) for k, v in acc.items()}


def main(tag, kernel="dt_trace_kernel_w5"):
    base = os.path.join("gpurun_out", tag)
    rows = {}
    for d in sorted(glob.glob(os.path.join(base, "pmc_*"))):
        if os.path.isdir(d):
            rows[os.path.basename(d)[4:]] = read(d, kernel)
    keys = sorted({k for r in rows.values() for k in r})
    print("%-12s" % "variant" + "".join("%16s" % k.replace("SQ_INSTS_", "").replace("SQ_", "")[:15] for k in keys))
    for v, r in rows.items():
        print("%-12s" % v + "".join("%16.4g" % r.get(k, 0) for k in keys))
    if "base" in rows:
        print("relative to base:")
        for v, r in rows.items():
            print("%-12s" % v + "".join("%16.4f" % (r.get(k, 0) / rows["base"][k] if rows["base"].get(k) else 0) for k in keys))


if __name__ == "__main__":
    main(*sys.argv[1:])
