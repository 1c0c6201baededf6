"""Compare rocprofv3 --pmc counters of tools/share_pmc.py's dispatches: the whole-frame repeat
launch against the sum of the WORLD share launches.
    python tools/share_pmc_cmp.py gpurun_out/<tag>/pmc*/ ..."""
import collections
import csv
import glob
import sys


def main():
    rows = collections.defaultdict(dict)   # dispatch -> counter -> value
    for d in sys.argv[1:]:
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            per = collections.defaultdict(lambda: collections.defaultdict(float))
            for r in csv.DictReader(open(f)):
                if r["Kernel_Name"].split("(")[0] != "dt_trace_kernel_w5":
                    continue
                per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
            for i, disp in enumerate(sorted(per)):
                rows[i].update(per[disp])
    order = sorted(rows)
    # dispatch 0: the warm-up render; 1: the whole frame x copies; 2..: the shares x copies
    whole, shares = rows[order[1]], [rows[i] for i in order[2:]]
    print("%-26s %14s %14s %8s" % ("counter", "whole", "sum(shares)", "ratio"))
    for c in sorted(whole):
        s = sum(x.get(c, 0.0) for x in shares)
        print("%-26s %14.4g %14.4g %8.4f" % (c, whole[c], s, s / whole[c] if whole[c] else float("nan")))
    if "TCC_HIT_sum" in whole:
        for name, x in [("whole", whole)] + [("r%d" % k, v) for k, v in enumerate(shares)]:
            h, m = x["TCC_HIT_sum"], x["TCC_MISS_sum"]
            print("L2 hit rate %-6s %.4f" % (name, h / (h + m)))


if __name__ == "__main__":
    main()
