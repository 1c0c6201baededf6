"""Diagnostic: where dt_trace_kernel touches scratch, from the compiler's -S output.

    make -C distraytracer_amd/csrc asm
    python tools/isa_loops.py distraytracer_amd/csrc/build/dt_kernels.s

For every loop the compiler annotates ("in Loop: Header=BB0_n") prints the line range, the
scratch accesses (spill/stack traffic) and the VALU count inside it, innermost loops first; then
the scratch stores and loads bucketed by the innermost loop holding them (a store inside the
DFS-step loop runs once per rayColor call and lane, one inside the item loop once per pixel).
"""
import collections
import re
import sys


def loops(lines):
    inloop = collections.defaultdict(list)
    for i, line in enumerate(lines):
        h = re.search(r"in Loop: Header=BB\d+_(\d+) Depth=(\d+)", line)
        if h:
            inloop[h.group(1)].append(i)
    rows = []
    for h, idx in inloop.items():
        a, b = min(idx), max(idx)
        j = b + 1
        while j < len(lines) and not re.match(r"^\.LBB\d+_\d+:", lines[j]) and not lines[j].startswith("; %bb"):
            j += 1
        rows.append((j - a, h, a, j))
    return sorted(rows)


def main(path, kernel="dt_trace_kernel"):
    text = open(path).read()
    m = re.search(r"^%s:.*?s_endpgm" % kernel, text, re.S | re.M)
    lines = (m.group(0) if m else text).split("\n")
    rows = loops(lines)
    for n, h, a, j in rows:
        body = lines[a:j]
        sc = sum(1 for x in body if "scratch_" in x)
        v = sum(1 for x in body if x.strip().startswith("v_"))
        print("loop BB0_%s lines %d-%d: scratch %d, valu %d" % (h, a, j, sc, v))

    def innermost(i):
        for n, h, a, j in rows:
            if a <= i < j:
                return "BB0_%s (%d lines)" % (h, n)
        return "outside loops"
    for kind in ("scratch_store", "scratch_load"):
        c = collections.Counter(innermost(i) for i, x in enumerate(lines) if kind in x)
        print("%s by innermost loop (total %d):" % (kind, sum(c.values())))
        for k, v in c.most_common():
            print("  %-28s %d" % (k, v))


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]))
