"""Diagnostic: per-loop instruction mix of dt_trace_kernel from the compiler's -S output.

    hipcc ... --cuda-device-only -S distraytracer_amd/csrc/dt_kernels.hip -o /tmp/k.s
    python tools/isa_loops.py /tmp/k.s

For every loop the compiler annotates ("in Loop: Header=BB0_n") prints the line range, the
scratch accesses (spill/stack traffic) and the VALU count inside it, innermost loops first.
"""
import collections
import re
import sys


def main(path):
    text = open(path).read()
    m = re.search(r"^dt_trace_kernel:.*?s_endpgm", text, re.S | re.M)
    lines = (m.group(0) if m else text).split("\n")
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
        body = lines[a:j]
        sc = sum(1 for x in body if "scratch_" in x)
        v = sum(1 for x in body if x.strip().startswith("v_"))
        rows.append((j - a, h, a, j, sc, v))
    for n, h, a, j, sc, v in sorted(rows):
        print("loop BB0_%s lines %d-%d: scratch %d, valu %d" % (h, a, j, sc, v))


if __name__ == "__main__":
    main(sys.argv[1])
