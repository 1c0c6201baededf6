"""Opcode histogram of a trace kernel's ISA (the compiler's -S output), for the whole kernel and
for each loop the compiler annotates, innermost loops first: which VALU classes the hot loops
spend their instructions on (FP64 arithmetic, conversions, compare/select, moves, lane
read/write of spilled SGPRs, integer, FP32), and the scalar and memory instructions beside them.

    make -C distraytracer_amd/csrc asm
    python tools/isa_hist.py distraytracer_amd/csrc/build/dt_kernels_w5.s dt_trace_kernel_w5 [--top 12]

Static counts: an instruction counts once however often it runs. The dynamic mix is the PMC
profile's (tools/profile_gpu.sh: SQ_INSTS_VALU, SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64, ...)."""
import collections
import json
import re
import sys

CLASSES = [  # (class, predicate on the mnemonic), first match wins
    ("spill_lane", lambda m: m in ("v_writelane_b32", "v_readlane_b32")),
    ("readfirstlane", lambda m: m == "v_readfirstlane_b32"),
    ("f64_fma", lambda m: m.startswith("v_fma_f64") or m.startswith("v_fmac_f64")),
    ("f64_addmul", lambda m: re.match(r"v_(add|mul|sub)_f64", m) is not None),
    ("f64_minmax", lambda m: re.match(r"v_(min|max)_f64|v_max3_f64|v_min3_f64", m) is not None),
    ("f64_trans", lambda m: re.match(r"v_(rcp|rsq|sqrt|frexp|ldexp|fract|trunc|floor|ceil|rndne)_f64", m) is not None
                 or m.startswith("v_div_") or m.startswith("v_trig_preop")),
    ("f64_cmp", lambda m: m.startswith("v_cmp") and "f64" in m or m.startswith("v_cmpx") and "f64" in m
               or m.startswith("v_cmp_class_f64")),
    ("cvt", lambda m: m.startswith("v_cvt")),
    ("f32_arith", lambda m: re.match(r"v_(add|sub|mul|fma|fmac|mac|mad|min|max|min3|max3|med3)_f32", m) is not None
                 or re.match(r"v_(rcp|rsq|sqrt|exp|log|sin|cos)_f32", m) is not None or m.startswith("v_pk_")),
    ("cmp_other", lambda m: m.startswith("v_cmp")),
    ("cndmask", lambda m: m.startswith("v_cndmask")),
    ("mov", lambda m: m.startswith("v_mov") or m.startswith("v_accvgpr")),
    ("int", lambda m: m.startswith("v_")),
    ("salu", lambda m: m.startswith("s_") and not m.startswith(("s_load", "s_buffer", "s_waitcnt", "s_cbranch",
                                                                 "s_branch", "s_setprio", "s_nop", "s_endpgm"))),
    ("smem", lambda m: m.startswith(("s_load", "s_buffer"))),
    ("branch", lambda m: m.startswith(("s_cbranch", "s_branch"))),
    ("waitcnt", lambda m: m.startswith("s_waitcnt")),
    ("scratch", lambda m: m.startswith("scratch_")),
    ("vmem", lambda m: m.startswith(("global_", "buffer_", "flat_"))),
    ("lds", lambda m: m.startswith("ds_")),
    ("other", lambda m: True),
]
VALU = ("spill_lane", "readfirstlane", "f64_fma", "f64_addmul", "f64_minmax", "f64_trans", "f64_cmp", "cvt",
        "f32_arith", "cmp_other", "cndmask", "mov", "int")


def klass(m):
    for k, p in CLASSES:
        if p(m):
            return k
    return "other"


def hist(lines):
    c = collections.Counter()
    for x in lines:
        s = x.strip()
        if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
            continue
        c[klass(s.split()[0])] += 1
    return c


def fmt(c):
    v = sum(c[k] for k in VALU)
    parts = ["valu %d" % v]
    if v:
        f64 = c["f64_fma"] + c["f64_addmul"] + c["f64_trans"]
        parts.append("f64 arith %.0f%%" % (100.0 * f64 / v))
    parts += ["%s %d" % (k, c[k]) for k, _ in CLASSES if c[k]]
    return ", ".join(parts)


def main(path, kernel, top=12, as_json=False):
    text = open(path).read()
    m = re.search(r"^%s:.*?s_endpgm" % re.escape(kernel), text, re.S | re.M)
    if not m:
        raise SystemExit("kernel %s not found in %s" % (kernel, path))
    lines = m.group(0).split("\n")
    total = hist(lines)
    inloop = collections.defaultdict(list)
    depth = {}
    for i, line in enumerate(lines):
        h = re.search(r"in Loop: Header=BB\d+_(\d+) Depth=(\d+)", line)
        if h:
            inloop[h.group(1)].append(i)
            depth[h.group(1)] = int(h.group(2))
    rows = []
    for h, idx in inloop.items():
        a, b = min(idx), max(idx)
        rows.append((b - a, h, a, b + 1))
    rows.sort()
    out = {"kernel": kernel, "total": dict(total), "loops": []}
    print("%s: %s" % (kernel, fmt(total)))
    for n, h, a, b in rows[:top]:
        c = hist(lines[a:b])
        out["loops"].append({"header": "BB_%s" % h, "depth": depth[h], "lines": [a, b], "hist": dict(c)})
        print("loop BB_%s depth %d lines %d-%d: %s" % (h, depth[h], a, b, fmt(c)))
    if as_json:
        json.dump(out, open(as_json, "w"), indent=1)
    return out


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    top = 12
    js = None
    for i, a in enumerate(sys.argv):
        if a == "--top":
            top = int(sys.argv[i + 1])
        if a == "--json":
            js = sys.argv[i + 1]
    args = [a for a in args if a not in (str(top), js)]
    main(args[0], args[1] if len(args) > 1 else "dt_trace_kernel_w5", top, js)
