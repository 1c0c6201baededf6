"""Compare the instruction streams of two `hipcc -S` outputs (directives, comments and metadata
dropped): were two source revisions compiled to the same code? Usage: asm_diff.py a.s b.s"""
import sys


def insns(path):
    out = []
    for line in open(path):
        t = line.split(";")[0].rstrip()
        s = t.strip()
        if not s or s.startswith(".") and not s.startswith(".LBB") or s.startswith("//"):
            continue
        if s.endswith(":") and not s.startswith(".LBB"):
            continue
        out.append(s)
    return out


a, b = insns(sys.argv[1]), insns(sys.argv[2])
same = a == b
print("%s: %d vs %d instruction lines, %s" % (sys.argv[2], len(a), len(b), "identical" if same else "DIFFERENT"))
if not same:
    import difflib
    for i, l in enumerate(difflib.unified_diff(a, b, lineterm="", n=1)):
        if i > 40:
            break
        print(l)
sys.exit(0 if same else 1)
