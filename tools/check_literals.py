"""Scan AMDGPU assembly (hipcc --cuda-device-only -S) for scalar 64-bit moves of a literal that does
not fit 32 bits. gfx950 (like every gfx9 target) encodes at most a 32-bit literal per instruction:
`s_mov_b64 s[0:1], 0x7ff0000000000000` cannot be encoded -- llvm-mc rejects it -- yet the compiler's
integrated assembler emits it with the literal's low 32 bits, here 0 (the LLVM defect
behind the wrong colours of the called sky march, triggered by -mllvm -disable-machine-cse).

    python tools/check_literals.py file.s [...]        # exit 1 and list them if any

As a module: bad_literals(text) -> [(line number, instruction)]."""
import re
import sys

_MOV64 = re.compile(r"^\s*s_mov_b64\s+s\[\d+:\d+\],\s*(0x[0-9a-fA-F]+|-?\d+)\s*(;.*)?$")


def bad_literals(text):
    out = []
    for i, line in enumerate(text.splitlines(), 1):
        m = _MOV64.match(line)
        if not m:
            continue
        v = int(m.group(1), 0)
        if v < 0:
            v &= (1 << 64) - 1
        # inline constants (-16..64) and anything a 32-bit literal reproduces (zero-extended or, for a
        # negative value, sign-extended) are encodable
        if v <= 0xFFFFFFFF or v >= (1 << 64) - (1 << 31):
            continue
        out.append((i, line.strip()))
    return out


def main(paths):
    bad = 0
    for p in paths:
        for i, ins in bad_literals(open(p).read()):
            print("%s:%d: %s" % (p, i, ins))
            bad += 1
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
