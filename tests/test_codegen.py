"""Code-generation guard (the called-sky defect). gfx950 encodes at most a 32-bit literal
per instruction, yet with -mllvm -disable-machine-cse LLVM emits `s_mov_b64 s[..], <64-bit literal>`,
which its integrated assembler encodes with the literal's low 32 bits (often 0): the called
cloud_color_lane lost its 1.5 constants this way (tools/call_repro: every pixel of C5 frame 2200's sky
differed; only that flag, alone or with the others, reproduces it). These tests need hipcc, not a GPU:
the reproducer pins the defect, and the product's code-generation flags must not produce such an
instruction in the trace kernels."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "distraytracer_amd", "csrc")
sys.path.insert(0, os.path.join(ROOT, "tools"))
from check_literals import bad_literals  # noqa: E402

HIPCC = "/opt/rocm/bin/hipcc"
pytestmark = pytest.mark.skipif(not os.path.exists(HIPCC), reason="needs hipcc")


def _make_var(name):
    return subprocess.check_output(["make", "-s", "-C", CSRC, "var-" + name], text=True).split()


def _asm(extra, out):
    base = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
            "-fhip-fp32-correctly-rounded-divide-sqrt"]
    return subprocess.Popen([HIPCC] + base + extra + ["-I" + CSRC, "--cuda-device-only", "-S",
                            os.path.join(CSRC, "dt_kernels.hip"), "-o", out],
                            stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)


def test_reproducer_pins_the_defect(tmp_path):
    """The reproducer's TU (dt_kernels.hip DT_REPRO) under -disable-machine-cse holds unencodable
    literal moves; without that flag it holds none."""
    a, b = str(tmp_path / "cse.s"), str(tmp_path / "nocse.s")
    pa = _asm(["-DDT_REPRO=1", "-mllvm", "-disable-machine-cse"], a)
    pb = _asm(["-DDT_REPRO=1"], b)
    assert pa.wait() == 0 and pb.wait() == 0
    bad = bad_literals(open(a).read())
    assert bad and all("0x3ff8000000000000" in ins for _, ins in bad), bad   # the 1.5 of sky_color
    assert bad_literals(open(b).read()) == []


def test_product_codegen_flags_encode_every_literal(tmp_path):
    """Every trace build (csrc/Makefile TRACE_BUILDS), compiled with the Makefile's code-generation
    flags: no scalar 64-bit move of a literal wider than 32 bits."""
    codegen = _make_var("CODEGEN")
    assert "-disable-machine-cse" not in codegen
    builds = _make_var("TRACE_BUILDS")
    assert "dt_kernels_w5" in builds and "dt_kernels_w5_tunnel" in builds
    pending = list(builds)
    running = []
    while pending or running:
        while pending and len(running) < 4:
            build = pending.pop(0)
            fl = subprocess.check_output(["make", "-s", "-C", CSRC, "flags-" + build], text=True).split()
            out = str(tmp_path / (build + ".s"))
            running.append((build, out, _asm(fl + codegen, out)))
        build, out, p = running.pop(0)
        assert p.wait() == 0, build
        assert bad_literals(open(out).read()) == [], build
