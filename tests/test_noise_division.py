"""The device's value noise (dt_kernels.hip noise3d) replaces noise.h's `t / 1073741823.0`
(noise.h:43) by a reciprocal product with one fma correction step. This checks, for every
t in [0, 2^31) -- the whole range of the masked hash -- that it yields the correctly rounded
quotient, so the noise stays bit-identical to the reference's (tools/noise_div_check.c)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_noise_division_exhaustive(tmp_path):
    exe = str(tmp_path / "noise_div_check")
    subprocess.check_call(["gcc", "-O2", "-fopenmp", "-ffp-contract=off",
                           os.path.join(ROOT, "tools", "noise_div_check.c"), "-o", exe, "-lm"])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and out.stdout.strip() == "0", out.stdout + out.stderr
