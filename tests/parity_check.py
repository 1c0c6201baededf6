"""The parity assertion every -m gpu oracle test uses (north_star: "within 1e-4 per-channel float
tolerance" on the ppmOut floats, render_final_project.cpp:1213-1217 `ppmOut[...] = clamp(c)*255`).

assert_parity bounds the LARGEST per-channel difference, not a fraction of channels: one channel
off by more than 1e-4 fails the test. NaN channels must coincide exactly (the reference's own NaN
pixels, Q25, are reproduced, never introduced); a test passes `nan_ok=True` only where the scene
is built to produce them, and says why. Each comparison appends one line to the file named by
DT_PARITY_LOG (label, channels, NaN channels, max|diff|, channels not bit-identical), which the GPU
runs commit under profiles/ (profiles/r04*_parity.log).
"""
import os
import time

import numpy as np

TOL = 1e-4


def _log(line):
    path = os.environ.get("DT_PARITY_LOG")
    if not path:
        return
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(path, "a") as f:
        f.write(line + "\n")


def assert_parity(label, gpu, ref, nan_ok=False, tol=TOL):
    """max |gpu - ref| <= tol over every channel; NaN masks equal (and empty unless nan_ok)."""
    gpu = np.asarray(gpu, dtype=np.float64).reshape(-1)
    ref = np.asarray(ref, dtype=np.float64).reshape(-1)
    assert gpu.shape == ref.shape, "%s: %s vs %s channels" % (label, gpu.shape, ref.shape)
    gn, rn = np.isnan(gpu), np.isnan(ref)
    ok = ~(gn | rn)
    diff = np.abs(gpu[ok] - ref[ok])
    mx = float(diff.max()) if diff.size else 0.0
    n_ne = int((gpu[ok] != ref[ok]).sum())
    line = "%s  %s: channels=%d nan=%d max|diff|=%.6g not_bit_identical=%d" % (
        time.strftime("%H:%M:%S"), label, gpu.size, int(rn.sum()), mx, n_ne)
    print(line)
    _log(line)
    assert np.array_equal(gn, rn), "%s: NaN channels differ (gpu %d, oracle %d)" % (label, int(gn.sum()), int(rn.sum()))
    if not nan_ok:
        assert not rn.any(), "%s: %d NaN channels" % (label, int(rn.sum()))
    assert mx <= tol, "%s: max|diff| %.6g > %g" % (label, mx, tol)
    return mx


def log_equal(label, a, b):
    """GPU-vs-GPU variants (acceleration structures against reference-tree walks): bit for bit."""
    a = np.asarray(a)
    b = np.asarray(b)
    same = bool(np.array_equal(a, b, equal_nan=True)) if a.dtype.kind == "f" else bool(np.array_equal(a, b))
    line = "%s  %s: channels=%d bit_identical=%s" % (time.strftime("%H:%M:%S"), label, a.size, same)
    print(line)
    _log(line)
    assert same, label
