"""Device numerics of the vector normalisation every kernel uses (dt_math.h normalized: Eigen's
v / sqrt((x*x + y*y) + z*z)) against correctly rounded division and square root (numpy's
float64), bit for bit, signed zeros and extreme magnitudes included. Guards any change to the
device division sequence (a shared-reciprocal variant passed this and was dropped for speed,
DESIGN.md §8)."""
import ctypes

import numpy as np
import pytest

import distraytracer_amd as dt

pytestmark = pytest.mark.gpu


def _reference(v):
    n = (v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1]) + v[:, 2] * v[:, 2]
    out = v.copy()
    pos = n > 0
    s = np.sqrt(n[pos])
    out[pos] = v[pos] / s[:, None]
    return out


def _device(v):
    v = np.ascontiguousarray(v, dtype=np.float64)
    out = np.empty_like(v)
    P = ctypes.POINTER(ctypes.c_double)
    dt.check(dt.lib.dt_debug_normalize(v.ctypes.data_as(P), out.ctypes.data_as(P), len(v)), "dt_debug_normalize")
    return out


def test_normalize_bit_exact(cuda):
    rng = np.random.default_rng(7)
    parts = [rng.normal(size=(200000, 3)),                                    # directions
             rng.normal(size=(100000, 3)) * 10.0 ** rng.integers(-6, 7, size=(100000, 1)),   # scales
             rng.uniform(-1, 1, size=(100000, 3)) * 10.0 ** rng.integers(-300, 300, size=(100000, 3)),  # wild
             np.array([[0.0, 1.0, 0.0], [-0.0, 1.0, 0.0], [0.0, -0.0, 5.0], [-0.0, -0.0, -3.0],
                       [1e-200, 1.0, 0.0], [1e-320, 1.0, 2.0], [1e200, 1e200, 1.0], [3.0, 4.0, 0.0],
                       [0.0, 0.0, 0.0], [-0.0, 0.0, -0.0], [1e-160, 0.0, 0.0], [2.0 ** -600, 2.0 ** -600, 0.0]])]
    # axis-aligned and two-axis vectors (exact zeros with either sign), as the scenes' normals are
    ax = rng.normal(size=(50000, 3))
    ax[rng.random(size=ax.shape) < 0.4] = 0.0
    ax[rng.random(size=ax.shape) < 0.2] *= -0.0
    parts.append(ax)
    v = np.concatenate(parts)
    with np.errstate(over="ignore", under="ignore", invalid="ignore"):
        ref = _reference(v)
    got = _device(v)
    bad = got.view(np.uint64) != ref.view(np.uint64)
    bad &= ~(np.isnan(got) & np.isnan(ref))
    assert not bad.any(), "first mismatch: %r -> %r vs %r" % (v[bad.any(axis=1)][0], got[bad.any(axis=1)][0],
                                                             ref[bad.any(axis=1)][0])
