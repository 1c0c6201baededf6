"""OBJ ingest pinned to the reference's own parser: the product loader (host_scenes.cpp load_obj,
exposed as dt_debug_load_obj) against tiny_obj_loader.h as the reference vendors it, through
objHelper.h's use of it (oracle/ref/obj_parse.cpp). Vertices and texcoords as the floats tinyobj's
real_t holds, and the triangles' vertex / texcoord indices: bit-identical.

The committed fixture (tests/golden/obj_tinyobj.npz, tools/gen_golden_obj.py) is what the reference
parser produced here; when oracle/_ref/obj_parse is built (this container, /root/reference present)
the reference parser is also run live."""
import ctypes
import os

import numpy as np
import pytest

import distraytracer_amd  # noqa: F401  (loads libdt.so)
from distraytracer_amd._lib import lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "obj_tinyobj.npz")


def product_parse(path):
    counts = (ctypes.c_int64 * 3)()
    assert lib.dt_debug_load_obj(path.encode(), None, 0, None, 0, None, 0, counts) == 0, lib.dt_last_error()
    nv, nt, nf = counts
    v = np.empty((nv, 3), np.float32)
    t = np.empty((nt, 2), np.float32)
    f = np.empty((nf, 6), np.int32)
    assert lib.dt_debug_load_obj(path.encode(), v.ctypes.data, nv, t.ctypes.data, nt, f.ctypes.data, nf, counts) == 0
    return v, t, f


def _same(a, b):
    return a.shape == b.shape and np.array_equal(a.view(np.uint32) if a.dtype == np.float32 else a,
                                                 b.view(np.uint32) if b.dtype == np.float32 else b)


def test_obj_ingest_matches_reference_fixture():
    g = np.load(GOLDEN, allow_pickle=False)
    for i, m in enumerate(g["models"]):
        v, t, f = product_parse(os.path.join(ROOT, "data", "models", str(m)))
        assert _same(v, g["v%d" % i]), m
        assert _same(t, g["t%d" % i]), m
        assert _same(f, g["f%d" % i]), m
        assert len(f) > 0 and (f[:, :3] >= 0).all()


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "obj_parse")),
                    reason="oracle/_ref/obj_parse not built (needs /root/reference)")
def test_obj_ingest_matches_reference_parser_live(tmp_path):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from gen_golden_obj import MODELS, tinyobj_parse
    # the committed models, and a file exercising what they do not: texcoord-less faces, v/vt/vn
    # corners, extra spaces, a comment, values with exponents and many digits
    extra = tmp_path / "extra.obj"
    extra.write_text("# comment\nv 1.0e-3 -2.5E+2 0.1234567890123\nv  0.3333333333 1 2\nv -0 5e-8 7\n"
                     "vt 0.5 0.25\nvt 1 0\nvn 0 1 0\nf 1/1/1 2/2/1 3/1/1\nf 3 2 1\n")
    for path in [os.path.join(ROOT, "data", "models", m) for m in MODELS] + [str(extra)]:
        rv, rt, rf = tinyobj_parse(path)
        v, t, f = product_parse(path)
        assert _same(v, rv) and _same(t, rt) and _same(f, rf), path
