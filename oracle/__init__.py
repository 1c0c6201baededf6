"""TEST INFRASTRUCTURE ONLY — ctypes access to the CPU oracle (oracle/liboracle.so) and to the
reference-compiled harness (oracle/_ref/libref_noise.so). Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg; never by distraytracer_amd/.
The struct layouts come from the C-ABI header mirror (distraytracer_amd._lib), since the
oracle consumes the same dt_scene_desc / dt_globals the device path does."""
import ctypes
import os

import numpy as np

from distraytracer_amd._lib import BVHNode, Globals, SceneDesc, Stats, Tiles

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_NOISE_SO = os.path.join(HERE, "_ref", "libref_noise.so")

_o = None


def oracle():
    global _o
    if _o is None:
        if not os.path.exists(ORACLE_SO):
            raise RuntimeError("oracle not built: make -C oracle")
        o = ctypes.CDLL(ORACLE_SO)
        P = ctypes.POINTER
        for f in ("or_noise3d", "or_smoothed3d"):
            getattr(o, f).restype = ctypes.c_double
            getattr(o, f).argtypes = [ctypes.c_int] * 4
        o.or_interpolated_noise3d.restype = ctypes.c_double
        o.or_interpolated_noise3d.argtypes = [ctypes.c_int] + [ctypes.c_double] * 3
        o.or_value_noise3d.restype = ctypes.c_double
        o.or_value_noise3d.argtypes = [ctypes.c_double] * 3
        o.or_cloud_color.argtypes = [P(Globals), P(ctypes.c_double), P(ctypes.c_double), ctypes.c_float,
                                     P(ctypes.c_double)]
        o.or_sky_color.argtypes = [P(Globals), P(ctypes.c_double), P(ctypes.c_double)]
        o.or_philox4x32.argtypes = [P(ctypes.c_uint32), P(ctypes.c_uint32), P(ctypes.c_uint32)]
        o.or_u01.restype = ctypes.c_double
        o.or_u01.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        o.or_render_sky.restype = ctypes.c_int
        o.or_render_sky.argtypes = [P(Globals), ctypes.c_float, P(Tiles), ctypes.c_void_p, ctypes.c_int]
        o.or_bvh.restype = ctypes.c_int
        o.or_bvh.argtypes = [P(SceneDesc), P(Globals), P(BVHNode), ctypes.c_int, P(ctypes.c_int), ctypes.c_int,
                             P(ctypes.c_int), P(ctypes.c_int)]
        o.or_render.restype = ctypes.c_int
        o.or_render.argtypes = [P(SceneDesc), P(Globals), ctypes.c_int, P(Tiles), ctypes.c_void_p, ctypes.c_int,
                                P(Stats)]
        o.or_render_work.restype = ctypes.c_int
        o.or_render_work.argtypes = [P(SceneDesc), P(Globals), ctypes.c_int, P(Tiles), ctypes.c_void_p, ctypes.c_int,
                                     P(Stats), P(ctypes.c_uint64)]
        o.or_primary_hit.restype = ctypes.c_int
        o.or_primary_hit.argtypes = [P(SceneDesc), P(Globals), ctypes.c_int, ctypes.c_longlong, ctypes.c_longlong,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        o.or_sample_color.restype = ctypes.c_int
        o.or_sample_color.argtypes = [P(SceneDesc), P(Globals), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, P(ctypes.c_double), P(ctypes.c_int)]
        _o = o
    return _o


def ref_noise():
    """The reference's noise.h compiled as-is (None when /root/reference was never built here)."""
    if not os.path.exists(REF_NOISE_SO):
        return None
    r = ctypes.CDLL(REF_NOISE_SO)
    for f in ("ref_Noise3D", "ref_Smoothed3D"):
        getattr(r, f).restype = ctypes.c_double
        getattr(r, f).argtypes = [ctypes.c_int] * 4
    r.ref_InterpolatedNoise3D.restype = ctypes.c_double
    r.ref_InterpolatedNoise3D.argtypes = [ctypes.c_int] + [ctypes.c_double] * 3
    r.ref_ValueNoise_3D.restype = ctypes.c_double
    r.ref_ValueNoise_3D.argtypes = [ctypes.c_double] * 3
    return r


def _desc_ptr(desc):
    return desc._ptr if hasattr(desc, "_ptr") else ctypes.pointer(desc)


def render(desc, g, frame, tile, out=None, nthreads=0):
    if out is None:
        out = np.zeros(3 * g.xRes * g.yRes, dtype=np.float32)
    st = Stats()
    rc = oracle().or_render(_desc_ptr(desc), ctypes.byref(g), int(frame), ctypes.byref(tile),
                            ctypes.c_void_p(out.ctypes.data), int(nthreads), ctypes.byref(st))
    if rc:
        raise RuntimeError("or_render failed %d" % rc)
    return out, st


def render_work(desc, g, frame, tile, out=None, nthreads=0):
    """render(), also returning the include/dt_work.h event counts of the reference's loop
    (numpy uint64[DT_WK_N])"""
    from distraytracer_amd.work import N_EVENTS
    if out is None:
        out = np.zeros(3 * g.xRes * g.yRes, dtype=np.float32)
    st = Stats()
    work = np.zeros(N_EVENTS, dtype=np.uint64)
    rc = oracle().or_render_work(_desc_ptr(desc), ctypes.byref(g), int(frame), ctypes.byref(tile),
                                 ctypes.c_void_p(out.ctypes.data), int(nthreads), ctypes.byref(st),
                                 work.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    if rc:
        raise RuntimeError("or_render_work failed %d" % rc)
    return out, st, work


def render_sky(g, frame, tile, out=None, nthreads=0):
    if out is None:
        out = np.zeros(3 * g.xRes * g.yRes, dtype=np.float32)
    rc = oracle().or_render_sky(ctypes.byref(g), float(frame), ctypes.byref(tile),
                                ctypes.c_void_p(out.ctypes.data), int(nthreads))
    if rc:
        raise RuntimeError("or_render_sky failed %d" % rc)
    return out


def bvh(desc, g):
    o = oracle()
    nn, ni = ctypes.c_int(), ctypes.c_int()
    o.or_bvh(_desc_ptr(desc), ctypes.byref(g), None, 0, None, 0, ctypes.byref(nn), ctypes.byref(ni))
    nodes = (BVHNode * max(nn.value, 1))()
    idx = (ctypes.c_int * max(ni.value, 1))()
    o.or_bvh(_desc_ptr(desc), ctypes.byref(g), nodes, nn.value, idx, ni.value, ctypes.byref(nn), ctypes.byref(ni))
    return list(nodes)[:nn.value], list(idx)[:ni.value]


def sample_color(desc, g, frame, x, y, sample):
    col = (ctypes.c_double * 3)()
    hit = ctypes.c_int()
    rc = oracle().or_sample_color(_desc_ptr(desc), ctypes.byref(g), int(frame), x, y, sample, col, ctypes.byref(hit))
    if rc:
        raise RuntimeError("or_sample_color failed %d" % rc)
    return list(col), bool(hit.value)


def primary_hit(desc, g, frame, first, n, nthreads=0):
    """closest hits of the intersection micro-benchmark's rays first .. first+n-1 (or_primary_hit):
    (shape int32[n], t float32[n])"""
    import numpy as np
    shape = np.empty(n, dtype=np.int32)
    t = np.empty(n, dtype=np.float32)
    rc = oracle().or_primary_hit(_desc_ptr(desc), ctypes.byref(g), int(frame), int(first), int(n),
                                 ctypes.c_void_p(shape.ctypes.data), ctypes.c_void_p(t.ctypes.data), int(nthreads))
    if rc:
        raise RuntimeError("or_primary_hit failed %d" % rc)
    return shape, t
