"""C-ABI boundary checks that need no GPU: the library loads, exports every function
include/dt.h declares, the Python struct mirrors match the C layout, defaults equal the
reference's globals, and errors come back as status codes (never exceptions/exit)."""
import ctypes
import os
import re
import subprocess

import pytest

import distraytracer_amd as dt
from distraytracer_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "dt.h")


def header_functions():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dt_[a-z0-9_]+)\s*\(", src)))


def test_exports_every_declared_symbol():
    names = header_functions()
    assert len(names) >= 15
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert sorted(_lib.EXPORTS) == names


def test_abi_version():
    assert dt.lib.dt_abi_version() == 8 == _lib.ABI_VERSION


STRUCTS = {"dt_globals": _lib.Globals, "dt_shape_desc": _lib.ShapeDesc, "dt_light_desc": _lib.LightDesc,
           "dt_texture_desc": _lib.TextureDesc, "dt_scene_desc": _lib.SceneDesc, "dt_tiles": _lib.Tiles,
           "dt_stats": _lib.Stats, "dt_bvh_node": _lib.BVHNode, "dt_accel_info": _lib.AccelInfo}


def test_struct_layout_matches_c(tmp_path):
    """offsetof/sizeof of every field, from gcc on include/dt.h, vs the ctypes mirror."""
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "%s"' % HDR, "int main(void){"]
    for cname, py in STRUCTS.items():
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (cname, cname))
        for f, _ in py._fields_:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, f, cname, f))
    lines.append("return 0;}")
    c = tmp_path / "layout.c"
    c.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-o", str(exe), str(c)])
    got = dict(l.split() for l in subprocess.check_output([str(exe)]).decode().splitlines())
    for cname, py in STRUCTS.items():
        assert int(got[cname]) == ctypes.sizeof(py), cname
        for f, _ in py._fields_:
            assert int(got["%s.%s" % (cname, f)]) == getattr(py, f).offset, (cname, f)


def test_globals_default_match_reference():
    """render_final_project.cpp:48-138 initial values."""
    g = dt.globals_default()
    assert (g.xRes, g.yRes) == (1920, 1080)
    assert list(g.eye) == [-6, 0.5, 1] and list(g.lookingAt) == [0.5, 0.5, 1] and list(g.up) == [0, 1, 0]
    assert g.aspect == ctypes.c_float(1920 / 1080).value
    assert (g.near_plane, g.fov) == (1.0, 45.0)
    assert g.aperture == ctypes.c_float(0.2).value and g.focal_length == 10
    assert (g.max_depth, g.antialias_samples, g.brdf_samples, g.blur_samples, g.frame_range) == (10, 10, 2, 2, 1)
    assert (g.frame_prism, g.frame_cloud, g.frame_blur, g.total) == (960, 1952, 1600, 2400)
    assert g.c_trav == ctypes.c_float(0.33).value and g.c_isect == 1
    assert g.reflect == 1 and g.perlin_cloud == 0 and g.use_model == 1 and g.nogloss == 0
    assert g.clouddist == 10 and g.cloudhoff == ctypes.c_float(0.2).value
    assert list(g.sundir) == [0, 0.1, -1]


def test_errors_are_status_codes():
    g = dt.globals_default()
    with pytest.raises(dt.DTError, match="unknown scene"):
        dt.build_scene("nope", 0, g)
    with pytest.raises(dt.DTError, match=r"failed \(-5\)"):
        dt.build_scene("final", 240, dt.globals_default(), data_dir="/nonexistent")   # DT_E_IO
    bad = _lib.SceneDesc()
    bad.n_shapes = -1
    h = ctypes.c_void_p()
    rc = dt.lib.dt_scene_create(ctypes.byref(bad), ctypes.byref(g), ctypes.byref(h))
    assert rc == -1 and b"invalid" in dt.lib.dt_last_error()
    # a shape type the device path does not implement is refused, not mis-rendered
    s = (_lib.ShapeDesc * 1)()
    s[0].type = 99
    d = _lib.SceneDesc(1, 0, 0, 0, s, None, None)
    rc = dt.lib.dt_scene_create(ctypes.byref(d), ctypes.byref(g), ctypes.byref(h))
    assert rc == -4


def test_write_ppm_truncates(tmp_path):
    """writePPM (helpers.h:174-195): float -> unsigned char conversion truncates."""
    import numpy as np
    g = dt.globals_default()
    g.xRes, g.yRes = 2, 1
    p = tmp_path / "x.ppm"
    dt.write_ppm(str(p), g, np.array([0.0, 254.9, 255.0, 1.5, 100.99, 7.0], dtype=np.float32))
    data = p.read_bytes()
    assert data.startswith(b"P6\n2 1\n255\n")
    assert list(data[-6:]) == [0, 254, 255, 1, 100, 7]


def test_write_png_matches_ppm_pixels(tmp_path):
    """dt_write_png: an RGB PNG holding exactly writePPM's truncated bytes."""
    import struct
    import zlib
    import numpy as np
    g = dt.globals_default()
    g.xRes, g.yRes = 3, 2
    vals = np.array([0.0, 254.9, 255.0, 1.5, 100.99, 7.0, 9, 8, 7, 6, 5, 4, 3, 2, 1, 0, 128.7, 64.2],
                    dtype=np.float32)
    p = tmp_path / "x.png"
    dt.write_png(str(p), g, vals)
    data = p.read_bytes()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    w, h, depth, ctype = struct.unpack(">IIBB", data[16:26])
    assert (w, h, depth, ctype) == (3, 2, 8, 2)
    i = data.index(b"IDAT")
    n = struct.unpack(">I", data[i - 4:i])[0]
    raw = zlib.decompress(data[i + 4:i + 4 + n])
    rows = [raw[r * 10 + 1:(r + 1) * 10] for r in range(2)]
    assert list(b"".join(rows)) == [int(v) for v in vals]


def test_scene_set_kernel_null_scene():
    """dt_scene_set_kernel (ABI 4) rejects a null scene without touching a device (the value
    checks on a real scene run in tests/test_gpu_donate.py)."""
    assert dt.lib.dt_scene_set_kernel(None, 0) == -1
    assert b"null scene" in dt.lib.dt_last_error()
