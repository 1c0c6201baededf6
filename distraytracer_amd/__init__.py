"""distraytracer_amd — MI355X-native (gfx950) render loop of distraytracer.

Python mirror of the reference's host interface over the C-ABI (include/dt.h):

    reference (render_final_project.cpp / scene.h)      here
    renderImage(filename, frame, sceneBuilder)  :965    renderImage(filename, frame, builder, g)
    renderImageCloud(filename, frame)           :1224   renderImageCloud(filename, frame, g)
    buildFinal / buildSceneSpheres / ...  (scene.h)     build_scene("final" | "spheres" | ...)
    globals (:48-137)                                   Globals / globals_default()
    writePPM (helpers.h:174)                            write_ppm

Everything computes through libdt.so's HIP kernels; a missing library or a missing GPU is
an error (there is no CPU path in this package).
"""
import ctypes

from ._lib import (DATA_DIR, DT_KERNEL_AUTO, DT_KERNEL_DONATE, DT_KERNEL_PRODUCT, DT_OUT_IMAGE, DT_OUT_SLAB, AccelInfo, BVHNode, DTError, Globals, SceneDesc,
                   Stats, Tiles, check, lib)

__all__ = ["Globals", "Tiles", "Stats", "DTError", "globals_default", "build_scene", "Scene",
           "render", "render_sky", "renderImage", "renderImageCloud", "write_ppm", "DATA_DIR",
           "DT_OUT_IMAGE", "DT_OUT_SLAB", "slab_floats", "slab_floats_max", "unpack_slabs", "tiles", "check", "lib",
           "accel_info", "DT_KERNEL_AUTO", "DT_KERNEL_PRODUCT", "DT_KERNEL_DONATE"]


def globals_default():
    """Fresh-process globals (render_final_project.cpp:48-137)."""
    g = Globals()
    lib.dt_globals_default(ctypes.byref(g))
    return g


def tiles(x0=0, y0=0, x1=0, y1=0, tile_w=32, tile_h=32, rank=0, world=1, layout=DT_OUT_IMAGE):
    return Tiles(x0, y0, x1, y1, tile_w, tile_h, rank, world, layout, 0)


class BuiltScene:
    """A dt_scene_desc owned by libdt (dt_build_scene)."""

    def __init__(self, ptr):
        self._ptr = ptr

    @property
    def desc(self):
        return self._ptr.contents

    def __del__(self):
        if getattr(self, "_ptr", None) and lib is not None:   # lib is None at interpreter exit
            lib.dt_scene_desc_free(self._ptr)
            self._ptr = None


def build_scene(name, frame, g, data_dir=DATA_DIR):
    """scene.h builders; mutates g as the reference builder mutates its globals."""
    out = ctypes.POINTER(SceneDesc)()
    check(lib.dt_build_scene(name.encode(), float(frame), ctypes.byref(g), data_dir.encode(), ctypes.byref(out)),
          "dt_build_scene(%s)" % name)
    return BuiltScene(out)


def accel_info(built, g):
    """The acceleration structures dt_scene_create would upload (trees, shadow grid), built on the
    host only: counts and content hashes (dt_accel_info_build). Build knobs are read from the
    environment (DT_SG_BLOCK, DT_SG_ORDER, DT_FAST_TREE, ...) at call time."""
    info = AccelInfo()
    desc = built._ptr if isinstance(built, BuiltScene) else ctypes.pointer(built)
    check(lib.dt_accel_info_build(desc, ctypes.byref(g), ctypes.byref(info)), "dt_accel_info_build")
    return info.as_dict()


def trace_build(built, g, frame):
    """The trace-kernel build dt_render launches for (built, g) at `frame` (automatic choice, host
    only, dt_trace_build): (kernel name, the scene's feature mask, the build's feature mask)."""
    name = ctypes.create_string_buffer(64)
    sf, bf = ctypes.c_uint32(), ctypes.c_uint32()
    desc = built._ptr if isinstance(built, BuiltScene) else ctypes.pointer(built)
    check(lib.dt_trace_build(desc, ctypes.byref(g), int(frame), name, 64, ctypes.byref(sf), ctypes.byref(bf)),
          "dt_trace_build")
    return name.value.decode(), sf.value, bf.value


class Scene:
    """Device-resident scene + reference-topology BVH (dt_scene_create). upload=False runs only the
    host half (dt_scene_prepare: no device work, safe beside a running render); upload() or the
    first render does the device half (dt_scene_upload)."""

    def __init__(self, built, g, upload=True):
        self._h = ctypes.c_void_p()
        desc = built._ptr if isinstance(built, BuiltScene) else ctypes.pointer(built)
        self._keep = built
        if upload:
            check(lib.dt_scene_create(desc, ctypes.byref(g), ctypes.byref(self._h)), "dt_scene_create")
        else:
            check(lib.dt_scene_prepare(desc, ctypes.byref(g), ctypes.byref(self._h)), "dt_scene_prepare")

    def upload(self):
        check(lib.dt_scene_upload(self._h), "dt_scene_upload")

    def set_kernel(self, kernel):
        """dt_scene_set_kernel: DT_KERNEL_AUTO (the DT_DONATE environment), DT_KERNEL_PRODUCT or
        DT_KERNEL_DONATE for this scene's renders"""
        check(lib.dt_scene_set_kernel(self._h, kernel), "dt_scene_set_kernel")

    @property
    def handle(self):
        return self._h

    def bvh(self):
        nn, ni = ctypes.c_int32(), ctypes.c_int32()
        check(lib.dt_scene_bvh(self._h, None, 0, None, 0, ctypes.byref(nn), ctypes.byref(ni)), "dt_scene_bvh")
        nodes = (BVHNode * max(nn.value, 1))()
        idx = (ctypes.c_int32 * max(ni.value, 1))()
        check(lib.dt_scene_bvh(self._h, nodes, nn.value, idx, ni.value, ctypes.byref(nn), ctypes.byref(ni)),
              "dt_scene_bvh")
        return list(nodes)[:nn.value], list(idx)[:ni.value]

    def close(self):
        if self._h:
            lib.dt_scene_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _ptr(out):
    """(address, on_device) for a torch tensor or numpy array."""
    if hasattr(out, "data_ptr"):
        if out.dtype.__str__() != "torch.float32" or not out.is_contiguous():
            raise DTError("output must be a contiguous float32 tensor")
        return ctypes.c_void_p(out.data_ptr()), 1 if out.is_cuda else 0
    import numpy as np
    if out.dtype != np.float32 or not out.flags["C_CONTIGUOUS"]:
        raise DTError("output must be a contiguous float32 array")
    return ctypes.c_void_p(out.ctypes.data), 0


def render(scene, g, frame, out, tile=None, stream=None):
    """renderImage's pixel loop into `out` (ppmOut layout, or slab layout per `tile`)."""
    st = Stats()
    p, dev = _ptr(out)
    check(lib.dt_render(scene.handle, ctypes.byref(g), int(frame), ctypes.byref(tile) if tile else None, p, dev,
                        ctypes.c_void_p(stream) if stream else None, ctypes.byref(st)), "dt_render")
    return st


def render_async(scene, g, frame, out_device, tile=None, stream=None):
    p, dev = _ptr(out_device)
    if not dev:
        raise DTError("render_async needs a device output")
    check(lib.dt_render_async(scene.handle, ctypes.byref(g), int(frame), ctypes.byref(tile) if tile else None, p,
                              ctypes.c_void_p(stream) if stream else None), "dt_render_async")


def collect_stats(scene, stream=None):
    st = Stats()
    check(lib.dt_collect_stats(scene.handle, ctypes.c_void_p(stream) if stream else None, ctypes.byref(st)),
          "dt_collect_stats")
    return st


def _ptr_typed(a, torch_dtype, np_dtype):
    if hasattr(a, "data_ptr"):
        if str(a.dtype) != torch_dtype or not a.is_contiguous():
            raise DTError("expected a contiguous %s tensor" % torch_dtype)
        return ctypes.c_void_p(a.data_ptr()), 1 if a.is_cuda else 0
    import numpy as np
    if a.dtype != np.dtype(np_dtype) or not a.flags["C_CONTIGUOUS"]:
        raise DTError("expected a contiguous %s array" % np_dtype)
    return ctypes.c_void_p(a.ctypes.data), 0


def intersect_primary(scene, g, frame, first_ray, hit_shape, hit_t, stream=None):
    """The intersection micro-benchmark: closest hit of primary rays first_ray ..
    first_ray + len(hit_shape) - 1 of the globals' camera (include/dt.h dt_intersect_primary).
    hit_shape: int32, hit_t: float32, both host or both device. Returns the kernel's ms."""
    sp, sdev = _ptr_typed(hit_shape, "torch.int32", "int32")
    tp, tdev = _ptr_typed(hit_t, "torch.float32", "float32")
    n = hit_shape.numel() if hasattr(hit_shape, "numel") else hit_shape.size
    nt = hit_t.numel() if hasattr(hit_t, "numel") else hit_t.size
    if sdev != tdev or n != nt:
        raise DTError("hit_shape and hit_t: same length, same side")
    ms = ctypes.c_float(0)
    check(lib.dt_intersect_primary(scene.handle, ctypes.byref(g), int(frame), int(first_ray), int(n), sp, tp, sdev,
                                   ctypes.c_void_p(stream) if stream else None, ctypes.byref(ms)),
          "dt_intersect_primary")
    return ms.value


def render_sky(g, frame, out, tile=None, stream=None):
    """renderImageCloud's pixel loop (sky only) into `out`."""
    st = Stats()
    p, dev = _ptr(out)
    check(lib.dt_render_sky(ctypes.byref(g), float(frame), ctypes.byref(tile) if tile else None, p, dev,
                            ctypes.c_void_p(stream) if stream else None, ctypes.byref(st)), "dt_render_sky")
    return st


def slab_floats(g, tile):
    return int(lib.dt_slab_floats(ctypes.byref(g), ctypes.byref(tile)))


def slab_floats_max(g, tile):
    return int(lib.dt_slab_floats_max(ctypes.byref(g), ctypes.byref(tile)))


def unpack_slabs(g, tile, world, slabs, image, stream=None):
    sp, sdev = _ptr(slabs)
    ip, idev = _ptr(image)
    if sdev != idev:
        raise DTError("slabs and image must be on the same side")
    check(lib.dt_unpack_slabs(ctypes.byref(g), ctypes.byref(tile), int(world), sp, ip, idev,
                              ctypes.c_void_p(stream) if stream else None), "dt_unpack_slabs")


def write_ppm(filename, g, values):
    import numpy as np
    v = np.ascontiguousarray(values, dtype=np.float32)
    check(lib.dt_write_ppm(filename.encode(), g.xRes, g.yRes, ctypes.c_void_p(v.ctypes.data)), "dt_write_ppm")


def write_png(filename, g, values):
    import numpy as np
    v = np.ascontiguousarray(values, dtype=np.float32)
    check(lib.dt_write_png(filename.encode(), g.xRes, g.yRes, ctypes.c_void_p(v.ctypes.data)), "dt_write_png")


def renderImage(filename, frame, sceneBuilder, g=None, builder_frame=None):
    """render_final_project.cpp:965: build (sceneBuilder names a scene.h builder), render the
    frame on the current GPU, write the PPM. Returns (image, stats)."""
    import numpy as np
    g = g if g is not None else globals_default()
    built = build_scene(sceneBuilder, frame if builder_frame is None else builder_frame, g)
    scene = Scene(built, g)
    img = np.zeros(3 * g.xRes * g.yRes, dtype=np.float32)
    st = render(scene, g, frame, img)
    if filename:
        (write_png if filename.endswith(".png") else write_ppm)(filename, g, img)
    scene.close()
    return img, st


def renderImageCloud(filename, frame, g=None):
    """render_final_project.cpp:1224 (sky/cloud only)."""
    import numpy as np
    g = g if g is not None else globals_default()
    img = np.zeros(3 * g.xRes * g.yRes, dtype=np.float32)
    st = render_sky(g, frame, img)
    if filename:
        write_ppm(filename, g, img)
    return img, st
