"""ctypes binding of libdt.so (include/dt.h).

The struct layouts below mirror include/dt.h field by field. Loading fails loudly: there is
no CPU fallback anywhere in this package — a missing or stale libdt.so is an error, never
a silent switch to another implementation.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DT_LIB") or os.path.join(_HERE, "libdt.so")   # DT_LIB: A/B builds
REPO_ROOT = os.path.dirname(_HERE)
DATA_DIR = os.path.join(REPO_ROOT, "data")

c_int32, c_uint32, c_int64, c_uint64 = ctypes.c_int32, ctypes.c_uint32, ctypes.c_int64, ctypes.c_uint64
c_float, c_double = ctypes.c_float, ctypes.c_double
D3 = c_double * 3

DT_OK = 0
DT_OUT_IMAGE = 0
DT_OUT_SLAB = 1
DT_KERNEL_AUTO, DT_KERNEL_PRODUCT, DT_KERNEL_DONATE = 0, 1, 2   # dt_scene_set_kernel

SHAPE_TYPES = {1: "sphere", 2: "cylinder", 3: "triangle", 4: "rectangle", 5: "rectprism_v2",
               6: "checkerboard", 7: "checkerboard_hole", 8: "checker_cylinder", 9: "rectprism_cyl"}
ABI_VERSION = 8


class ShapeDesc(ctypes.Structure):
    _fields_ = [("type", c_int32), ("model", c_int32), ("material", c_int32), ("emit", c_int32),
                ("flags", c_uint32), ("tex_frame", c_int32), ("roughness", c_float), ("radius", c_float),
                ("S", c_float), ("borderwidth", c_float), ("length", c_float), ("width", c_float),
                ("refr", c_double * 2), ("color", D3), ("color1", D3), ("color2", D3),
                ("bordercolor", D3), ("center", D3), ("v", D3 * 8), ("mesh_normal", D3),
                ("uv", (c_double * 2) * 3), ("hole_first", c_int32), ("n_holes", c_int32)]


class LightDesc(ctypes.Structure):
    _fields_ = [("type", c_int32), ("shape_index", c_int32), ("radius", c_float), ("_pad", c_float),
                ("center", D3), ("color", D3), ("baxis", D3), ("A", D3), ("B", D3), ("D", D3)]


class TextureDesc(ctypes.Structure):
    _fields_ = [("width", c_int32), ("height", c_int32), ("channels", c_int32), ("_pad", c_int32),
                ("pixels", ctypes.POINTER(ctypes.c_uint8))]


class SceneDesc(ctypes.Structure):
    _fields_ = [("n_shapes", c_int32), ("n_lights", c_int32), ("n_textures", c_int32), ("_pad", c_int32),
                ("shapes", ctypes.POINTER(ShapeDesc)), ("lights", ctypes.POINTER(LightDesc)),
                ("textures", ctypes.POINTER(TextureDesc)), ("n_holes", c_int32), ("_pad2", c_int32),
                ("holes", ctypes.POINTER(ShapeDesc))]


class Globals(ctypes.Structure):
    """render_final_project.cpp:48-137, 1:1 (dt_globals)."""
    _fields_ = [("xRes", c_int32), ("yRes", c_int32), ("eye", D3), ("lookingAt", D3), ("up", D3),
                ("aspect", c_float), ("near_plane", c_float), ("fov", c_float), ("aperture", c_float),
                ("focal_length", c_float), ("use_model", c_int32), ("nogloss", c_int32),
                ("refr_air", c_float), ("refr_glass", c_float), ("max_depth", c_int32), ("phong", c_float),
                ("default_col", D3), ("c_isect", c_float), ("c_trav", c_float),
                ("antialias_samples", c_int32), ("brdf_samples", c_int32), ("blur_samples", c_int32),
                ("frame_range", c_int32), ("frame_prism", c_int32), ("frame_cloud", c_int32),
                ("frame_blur", c_int32), ("frame_start", c_int32), ("frame_move1", c_int32),
                ("frame_move2", c_int32), ("frame_sculp", c_int32), ("total", c_int32),
                ("far_dist", c_float), ("move_per_frame", c_float), ("tot_move", c_float), ("accel_t", c_float),
                ("cap_center", D3), ("sundir", D3), ("perlin_cloud", c_int32), ("saturation", c_float),
                ("clouddist", c_float), ("cloudhoff", c_float), ("sun_outer", D3), ("sun_inner", D3),
                ("sun_core", D3), ("bluesky", D3), ("redsky", D3), ("reflect", c_int32), ("seed", c_uint32)]

    def copy(self):
        g = Globals()
        ctypes.pointer(g)[0] = self
        return g


class Tiles(ctypes.Structure):
    _fields_ = [("x0", c_int32), ("y0", c_int32), ("x1", c_int32), ("y1", c_int32), ("tile_w", c_int32),
                ("tile_h", c_int32), ("rank", c_int32), ("world", c_int32), ("layout", c_int32),
                ("_pad", c_int32)]


class Stats(ctypes.Structure):
    _fields_ = [("pixels", c_uint64), ("samples", c_uint64), ("rays", c_uint64), ("shadow_rays", c_uint64),
                ("sky_pixels", c_uint64), ("uv_out_of_range", c_uint64), ("glossy_exhausted", c_uint64),
                ("spherelight_exhausted", c_uint64), ("prism_norm_fallback", c_uint64),
                ("reflect_errors", c_uint64), ("nan_pixels", c_uint64), ("tex_fetches", c_uint64),
                ("stack_overflows", c_uint64), ("box_tests", c_uint64), ("prim_tests", c_uint64),
                ("wave_node_visits", c_uint64), ("kernel_ms", c_double),
                ("trace_kernel_ms", c_double), ("donations", c_uint64), ("donate_overflow", c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class BVHNode(ctypes.Structure):
    _fields_ = [("first_child", c_int32), ("n_children", c_int32), ("first_index", c_int32),
                ("n_indices", c_int32), ("leaf", c_int32), ("depth", c_int32), ("lbound", D3), ("ubound", D3)]


class AccelInfo(ctypes.Structure):
    _fields_ = [("n_nodes", c_int32), ("n_fnodes", c_int32), ("n_bnodes", c_int32), ("boxes_ordered", c_int32),
                ("sg_lights", c_int32), ("sg_dim", c_int32 * 3), ("sg_cells", c_int64), ("sg_tree_cells", c_int64),
                ("sg_list_pool", c_int64), ("sg_list_entries", c_int64), ("nodes_hash", c_uint64),
                ("fnodes_hash", c_uint64), ("bnodes_hash", c_uint64), ("sg_hash", c_uint64),
                ("sg_contents_hash", c_uint64), ("bump_pad", c_float), ("sg_reach", c_float),
                ("sg_umbra_cells", c_int64), ("features", ctypes.c_uint32),
                ("sg_sub_blocks", c_int32), ("sg_sub_nodes", c_int64), ("sg_sub_hash", c_uint64)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d["sg_dim"] = tuple(self.sg_dim)
        return d


# every symbol include/dt.h declares (checked by tests/test_abi.py)
EXPORTS = ["dt_abi_version", "dt_last_error", "dt_globals_default", "dt_scene_create", "dt_scene_destroy",
           "dt_scene_prepare", "dt_scene_upload", "dt_scene_set_kernel",
           "dt_scene_bvh", "dt_bvh_build", "dt_accel_info_build", "dt_trace_build", "dt_slab_floats", "dt_slab_floats_max",
           "dt_render", "dt_render_async", "dt_collect_stats", "dt_debug_counters", "dt_debug_item_costs", "dt_render_sky",
           "dt_unpack_slabs", "dt_build_scene", "dt_scene_desc_free", "dt_write_ppm", "dt_write_png",
           "dt_mocap_bone_table", "dt_debug_normalize", "dt_intersect_primary",
           "dt_debug_load_obj"]


class DTError(RuntimeError):
    pass


def _share_torch_hip_runtime():
    """PyTorch-ROCm ships its own libamdhip64 (soname libamdhip64.so.7, but its libraries
    NEED it as "libamdhip64.so"). If libdt.so is loaded first it binds /opt/rocm's runtime and
    a later `import torch` loads a second HIP runtime into the process, after which one of the
    two sees no device. Importing torch first makes libdt's libamdhip64.so.7 dependency
    resolve to the runtime torch already loaded: one HIP runtime, shared streams/pointers."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def _load():
    _share_torch_hip_runtime()
    if not os.path.exists(LIB_PATH):
        raise DTError("libdt.so not built (%s): run __graft_entry__.build() / make -C "
                      "distraytracer_amd/csrc" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    lib.dt_abi_version.restype = c_int32
    if lib.dt_abi_version() != ABI_VERSION:   # a stale library would misread every descriptor
        raise DTError("libdt.so ABI %d, this binding expects %d: rebuild (make -C distraytracer_amd/csrc)"
                      % (lib.dt_abi_version(), ABI_VERSION))
    P = ctypes.POINTER
    sig = {
        "dt_abi_version": (c_int32, []),
        "dt_last_error": (ctypes.c_char_p, []),
        "dt_globals_default": (None, [P(Globals)]),
        "dt_scene_create": (c_int32, [P(SceneDesc), P(Globals), P(ctypes.c_void_p)]),
        "dt_scene_destroy": (None, [ctypes.c_void_p]),
        "dt_scene_prepare": (c_int32, [P(SceneDesc), P(Globals), P(ctypes.c_void_p)]),
        "dt_scene_upload": (c_int32, [ctypes.c_void_p]),
        "dt_scene_set_kernel": (c_int32, [ctypes.c_void_p, c_int32]),
        "dt_scene_bvh": (c_int32, [ctypes.c_void_p, P(BVHNode), c_int32, P(c_int32), c_int32, P(c_int32),
                                   P(c_int32)]),
        "dt_bvh_build": (c_int32, [P(SceneDesc), P(Globals), P(BVHNode), c_int32, P(c_int32), c_int32, P(c_int32),
                                   P(c_int32)]),
        "dt_accel_info_build": (c_int32, [P(SceneDesc), P(Globals), P(AccelInfo)]),
        "dt_trace_build": (c_int32, [P(SceneDesc), P(Globals), c_int32, ctypes.c_char_p, c_int32,
                                     P(ctypes.c_uint32), P(ctypes.c_uint32)]),
        "dt_slab_floats": (c_int64, [P(Globals), P(Tiles)]),
        "dt_slab_floats_max": (c_int64, [P(Globals), P(Tiles)]),
        "dt_render": (c_int32, [ctypes.c_void_p, P(Globals), c_int32, P(Tiles), ctypes.c_void_p, c_int32,
                                ctypes.c_void_p, P(Stats)]),
        "dt_render_async": (c_int32, [ctypes.c_void_p, P(Globals), c_int32, P(Tiles), ctypes.c_void_p,
                                      ctypes.c_void_p]),
        "dt_collect_stats": (c_int32, [ctypes.c_void_p, ctypes.c_void_p, P(Stats)]),
        "dt_debug_counters": (c_int32, [ctypes.c_void_p, P(c_uint64), c_int32]),
        "dt_debug_item_costs": (c_int64, [ctypes.c_void_p, P(ctypes.c_uint32), c_int64]),
        "dt_debug_normalize": (c_int32, [P(c_double), P(c_double), c_int64]),
        "dt_render_sky": (c_int32, [P(Globals), c_float, P(Tiles), ctypes.c_void_p, c_int32, ctypes.c_void_p,
                                    P(Stats)]),
        "dt_intersect_primary": (c_int32, [ctypes.c_void_p, P(Globals), c_int32, c_int64, c_int64, ctypes.c_void_p,
                                           ctypes.c_void_p, c_int32, ctypes.c_void_p, P(c_float)]),
        "dt_unpack_slabs": (c_int32, [P(Globals), P(Tiles), c_int32, ctypes.c_void_p, ctypes.c_void_p, c_int32,
                                      ctypes.c_void_p]),
        "dt_build_scene": (c_int32, [ctypes.c_char_p, c_float, P(Globals), ctypes.c_char_p, P(P(SceneDesc))]),
        "dt_scene_desc_free": (None, [P(SceneDesc)]),
        "dt_debug_load_obj": (c_int32, [ctypes.c_char_p, ctypes.c_void_p, c_int64, ctypes.c_void_p, c_int64,
                                        ctypes.c_void_p, c_int64, P(c_int64)]),
        "dt_write_ppm": (c_int32, [ctypes.c_char_p, c_int32, c_int32, ctypes.c_void_p]),
        "dt_write_png": (c_int32, [ctypes.c_char_p, c_int32, c_int32, ctypes.c_void_p]),
        "dt_mocap_bone_table": (c_int32, [ctypes.c_char_p, ctypes.c_char_p, P(c_int32), c_int32,
                                          P(c_double), P(c_int32), P(c_int32)]),
    }
    for name, (res, args) in sig.items():
        # a variant library built from an older tree for an A/B (DT_LIB) may lack a newer debug hook
        if name.startswith("dt_debug_") and os.environ.get("DT_LIB") and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def check(rc, what=""):
    if rc != DT_OK:
        raise DTError("%s failed (%d): %s" % (what, rc, lib.dt_last_error().decode(errors="replace")))
    return rc
