"""Host-side logic without a GPU: scene builders, the reference-topology BVH (product builder
vs the oracle's independent restatement of helpers.h:330-472), tile ownership and slab
scatter, and analytic anchors of the oracle renderer."""
import collections
import ctypes

import numpy as np
import pytest

import distraytracer_amd as dt
import oracle
from distraytracer_amd._lib import SHAPE_TYPES


def final240():
    g = dt.globals_default()
    g.use_model = 0
    return g, dt.build_scene("final", 240, g)


def test_build_final_240_inventory():
    """buildFinal(240), use_model=false: 30 bone cylinders, 2 doors, floor, 3 walls,
    4 window prisms, ceiling, 4 area lights, checker cylinder, 8 stairs."""
    g, b = final240()
    d = b.desc
    c = collections.Counter(SHAPE_TYPES[d.shapes[i].type] for i in range(d.n_shapes))
    assert c == {"cylinder": 30, "rectprism_v2": 12, "rectangle": 10, "checkerboard_hole": 1,
                 "checker_cylinder": 1}
    assert d.n_lights == 5 and d.n_textures == 3
    types = [d.lights[i].type for i in range(5)]
    assert types == [1, 3, 3, 3, 3]
    for i in range(1, 5):   # each area light is also a shape (skipped by its own shadow test)
        si = d.lights[i].shape_index
        assert d.shapes[si].emit == 2 and d.shapes[si].flags & 1
    assert g.perlin_cloud == 1
    # camera choreography at frame 240 (scene.h:671-686): eye rotated about +y by 9pi/16
    assert g.eye[1] == pytest.approx(9.0, abs=1e-6)
    assert g.lookingAt[1] == pytest.approx(11 - 5, abs=1e-6)
    tex = [(d.textures[i].width, d.textures[i].height) for i in range(3)]
    assert tex == [(350, 653), (351, 653), (280, 280)]


def test_build_spheres_matches_reference_constants():
    g = dt.globals_default()
    b = dt.build_scene("spheres", 0, g)
    d = b.desc
    radii = [d.shapes[i].radius for i in range(5)]
    assert radii == pytest.approx([0.3, 0.45, 0.675, 1.0125, 999], rel=1e-6)
    assert [bool(d.shapes[i].flags & 2) for i in range(5)] == [True] * 4 + [False]
    assert list(d.lights[0].center) == [-6, 0.5, 1]


def test_build_final_models_inventory():
    """use_model=true: finalBuildModels (scene.h:258-602) adds two textured columns and two
    busts from the substitute OBJs (tools/gen_models.py): 2 x 832 + 2 x (364 - 2) triangles,
    Oren-Nayar marble, per-vertex UVs flipped in v, roughness from the map."""
    g = dt.globals_default()
    g.use_model = 1
    b = dt.build_scene("final", 240, g)   # keep the owner alive while reading its desc
    d = b.desc
    tris = [d.shapes[i] for i in range(d.n_shapes) if d.shapes[i].type == 3]
    assert len(tris) == 2 * 832 + 2 * 362 and d.n_textures == 4
    col, bust = tris[:2 * 832], tris[2 * 832:]
    assert all(t.model == 1 and t.flags & 4 and t.flags & 64 and t.tex_frame == 3 for t in col)
    assert all(0 <= t.uv[k][j] <= 1 for t in col for k in range(3) for j in range(2))
    assert all(0.2 < t.roughness < 0.8 for t in col)
    assert all(t.roughness == 0.5 and not t.flags & 4 for t in bust)


def test_build_final_tunnel_frames():
    """frames >= frame_prism (C5): generateTrianglePrismMesh (scene.h:135-256) adds the bottom
    cap triangle and the ad rectangles (substitute ./ads frames), all in motion and named
    "rectangle", each with its own texture; the doors/room are gone once the eye passed them."""
    g = dt.globals_default()
    g.use_model = 0
    b = dt.build_scene("final", 1200, g)
    d = b.desc
    rects = [d.shapes[i] for i in range(d.n_shapes) if d.shapes[i].type == 4]
    assert len(rects) == d.n_textures > 500
    assert all(r.flags & 2 and r.flags & 4 and r.flags & 16 and r.model == 3 for r in rects)
    assert sum(d.shapes[i].type == 3 for i in range(d.n_shapes)) == 1
    assert g.focal_length == 20 and list(g.up) == [0, 0, -1]


def test_build_prismcyl():
    """BuildScenePrismCylinder (scene.h:3227-3263): one RectPrismWithCylinder (4x4x1 box at
    x in [0, 1]) with one radius-1 cylinder hole along x through its centre, a point light; the
    eye is rotated about itself, so it stays at og_eye up to rounding."""
    g = dt.globals_default()
    b = dt.build_scene("prismcyl", 7, g)
    d = b.desc
    assert d.n_shapes == 1 and d.n_lights == 1 and d.n_holes == 1
    p = d.shapes[0]
    assert SHAPE_TYPES[p.type] == "rectprism_cyl" and (p.hole_first, p.n_holes) == (0, 1)
    assert [list(p.v[k]) for k in (0, 6)] == [[0, -2, -2], [1, 2, 2]]
    assert list(p.color) == [1, 0, 0] and list(p.center) == [0.5, 0, 0]
    h = d.holes[0]
    assert SHAPE_TYPES[h.type] == "cylinder" and h.radius == 1
    assert list(h.v[0]) == [0, 0, 0] and list(h.v[1]) == [1, 0, 0] and list(h.color) == [0, 0, 1]
    assert list(g.eye) == pytest.approx([-6, 0.5, 1], abs=1e-12)
    assert d.lights[0].type == 1 and list(d.lights[0].center) == [-5, 1, 0]


def test_oracle_prismcyl_hole_and_face():
    """RectPrismWithCylinder through the oracle (geometry.cpp:1507-1651). A camera ray toward the
    box crosses the hole's front cap plane (x = 0) and enters the box there too; the two distances
    are computed differently (-s.x / float(ray.x) against -s.x * (1 / ray.x)), and when the cap's is
    not larger the ray passes (return false), even outside the hole's radius: intersectCap tests
    planes. With the scene's own camera (eye (-6, 0.5, 1) looking along +x; the DoF offsets have no x
    component) ray.x = 10 exactly, both distances round to 0.6f and every ray passes: the reference's
    prismcyl frame 0 is black. From an oblique eye part of the rays stop on the red front face: red
    speckle, never the hole's blue (its body branch needs the cap plane behind the ray's start)."""
    g = dt.globals_default()
    b = dt.build_scene("prismcyl", 0, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth = 64, 48, 4, 2
    img, st = oracle.render(b, g, 0, dt.tiles())
    assert (img == 0).all() and st.rays == 64 * 48 * 4
    g.eye[0], g.eye[1], g.eye[2] = -5.0, 1.3, 2.2
    img, st = oracle.render(b, g, 0, dt.tiles())
    px = img.reshape(48, 64, 3)
    assert (px[..., 1] == 0).all() and (px[..., 2] == 0).all()
    assert px[..., 0].max() > 0 and (px[..., 0] == 0).sum() > 0
    assert st.prism_norm_fallback == 0      # every hit lies on the front face (getNorm's normbot)


@pytest.mark.parametrize("name,frame,models", [("final", 240, 0), ("spheres", 0, 0), ("dof", 0, 0), ("hw4", 0, 0),
                                               ("prismcyl", 3, 0), ("final", 0, 0), ("final", 480, 0), ("final", 2000, 0),
                                               ("final", 480, 1), ("final", 240, 1), ("final", 1200, 0),
                                               ("final", 1680, 0)])
def test_bvh_topology_equals_oracle(name, frame, models):
    g = dt.globals_default()
    g.use_model = models
    b = dt.build_scene(name, frame, g)
    scene_nodes, scene_idx = _device_free_bvh(b, g)
    or_nodes, or_idx = oracle.bvh(b, g)
    assert scene_idx == or_idx
    assert len(scene_nodes) == len(or_nodes)
    for a, o in zip(scene_nodes, or_nodes):
        assert (a.leaf, a.n_children, a.depth, a.n_indices) == (o.leaf, o.n_children, o.depth, o.n_indices)
        assert list(a.lbound) == list(o.lbound) and list(a.ubound) == list(o.ubound)


def _device_free_bvh(b, g):
    """the product's host BVH builder (dt_bvh_build), no device needed"""
    import ctypes
    from distraytracer_amd._lib import BVHNode
    nn, ni = ctypes.c_int32(), ctypes.c_int32()
    dt.check(dt.lib.dt_bvh_build(b._ptr, ctypes.byref(g), None, 0, None, 0, ctypes.byref(nn), ctypes.byref(ni)))
    nodes = (BVHNode * max(nn.value, 1))()
    idx = (ctypes.c_int32 * max(ni.value, 1))()
    dt.check(dt.lib.dt_bvh_build(b._ptr, ctypes.byref(g), nodes, nn.value, idx, ni.value, ctypes.byref(nn),
                                 ctypes.byref(ni)))
    return list(nodes)[:nn.value], list(idx)[:ni.value]


@pytest.mark.parametrize("world", [1, 2, 3, 5, 8])
def test_tiles_partition_every_pixel_once(world):
    g = dt.globals_default()
    g.xRes, g.yRes = 100, 70   # ragged edge tiles
    base = dt.tiles(tile_w=32, tile_h=16, world=world, layout=dt.DT_OUT_SLAB)
    per = dt.slab_floats_max(g, base)
    slabs = np.zeros(world * per, dtype=np.float32)
    for r in range(world):
        t = dt.tiles(tile_w=32, tile_h=16, rank=r, world=world, layout=dt.DT_OUT_SLAB)
        n = dt.slab_floats(g, t)
        assert n <= per
        slabs[r * per:r * per + n] = r + 1
    img = np.zeros(3 * g.xRes * g.yRes, dtype=np.float32)
    dt.unpack_slabs(g, base, world, slabs, img)
    assert (img > 0).all()
    owner = img.reshape(g.yRes, g.xRes, 3)[::-1, :, 0] - 1   # back to y-up
    ty, tx = np.meshgrid(np.arange(g.yRes) // 16, np.arange(g.xRes) // 32, indexing="ij")
    tiles_x = (g.xRes + 31) // 32
    assert np.array_equal(owner, _tile_owner(ty * tiles_x + tx, world))


def _tile_owner(tid, world):
    """rank owning tile tid (dt_scene_dev.h tile_of: groups of `world` tiles, ranks rotated by a
    hash of the group)"""
    slot = (tid // world).astype(np.uint64)
    h = (slot * 2654435761) & 0xffffffff
    h ^= h >> 15
    h = (h * 0x2c1b3c6d) & 0xffffffff
    h ^= h >> 12
    return ((tid % world) + world - (h % world).astype(np.int64)) % world


def test_tile_split_balances_columns():
    """At 1920 px (60 tiles a row) a plain t % 8 interleave gives ranks r and r+4 the same tile
    columns; the hashed rotation spreads every rank over all columns."""
    tiles_x, tiles_y, world = 60, 34, 8
    tid = np.arange(tiles_x * tiles_y)
    owner = _tile_owner(tid, world)
    for r in range(world):
        cols = np.bincount(tid[owner == r] % tiles_x, minlength=tiles_x)
        assert (cols > 0).sum() >= 50            # t % 8: 15 columns per rank
        assert ((tid % world == r) & (tid % tiles_x % 4 == r % 4)).sum() == (tid % world == r).sum()
        assert abs(int((owner == r).sum()) - len(tid) / world) <= 1


def test_oracle_center_pixel_anchor():
    """C1 (buildSceneSpheres(0), aperture 0): the centre pixel's ray is the gaze +x from the eye,
    hits sphere 0 head-on; the point light sits at the eye, so Lambert = 0.9 and Phong
    pow(1, 10) * 0.9 -> colour (1.8, 0, 0) for the primary and both motion-blur re-traces."""
    g = dt.globals_default()
    b = dt.build_scene("spheres", 0, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth, g.aperture = 256, 256, 1, 1, 0.0
    col, hit = oracle.sample_color(b, g, 0, 128, 128, 0)
    assert hit
    assert col == pytest.approx([1.8, 0, 0], abs=1e-12)


def test_oracle_sky_image_cloud_anchor():
    """renderImageCloud: pixels are finite, in [0,255], and rows far above the cloud layer
    equal the analytic sky gradient's clamp."""
    g = dt.globals_default()
    g.xRes, g.yRes = 64, 48
    img = oracle.render_sky(g, 1.0, dt.tiles())
    assert np.isfinite(img).all() and img.min() >= 0 and img.max() <= 255


# ---- acceleration structures built on the host (dt_accel_info_build) ------------------------

def _accel(name, frame, models, env, monkeypatch):
    for k in ("DT_SG_BLOCK", "DT_SG_ORDER", "DT_SG_HULL", "DT_SG_UMBRA"):
        monkeypatch.delenv(k, raising=False)
    # the padded grid alone (its walk-cell share decides whether a pass-0 grid is appended)
    monkeypatch.setenv("DT_SG_PASS0", "0")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = dt.globals_default()
    g.use_model = models
    b = dt.build_scene("final", frame, g)
    return dt.accel_info(b, g)


def test_shadow_grid_pass0_grid_appended(monkeypatch):
    """Frame 1920's blur shifts (<= 81) pad the lists; with a short list cap (24) many cells walk
    (over the 10% that appends a pass-0 grid by default), and the pass-0 grid (same cells, unpadded
    lists) walks almost nowhere. With the default cap (96) no cell walks and nothing is appended."""
    cap = {"DT_SG_MAX_LIST": "24"}
    pad = _accel("c5-1920", 1920, 0, cap, monkeypatch)
    both = _accel("c5-1920", 1920, 0, dict(cap, DT_SG_PASS0="1"), monkeypatch)
    assert pad["sg_tree_cells"] > pad["sg_cells"] // 10
    assert both["sg_cells"] == 2 * pad["sg_cells"]
    assert both["sg_tree_cells"] - pad["sg_tree_cells"] < pad["sg_cells"] // 20
    monkeypatch.delenv("DT_SG_PASS0")
    g = dt.globals_default()
    g.use_model = 0
    dflt = dt.accel_info(dt.build_scene("final", 1920, g), g)
    assert dflt["sg_cells"] == both["sg_cells"]
    monkeypatch.delenv("DT_SG_MAX_LIST")
    g = dt.globals_default()
    g.use_model = 0
    dflt96 = dt.accel_info(dt.build_scene("final", 1920, g), g)
    assert dflt96["sg_cells"] == pad["sg_cells"] and dflt96["sg_tree_cells"] <= pad["sg_cells"] // 10


# C3's room, C4's meshes (2442 leaves), a C5 tunnel frame with blur-padded lists
ACCEL_SCENES = [("c3", 240, 0), ("c4", 240, 1), ("c5-tunnel", 1200, 0)]


@pytest.mark.parametrize("hull", ["0", "2"])
@pytest.mark.parametrize("name,frame,models", ACCEL_SCENES, ids=[s[0] for s in ACCEL_SCENES])
def test_shadow_grid_block_tests_give_identical_lists(name, frame, models, hull, monkeypatch):
    """The per-block (leaf, cell) rejection (host_shadowgrid.cpp) is exact only while the swept
    test, the plane separation and the hull separation stay monotone in the cell box: with hull
    culling off (0) or on every cell (2), every block size must give the per-cell build's lists
    bit for bit (cells, counts and pool, in storage order). Umbra cells off: their default marks
    whole blocks, by design coarser for larger blocks."""
    env = {"DT_SG_HULL": hull, "DT_SG_UMBRA": "0"}
    base = _accel(name, frame, models, dict(env, DT_SG_BLOCK="0"), monkeypatch)
    assert base["sg_lights"] > 0 and base["sg_list_entries"] > 0
    for blk in ("4x2", "8x4", "32x8", "1x1"):
        got = _accel(name, frame, models, dict(env, DT_SG_BLOCK=blk), monkeypatch)
        assert got["sg_hash"] == base["sg_hash"], blk
        assert got["sg_list_entries"] == base["sg_list_entries"], blk
    dflt = _accel(name, frame, models, env, monkeypatch)
    assert dflt["sg_hash"] == base["sg_hash"]
    assert dflt["nodes_hash"] == base["nodes_hash"] and dflt["fnodes_hash"] == base["fnodes_hash"]


@pytest.mark.parametrize("name,frame,models", ACCEL_SCENES, ids=[s[0] for s in ACCEL_SCENES])
def test_shadow_grid_hull_culling_only_drops(name, frame, models, monkeypatch):
    """Hull culling removes list entries and never adds any: off >= blocks (the default) >=
    blocks + cells, in entries per list cell, and no cell turns into a tree cell."""
    off = _accel(name, frame, models, {"DT_SG_HULL": "0"}, monkeypatch)
    blk = _accel(name, frame, models, {}, monkeypatch)
    cel = _accel(name, frame, models, {"DT_SG_HULL": "2"}, monkeypatch)
    assert off["sg_cells"] == blk["sg_cells"] == cel["sg_cells"]
    assert off["sg_tree_cells"] >= blk["sg_tree_cells"] >= cel["sg_tree_cells"]
    per = [d["sg_list_entries"] / max(d["sg_cells"] - d["sg_tree_cells"], 1) for d in (off, blk, cel)]
    if off["sg_tree_cells"] == 0:
        assert per[0] >= per[1] >= per[2]


def test_shadow_grid_umbra_cells(monkeypatch):
    """C3's window point light sits behind the wall the window is cut into: whole blocks of cells
    see it only through one prism face (host_shadowgrid.cpp umbra cells). Off: none; blocks (the
    default); blocks + single cells: a superset. Each umbra cell keeps a one-leaf list, so the
    lists only shrink."""
    off = _accel("c3", 240, 0, {"DT_SG_UMBRA": "0"}, monkeypatch)
    blk = _accel("c3", 240, 0, {}, monkeypatch)
    cel = _accel("c3", 240, 0, {"DT_SG_UMBRA": "2"}, monkeypatch)
    assert off["sg_umbra_cells"] == 0
    assert blk["sg_umbra_cells"] >= off["sg_cells"] // off["sg_lights"] // 2
    assert cel["sg_umbra_cells"] >= blk["sg_umbra_cells"]
    assert off["sg_list_entries"] > blk["sg_list_entries"] >= cel["sg_list_entries"]
    assert off["sg_tree_cells"] == blk["sg_tree_cells"] == 0


@pytest.mark.parametrize("name,frame,models", ACCEL_SCENES[:1] + ACCEL_SCENES[2:],
                         ids=[ACCEL_SCENES[0][0], ACCEL_SCENES[2][0]])
def test_shadow_grid_ordered_lists_hold_the_same_leaves(name, frame, models, monkeypatch):
    """DT_SG_ORDER=1 reorders each cell's list (likely occluder first) and nothing else."""
    plain = _accel(name, frame, models, {}, monkeypatch)
    ordered = _accel(name, frame, models, {"DT_SG_ORDER": "1"}, monkeypatch)
    assert ordered["sg_contents_hash"] == plain["sg_contents_hash"]
    assert ordered["sg_list_entries"] == plain["sg_list_entries"]
    assert ordered["sg_cells"] == plain["sg_cells"] and ordered["sg_tree_cells"] == plain["sg_tree_cells"]


def test_shadow_grid_block_knob_is_strict(monkeypatch, capfd):
    """Malformed DT_SG_BLOCK values are reported and fall back to the default 8x4 blocks."""
    dflt = _accel("c3", 240, 0, {}, monkeypatch)
    capfd.readouterr()
    for bad in ("1", "8", "0x4", "8x", "x4", "8x4junk"):
        got = _accel("c3", 240, 0, {"DT_SG_BLOCK": bad}, monkeypatch)
        assert got["sg_hash"] == dflt["sg_hash"]
        assert "DT_SG_BLOCK" in capfd.readouterr().err, bad


def test_accel_info_matches_scene_bvh():
    """dt_accel_info_build builds the tree dt_bvh_build exports (same node count)."""
    g, b = final240()
    info = dt.accel_info(b, g)
    nodes = (dt.BVHNode * 4096)()
    idx = (ctypes.c_int32 * 4096)()
    nn, ni = ctypes.c_int32(), ctypes.c_int32()
    dt.check(dt.lib.dt_bvh_build(b._ptr, ctypes.byref(g), nodes, 4096, idx, 4096, ctypes.byref(nn),
                                 ctypes.byref(ni)), "dt_bvh_build")
    assert info["n_nodes"] == nn.value
    assert info["boxes_ordered"] == 1 and info["n_fnodes"] == info["n_nodes"]


def test_work_header_and_oracle_counts():
    """SURVEY §8(d)'s work unit: include/dt_work.h parsed by distraytracer_amd/work.py (the weights
    bench.py prices with), and the oracle's reference-loop counts on a small C2-like render: one
    camera event per sample, one light event per shadow ray, counting leaves the image unchanged."""
    from distraytracer_amd import work
    assert work.N_EVENTS == 35 and len(work.WEIGHTS) == work.N_EVENTS and work.PEAK_FP64_TFLOPS == 78.6
    assert work.NAMES[0] == "box" and work.NAMES[work.SKY] == "sky"
    assert work.NAMES[1 + 4] == "hit_shape.rectangle" and work.NAMES[23 + 2] == "brdf.cook_torrance"
    g, b = final240()
    g.xRes, g.yRes, g.antialias_samples, g.max_depth = 40, 24, 4, 4
    tile = dt.tiles()
    img, st, wk = oracle.render_work(b, g, 240, tile)
    ref, _ = oracle.render(b, g, 240, tile)
    assert np.array_equal(img, ref)
    n = dict(zip(work.NAMES, wk.tolist()))
    assert n["camera"] == st.samples == 40 * 24 * 4
    assert n["light"] == st.shadow_rays and n["hit"] <= st.rays and n["box"] > 0
    assert n["sky"] >= st.sky_pixels   # the reference loop marches once per missing sample
    assert work.price(wk) == pytest.approx(sum(float(c) * w for c, w in zip(wk, work.WEIGHTS)))


def test_oracle_primary_hit_numbering():
    """or_primary_hit (the intersection micro-benchmark's reference) follows dt_intersect_primary's
    ray numbering and the render's camera: a ray hits iff the same pixel-sample's rayColor tree in
    or_sample_color reports a hit (the root step decides it: no hit, no children); and the closest hit
    is the first of the ray's gathered shapes in distance, t > 0."""
    g, b = final240()
    g.xRes, g.yRes = 64, 48
    npx = g.xRes * g.yRes
    rays = [0, 7, 8, 1000, 8 * npx - 1, 8 * npx, 8 * npx + 13, 3 * 8 * npx + 5]
    for r in rays:
        shape, t = oracle.primary_hit(b, g, 240, r, 1)
        q = r // 8
        p = q % npx
        x, y, s = p % g.xRes, p // g.xRes, r % 8 + 8 * (q // npx)
        _, hit = oracle.sample_color(b, g, 240, x, y, s)
        assert (shape[0] >= 0) == hit, r
        assert (t[0] > 0 and t[0] < 3.4e38) if hit else t[0] == np.float32(3.4028235e38)
    # a window equals the concatenation of its halves (per-ray results, any thread count)
    s1, t1 = oracle.primary_hit(b, g, 240, 100, 512, nthreads=4)
    s2, t2 = oracle.primary_hit(b, g, 240, 100, 256, nthreads=1)
    s3, t3 = oracle.primary_hit(b, g, 240, 356, 256, nthreads=2)
    assert np.array_equal(s1, np.concatenate([s2, s3])) and np.array_equal(t1, np.concatenate([t2, t3]))


# the trace-kernel feature masks (distraytracer_amd/csrc/dt_scene_dev.h)
_ROOM = (1 << 2) | (1 << 4) | (1 << 5) | (1 << 7) | (1 << 8) | (1 << 15)
_MESH = _ROOM | (1 << 3) | (1 << 13)
_TUNNEL = (1 << 2) | (1 << 3) | (1 << 4)


@pytest.mark.parametrize("name,frame,models,build", [
    ("final", 240, 0, "room"), ("final", 0, 0, "room"), ("final", 952, 0, "room"),
    ("final", 240, 1, "mesh"), ("final", 1120, 0, "tunnel"), ("final", 1920, 0, "tunnel"),
    ("final", 2000, 0, "tunnel"), ("spheres", 0, 0, "full"), ("prismcyl", 7, 0, "full")])
def test_scene_features_select_the_build(name, frame, models, build):
    """dt_accel_info.features: the scene's feature mask, from which dt_render picks the trace-kernel
    build (room / mesh / full for still frames, tunnel / full blur for motion-blur frames). The C2,
    C3 and C5 room frames take the room build, C4 the mesh build, C5's tunnel and cloud frames the
    tunnel build; the spheres scene (spheres, sphere lights) and RectPrismWithCylinder the full."""
    g = dt.globals_default()
    g.use_model = models
    built = dt.build_scene(name, frame, g)
    f = dt.accel_info(built, g)["features"]
    within = lambda m: f & ~m == 0
    if frame >= g.frame_prism:   # motion-blur frames (dt_api.cpp enqueue_render)
        got = "tunnel" if within(_TUNNEL) else "full"
    else:
        got = "room" if within(_ROOM) else "mesh" if within(_MESH) else "full"
    assert got == build, "features %#x" % f


def test_every_builder_scene_has_a_covering_build():
    """No render can reach a case its trace-kernel build compiled out (dt_kernels.hip DT_NEED:
    __builtin_unreachable()): for every scene the builders produce -- buildFinal(n*8) for all 300
    frames n of `final n` / C5, with and without the OBJ models, and the dtrender modes' scenes
    (spheres, dof, hw4, prismcyl 0..7) -- at 1, 4, 16, 64 and 256 spp (the 4- and 5-wave builds),
    the build dt_render would launch (dt_trace_build, the same choose_build as the render) covers the
    scene's features. dt_render also refuses a scene outside its build's mask (DT_E_INVALID)."""
    cases = [("final", n * 8, 0) for n in range(300)] + [("final", n * 8, 1) for n in range(0, 300, 20)]
    cases += [("spheres", 0, 0), ("dof", 0, 0), ("hw4", 0, 0)] + [("prismcyl", f, 0) for f in range(8)]
    seen = set()
    for name, frame, models in cases:
        g = dt.globals_default()
        g.use_model = models
        built = dt.build_scene(name, frame, g)
        for spp in (1, 4, 16, 64, 256):
            g.antialias_samples = spp
            kernel, sf, bf = dt.trace_build(built, g, frame)
            assert sf & ~bf == 0, "%s(%d) models=%d spp=%d: %s covers %#x, scene %#x" % (
                name, frame, models, spp, kernel, bf, sf)
            seen.add(kernel)
    # the feature builds are the ones these scenes take
    assert {"dt_trace_kernel", "dt_trace_kernel_w5", "dt_trace_kernel_mesh", "dt_trace_kernel_w5_mesh",
            "dt_trace_kernel_tunnel", "dt_trace_kernel_w5_tunnel", "dt_trace_kernel_full",
            "dt_trace_kernel_rpc"} <= seen, seen


def test_block_subtrees_host_build(monkeypatch):
    """DT_SG_SUBTREE=1 (host_shadowgrid.cpp): C4's mesh cells walk the tree (lists over the cap), so
    their blocks get subtrees; the build is deterministic (thread pool, same hash twice) and off by
    default; smaller blocks give more, smaller subtrees."""
    g = dt.globals_default()
    g.use_model = 1
    built = dt.build_scene("final", 240, g)
    g.xRes, g.yRes, g.antialias_samples = 1920, 1080, 256
    monkeypatch.delenv("DT_SG_SUBTREE", raising=False)
    monkeypatch.delenv("DT_SG_SUB_BLOCK", raising=False)
    off = dt.accel_info(built, g)
    assert off["sg_tree_cells"] > 0 and off["sg_sub_blocks"] == 0 and off["sg_sub_nodes"] == 0
    monkeypatch.setenv("DT_SG_SUBTREE", "1")
    a, b = dt.accel_info(built, g), dt.accel_info(built, g)
    assert a["sg_sub_blocks"] > 0 and a["sg_sub_nodes"] >= a["sg_sub_blocks"]
    assert a["sg_sub_hash"] == b["sg_sub_hash"]
    assert a["sg_hash"] == off["sg_hash"]   # the cells and lists themselves are unchanged
    monkeypatch.setenv("DT_SG_SUB_BLOCK", "4x2")
    c = dt.accel_info(built, g)
    assert c["sg_sub_blocks"] > a["sg_sub_blocks"]


def test_shadow_grid_start_side_culling(monkeypatch):
    """Start-side culling (host_shadowgrid.cpp header) only removes (leaf, cell) pairs: the same
    cells, tree-walk cells and umbra cells, and at least 27% fewer list entries for C3's room (its
    ceiling, back and side walls leave the lists of the cells next to them, for the four ceiling
    lights: 263802 -> 187288 with the box of ray origins, 225677 with the root box), more than 25%
    fewer for C5 frame 1920's tunnel."""
    for name, frame, least in (("c3", 240, 0.27), ("c5-1920", 1920, 0.25)):
        off = _accel(name, frame, 0, {"DT_SG_START": "0"}, monkeypatch)
        on = _accel(name, frame, 0, {"DT_SG_START": "1"}, monkeypatch)
        for k in ("sg_cells", "sg_tree_cells", "sg_umbra_cells", "sg_lights"):
            assert on[k] == off[k], (name, k)
        assert on["sg_list_entries"] <= (1 - least) * off["sg_list_entries"], (name, on["sg_list_entries"], off["sg_list_entries"])


def test_shadow_grid_quadric_hull_culling(monkeypatch):
    """Hull culling of sphere and cylinder leaves (host_shadowgrid.cpp header, round 6) only
    removes (leaf, cell) pairs: the same cells, tree-walk cells and umbra cells; C5 frame 1920's
    tunnel (cylinder columns) loses at least 10% of its list entries, C3's room at least 1%."""
    for name, frame, least in (("c3", 240, 0.01), ("c5-1920", 1920, 0.10)):
        off = _accel(name, frame, 0, {"DT_SG_START": "0", "DT_SG_QUAD": "0"}, monkeypatch)
        on = _accel(name, frame, 0, {"DT_SG_START": "0", "DT_SG_QUAD": "1"}, monkeypatch)
        for k in ("sg_cells", "sg_tree_cells", "sg_umbra_cells", "sg_lights"):
            assert on[k] == off[k], (name, k)
        assert on["sg_list_entries"] <= (1 - least) * off["sg_list_entries"], (name, on["sg_list_entries"], off["sg_list_entries"])
