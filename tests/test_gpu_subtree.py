"""Shadow-grid block subtrees (host_shadowgrid.cpp, DT_SG_SUBTREE=1): pass-0 shadow waves whose
lanes all lie in one block of a cell that walks the tree (a list over the cap: C4's mesh cells)
walk an SAH subtree over the leaves the block's swept box to the light can meet, instead of the
whole tree. Every leaf that can hold an occluder of a segment from the block is in it, and the box
and shape tests are the tree walk's (render_final_project.cpp:806-855, geometry.cpp:2657-2740), so
the image and the shadow-ray count must equal the tree walks' bit for bit, at several block sizes,
and the oracle's."""
import numpy as np
import pytest
import torch

import distraytracer_amd as dt
import oracle
from parity_check import assert_parity, log_equal

pytestmark = pytest.mark.gpu


def _c4_share(spp):
    g = dt.globals_default()
    g.use_model = 1
    built = dt.build_scene("final", 240, g)
    g.xRes, g.yRes, g.antialias_samples, g.max_depth, g.brdf_samples = 1920, 1080, spp, 8, 2
    # rank 0's share of a 256-way split of 8x8 tiles: ~8k pixels spread over the frame, the
    # meshes included
    return g, built, dt.tiles(tile_w=8, tile_h=8, rank=0, world=256, layout=dt.DT_OUT_SLAB)


def _render(built, g, tile):
    scene = dt.Scene(built, g)
    out = torch.zeros(dt.slab_floats(g, tile), dtype=torch.float32, device="cuda")
    st = dt.render(scene, g, 240, out, tile)
    scene.close()
    return out.cpu().numpy(), st


def test_block_subtrees_match_tree_walks(cuda, monkeypatch):
    g, built, tile = _c4_share(64)
    for k in ("DT_SG_SUBTREE", "DT_SG_SUB_BLOCK", "DT_SHADOW_GRID"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("DT_SHADOW_GRID", "0")
    ref_img, ref_st = _render(built, g, tile)
    monkeypatch.setenv("DT_SHADOW_GRID", "1")
    base_img, base_st = _render(built, g, tile)
    assert base_st.shadow_rays == ref_st.shadow_rays
    log_equal("C4 share: shadow grid vs tree walks", base_img, ref_img)
    monkeypatch.setenv("DT_SG_SUBTREE", "1")
    for blk in ("8x4", "4x2", "16x8"):
        monkeypatch.setenv("DT_SG_SUB_BLOCK", blk)
        img, st = _render(built, g, tile)
        assert st.shadow_rays == ref_st.shadow_rays and st.rays == ref_st.rays, blk
        log_equal("C4 share: block subtrees %s vs tree walks" % blk, img, ref_img)


def test_block_subtrees_oracle(cuda, monkeypatch):
    monkeypatch.setenv("DT_SG_SUBTREE", "1")
    g, built, tile = _c4_share(16)
    img, st = _render(built, g, tile)
    ref = np.zeros(dt.slab_floats(g, tile), dtype=np.float32)
    _, rst = oracle.render(built, g, 240, tile, out=ref)
    assert st.rays == rst.rays and st.shadow_rays == rst.shadow_rays
    assert_parity("C4 share (16 spp) with block subtrees vs oracle", img, ref)
