// dt_scene_dev.h — device-resident scene layout (host flattener <-> HIP kernels).
//
// Layout in HBM (all arrays are tiny next to the 288 GB; the whole scene of the default
// frame is ~60 KB and lives in L2/scalar cache during a render):
//   nodes[]    BVH in the reference's traversal order (pre-order, last child first,
//              render_final_project.cpp:491-512), with skip links -> stackless,
//              wave-uniform traversal (each wave walks the union of its lanes' paths).
//   leaf_idx[] shape indices of each leaf, in leaf order.
//   hdr[]      per-shape {type, geom offset, flags}; read with a wave-uniform index.
//   geom[]     per-shape doubles, layout per type below; every value is computed on the host
//              with the same IEEE operation sequence the reference performs per call
//              (e.g. Rectangle::intersect's getNorm(start).normalized()), so precomputation
//              changes no bit of any result.
//   mat[]      per-shape shading record; read with a per-lane index (hit shape).
//   lights[]   light records.
//   tex[]      RGB8 texel pool (stb_image bytes; the renderer uses byte/255.0).
#pragma once
#include <stdint.h>

// Scene features a trace-kernel build handles (dt_kernels.hip DT_FEATURES; dt_api.cpp picks the
// build from the scene's mask): bit t for shape type t (dt.h dt_shape_type), sphere lights and
// "spherelight" emitters, rectangle lights and "rectanglelight" emitters, Oren-Nayar materials and
// glass (refraction). Point lights and Phong, Cook-Torrance and raw materials are in every build.
#define DT_FEAT_SPHL 12
#define DT_FEAT_ON 13
#define DT_FEAT_GLASS 14
#define DT_FEAT_RECTL 15
// buildFinal's room (C2, C3, C5 n < 120): cylinders, rectangles, RectPrismV2, checkerboards with a
// hole, checker cylinders, rectangle lights
#define DT_ROOM_FEATURES ((1u << 2) | (1u << 4) | (1u << 5) | (1u << 7) | (1u << 8) | (1u << DT_FEAT_RECTL))
// the room with OBJ meshes (C4): + triangles, Oren-Nayar
#define DT_MESH_FEATURES (DT_ROOM_FEATURES | (1u << 3) | (1u << DT_FEAT_ON))
// buildFinal's tunnel (C5 n >= 140) and cloud frames: cylinders, triangles, rectangles, a point light
#define DT_TUNNEL_FEATURES ((1u << 2) | (1u << 3) | (1u << 4))

namespace dtd {

struct alignas(16) DNode {
  double lb[3];
  double ub[3];
  int32_t skip;   // index of the first node after this subtree
  int32_t leaf;
  int32_t first;  // leaf: first entry in leaf_idx
  int32_t count;  // leaf: number of shapes
};

// The node as the kernels read it (one 64 B scalar load per visit): the shape header of a
// single-shape leaf is folded in, so the common leaf costs no dependent leaf_idx -> hdr loads.
enum { DN_LEAF = 1u, DN_SINGLE = 2u };
struct alignas(16) DNodeDev {
  double lb[3];
  double ub[3];
  int32_t skip;
  uint32_t meta;   // bit0 leaf, bit1 single shape, bits 4-7 shape type, bits 8-15 shape flags,
                   // bits 16-31 (fast tree) leaf rank in the reference's gather order
  int32_t first;   // single: shape id ; multi: first entry in leaf_idx
  int32_t aux;     // single: geom offset ; multi: shape count
};

struct alignas(16) DShapeHdr {
  int32_t type;
  int32_t off;     // offset into geom[] (doubles)
  uint32_t flags;  // DT_F_*
  int32_t _pad;
};

struct alignas(16) DMat {
  int32_t model, material, emit;
  uint32_t flags;
  int32_t tex;     // texture index or -1
  int32_t tex_w, tex_h, tex_ch;
  int64_t tex_off; // byte offset into tex pool
  float roughness, radius;
  // per-material constants of the BRDFs, computed on the host with the reference's expressions
  // (same IEEE double operations, no contraction): schlick's R0 (helpers.h:313-317), Oren-Nayar's
  // A and B (render_final_project.cpp:896-897)
  float ct_r0, on_a, on_b, _pad_m;
  double refr[2];
  double color[3];
  double bordercolor[3];
  double center[3];
};

struct alignas(16) DLight {
  int32_t type, shape_index, use_baxis, _pad;
  double radius;
  double center[3], color[3], baxis[3], A[3], B[3], D[3];
};

// ---- geometry record layouts (offsets in doubles) ----------------------------------------
// Rectangle plane record R (Rectangle::intersect/intersectShadow, geometry.cpp:640-741):
//   n   = normalized(normalized((B-A) x (C-A)))   (getNorm(start).normalized())
//   V1n = normalized(B-A), V2n = normalized(D-A), len1 = |B-A|, len2 = |D-A|
enum { R_A = 0, R_N = 3, R_V1N = 6, R_V2N = 9, R_LEN1 = 12, R_LEN2 = 13, R_SIZE = 14 };

// SPHERE: center, r2 = pow(radius,2)
enum { SP_C = 0, SP_R2 = 3, SP_SIZE = 4 };
// CYLINDER / CHECKER_CYLINDER: c1, c2, axis = normalized(c2-c1), r2; UV block for checker:
//   objM rows 0..2 (12), |axis|, miniu_dist, miniv_dist, bw (floats stored as double)
enum { CY_C1 = 0, CY_C2 = 3, CY_AX = 6, CY_R2 = 9, CY_M = 10, CY_NAX = 22, CY_MUD = 23,
       CY_MVD = 24, CY_BW = 25, CY_SIZE = 26 };
// TRIANGLE: A, B, C, r1 = B-A, r2 = C-A, mesh_normal, uvA, uvB, uvC
enum { TR_A = 0, TR_B = 3, TR_C = 6, TR_R1 = 9, TR_R2 = 12, TR_MN = 15, TR_UV = 18, TR_SIZE = 24 };
// RECTANGLE: R, raw A B C D, UV: ad = D-A, dc = C-D, nadc = |ad|*|dc|
enum { RC_R = 0, RC_A = 14, RC_B = 17, RC_C = 20, RC_D = 23, RC_AD = 26, RC_DC = 29, RC_NADC = 32,
       RC_SIZE = 33 };
// RECTPRISM_V2: six face records, getNorm constants, face-0 UV block
enum { PR_F = 0, PR_NBOT = 84, PR_NRIGHT = 87, PR_NFRONT = 90, PR_A = 93, PR_G = 96, PR_AD = 99,
       PR_DC = 102, PR_NADC = 105, PR_D = 106, PR_SIZE = 109 };
// CHECKERBOARD / CHECKERBOARD_HOLE: R, gn = normalized((B-A)x(C-A)) (edge test), raw A B C D,
//   hole R, S, color1, color2, color, UV: ad, dc, nadc, miniu_dist, miniv_dist, bw
enum { CK_R = 0, CK_GN = 14, CK_A = 17, CK_B = 20, CK_C = 23, CK_D = 26, CK_HOLE = 29, CK_S = 43,
       CK_COL1 = 44, CK_COL2 = 47, CK_COL = 50, CK_AD = 53, CK_DC = 56, CK_NADC = 59, CK_MUD = 60,
       CK_MVD = 61, CK_BW = 62, CK_SIZE = 63 };

// RECTPRISM_CYL (RectPrismWithCylinder, geometry.cpp:1467-1821): the box's own bounds
// (RectPrism::getBounds of the 8 vertices, used by its slab-test intersect), getNorm's normals
// (1802-1804) and A, RectPrism::getUV's block (1442-1461: ad = D-A, dc = C-D, ad x dc,
// |ad||dc|, D), the hole count, then one record per hole (Cylinder, geometry.cpp:227-240):
// c1, c2, axis, r2 at the CYLINDER offsets (CY_C1..CY_R2, so the cylinder tests take a hole
// record as is), its colour, and c1.axis, c2.axis of intersectCap (297-324)
enum { RP_LB = 0, RP_UB = 3, RP_NBOT = 6, RP_NRIGHT = 9, RP_NFRONT = 12, RP_A = 15, RP_AD = 18, RP_DC = 21,
       RP_ADC = 24, RP_NADC = 27, RP_D = 30, RP_NH = 33, RP_H = 34 };
enum { RH_C1 = 0, RH_C2 = 3, RH_AX = 6, RH_R2 = 9, RH_COL = 10, RH_C1A = 13, RH_C2A = 14, RH_SIZE = 15 };

#define DT_DN_POOL_REC 8192    // DFS work-sharing records (32 B) per resident wave (dt_trace_kernel_dn)
#define DT_MAX_SGRID 16        // lights with a shadow grid (host_shadowgrid.cpp)
#define DT_SGRID_MAX_LIST 96   // longer candidate lists: the cell walks the tree instead
#define DT_SG_REACH_DEFAULT 0.25f   // a cell's list covers points this many cells outside it
#define DT_SG_WALK 0xffffffffu   // cell record count: the list was too long, walk the tree
#define DT_SG_UMBRA 0x80000000u  // cell record offset flag: every segment to the light is occluded (host_shadowgrid.cpp)

// per-render constants (kernel argument, < 4 KB)
struct DParams {
  int32_t xRes, yRes;
  int32_t spp;            // sampled_n = int(sqrt(antialias_samples))^2 (cpp:1046,1061)
  int32_t ppw;            // pixels per wave item (spp <= 64) ; 1 otherwise
  int32_t chunks;         // ceil(spp/64)
  int32_t max_depth, brdf_samples, blur_samples, frame_range;
  int32_t frame;
  int32_t frame_prism, frame_blur, frame_cloud;
  int32_t reflect, nogloss, perlin_cloud;
  int32_t n_nodes, n_lights, n_shapes;
  int32_t n_fnodes;       // fast tree (host_fasttree.cpp); 0: every wave walks the reference tree
  int32_t n_bnodes;       // motion-blur bump tree (host_fasttree.cpp); 0: blur passes walk the reference tree
  float bump_pad;         // its leaves' y padding; lanes with |shift| > bump_pad walk the reference tree
  int32_t sg_n;           // shadow grid: lights 0..sg_n-1 (sg_base < 0: none for that light)
  int32_t sg_dim[3];
  int32_t sg_base[DT_MAX_SGRID];
  int32_t sg_base0[DT_MAX_SGRID];   // pass-0 rays (no shift): the unpadded grid when one was built
  float sg_lo[3], sg_inv[3];
  float sg_reach;         // a cell's list also covers points this many cells outside it
  float sg_ypad;          // the lists also hold for blur passes whose |shift| <= sg_ypad
  int32_t ftree_mode;     // walks that use it: bit 0 closest hit, bit 1 shadow
  int32_t boxes_ordered;  // every node of both trees has lb <= ub (finite walks take slab ends by min/max)
  int32_t pl_block, pl_nbx, pl_nby;   // primary-ray candidate lists per pl_block^2 pixels (0: none)
  int32_t pl_bump;                     // 1: blur-pass lists (bump tree) follow, cells pl_nbx*pl_nby on
  int32_t n_cloud_steps;
  int32_t item_batch;     // wave items per queue atomic (dt_api.cpp: 2 when waves take >= 64 items, else 1)
  int32_t queue_segs;     // the queue in this many contiguous segments with a counter each (DT_QSEG_*)
  int32_t prio_steps;     // DFS steps after which a wave raises its issue priority (0: never)
  int32_t ls_first;       // first area (rectangle) light: where the light-sample cache starts
  int32_t sky_defer;      // 1 spp: missed pixels are flagged, dt_sky_miss_kernel marches them per lane
  int32_t sky_again;      // builds without the in-kernel sky (DT_SKY_AGAIN): an item with a missed
                          // sample is listed (DScene::again_list) instead of stored; 2: this launch
                          // (a build with the sky) renders the listed items
  int32_t no_cull;        // 1: no t-culling of boxes (closest hit past the best t, shadow past the light):
                          // a RectPrismWithCylinder occludes beyond the light and its hole can be hit
                          // outside its box (host: no shadow grid, no primary lists either)
  int32_t bump_up_only;   // the bump tree / blur-padded lists were built for shifts >= 0 only (host_accel.cpp):
                          // a lane with a negative shift sends its wave to the reference-tree walk
  int32_t donate;         // dt_trace_kernel_dn: idle lanes take pending DFS subtrees of other lanes
  int32_t donate_after;   // ... once a pass has run this many DFS steps
  uint32_t seed;
  float aperture, focal_length, near_plane;
  float l, r, t, b;
  float refr_air, refr_glass, phong;
  float move_per_frame, accel_t;
  float saturation, cloudhoff;
  float frame_f;          // float(frame) as passed to cloudColor
  // tiles
  int32_t x0, y0, x1, y1, tw, th, rank, world, layout, tiles_x;
  int64_t n_owned_tiles;  // slots per rank: ceil(n_tiles / world), the last one may hold no tile
  int64_t n_tiles;
  int64_t n_items;
  // camera
  double eye[3], X[3], Y[3], Z[3];
  double sky_m[3][4];     // rows 0..2 of mcam / new_mcam (cpp:1013-1021)
  double default_col[3];
  double sun[3];          // sundir.normalized() (cpp:152)
  double sun_outer[3], sun_inner[3], sun_core[3], bluesky[3], redsky[3];
  // shadow-grid block subtrees (host_internal.h ShadowGrid::sub_*): blocks of sgb_bx x sgb_by x sgb_bz
  // cells, sgb_nbx x sgb_nby per layer of blocks; light l's records at sgb_base[l] (-1: none)
  int32_t sgb_base[DT_MAX_SGRID];
  int32_t sgb_bx, sgb_by, sgb_nbx, sgb_nby;
  int32_t sgb_multi;      // a wave walks the subtrees of up to this many blocks in turn (DT_SG_SUB_MULTI)
  int32_t sgb_bz;         // the blocks' depth in cells (z; DT_SG_SUB_BLOCK XxYxZ)
  // spp > 64: 1 = each 64-sample chunk of a pixel is a queue item of its own (code = pixel item *
  // chunks + chunk), so a pixel's chunks run on different waves; the chunk that completes the pixel
  // adds every sample colour in sample order (dt_kernels.hip item loop). 2 = the same with the queue
  // chunk-major (code = chunk * n_items + pixel item: a pixel's chunks far apart; the tests' check)
  int32_t chunk_items;
};

#ifndef DT_HD
#if defined(__HIPCC__)
#define DT_HD __host__ __device__ __forceinline__
#else
#define DT_HD inline
#endif
#endif

// The trace launch's counter block (dt_api.cpp STATS1): ST_N counters, the queue word, the stamps
// builds' slots, then one queue counter per segment, DT_QSEG_STRIDE words apart (own cache lines)
#define DT_N_STAMPS (72 + 3 * 8 * 256)
#define DT_QSEG_MAX 8
#define DT_QSEG_STRIDE 16
#define DT_QSEG_OFF (1 + DT_N_STAMPS)   // from the queue word
// copies 1..DT_STAT_SLOTS-1 of the ST_N counters (copy 0: the block's head), one per DT_STAT_SLOT_STRIDE
// words from DT_STAT_SLOT_OFF past the queue word: wave b adds its counters to copy b % DT_STAT_SLOTS
#define DT_STAT_SLOTS 16
#define DT_STAT_SLOT_STRIDE 32
#define DT_STAT_SLOT_OFF (DT_QSEG_OFF + DT_QSEG_MAX * DT_QSEG_STRIDE)

// Tile ownership of the multi-GPU split: the tiles (raster order over the window) fall into groups
// of `world` consecutive tiles, and slot s of rank r is tile s*world + (r + rot(s)) % world. Every
// rank takes one tile of every group, like a plain t % world interleave, but each group's ranks
// are rotated by a hash of the group: with a fixed rotation the interleave aliases with the image
// rows (1920 px = 60 tiles = 7.5 groups of 8, so ranks r and r+4 took the same tile columns, and
// at 8 GPUs the two ranks owning the window's columns ran 21% longer than the others).
DT_HD uint32_t tile_rot(int64_t slot, int world)
{
  uint32_t h = (uint32_t)slot * 2654435761u;
  h ^= h >> 15;
  h *= 0x2c1b3c6du;
  h ^= h >> 12;
  return h % (uint32_t)world;
}
DT_HD int64_t tile_of(int64_t slot, int rank, int world)
{
  return slot * world + (int64_t)(((uint32_t)rank + tile_rot(slot, world)) % (uint32_t)world);
}

}  // namespace dtd
