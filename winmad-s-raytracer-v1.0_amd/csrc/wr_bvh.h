// Verified BVH closest hit: a second acceleration structure that finds the
// same winner as the reference's KD traversal (KDtreeAccel::traverse,
// src/scene/KDtreeAccel.cpp:309-388) with far less work, or hands the ray to
// the faithful KD kernel (wr_traverse.h) when it cannot prove that.
//
// Why the winner can be found without the reference's tree.  The reference
// tests, in leaf order, every triangle of every leaf its ray crosses (no early
// exit) and keeps a hit iff `cmp(t - best) < 0` (first found wins within EPS).
// Triangle::hit (triangle.cpp:22-87) depends only on (ray, triangle).  Let m be
// the hit with the smallest t over ALL triangles of the scene.  If
//   (1) m is in a leaf the reference visits (checked by replaying the
//       reference's near/far decisions down the root-to-leaf path of m's
//       leaves with the same float operations), and
//   (2) every other triangle's hit t_h has fl(t_h - t_m) > EPS,
// then m is taken whenever the reference reaches it (every earlier best is an
// accepted hit of another triangle, so cmp(t_m - best) < 0) and nothing after
// it can replace it (t_h >= t_m gives cmp(t_h - t_m) >= 0).  So the reference
// returns exactly (t_m, m).  A miss everywhere is a miss for the reference.
// Any ray failing (1) or (2) -- near-ties (e.g. hits on a shared mesh edge,
// where the EPS-fattened barycentrics of both triangles accept), or a smallest
// hit in a leaf the reference never reaches -- is traced by the faithful kernel.
//
// The BVH search must report every hit with t <= t_m + 2 EPS.  Its boxes are
// the triangles' boxes grown by the EPS fattening of Triangle::hit
// (barycentrics down to -EPS, so hits lie up to ~EPS x edge outside the
// triangle) with a tenfold margin, and each ray widens them further by
// 1e-4 x (its distance + 1) for the float error of the Cramer solve.  That
// covers every test whose barycentric error is below ~9 EPS, i.e. every ray not
// within ~1e-3 rad of grazing the triangle's plane; a test closer to
// degenerate (denominator at the rounding noise of the Cramer sums) yields a
// t the reference itself only gets by rounding, and is the documented residual
// (measured 0 mismatches against the faithful kernel).
#pragma once
#include <stdint.h>

namespace wrf {

// 64 bytes: the two children's boxes and links.
//   b[0..5]  child 0 box (lo.xyz, hi.xyz), b[6..11] child 1 box
//   c[0], c[1] links: >= 0 inner node index; < 0 leaf, ~link = first << 3 | (count - 1)
//   (an empty child has an inverted box and never hits)
struct BNode {
  float b[12];
  int32_t c[4];
};
static_assert(sizeof(BNode) == 64, "BVH node record is 64 bytes");

// 128 bytes (one cache line): a 4-wide node of the search, collapsed from the
// binary BVH (same leaves).  Boxes by axis across the children, then links:
//   lo[a][k], hi[a][k]  child k's box; c[k] child link as in BNode (empty
//   slot: inverted box, never hit)
struct BNode4 {
  float lo[3][4];
  float hi[3][4];
  int32_t c[4];
  int32_t pad[4];
};
static_assert(sizeof(BNode4) == 128, "4-wide BVH node is 128 bytes");

// 64 bytes (half a cache line): the 4-wide node with its child boxes quantised
// to bytes on a per-node grid as BNode8 does (decoded fmaf(q, scale[a],
// org[a]), each decoded box containing the binary tree's box bit for bit) --
// twice the nodes per line of BNode4, for scenes whose tree outgrows the L2.
// Layout (float4 words):
//   [0] org.xyz, scale.x    [1] scale.y, scale.z, qlo.x[0..3], qlo.y[0..3]
//   [2] qlo.z[0..3], qhi.x[0..3], qhi.y[0..3], qhi.z[0..3]
//   [3] c[0..3]  (links as in BNode; kEmptyLink: no child in the slot)
struct BNode4Q {
  float org[3];
  float scale[3];
  uint8_t qlo[3][4];
  uint8_t qhi[3][4];
  int32_t c[4];
};
static_assert(sizeof(BNode4Q) == 64, "quantised 4-wide BVH node is 64 bytes");
constexpr int32_t kEmptyLink = static_cast<int32_t>(0x80000000u);  // BNode4Q: an unused child slot
#ifndef WR_BVH4_QUANT
#define WR_BVH4_QUANT 0  // 1: the 4-wide search reads BNode4Q (measured C4 -1.3 %)
#endif
#if WR_BVH4_QUANT
using BNode4S = BNode4Q;  // the 4-wide search's node
#else
using BNode4S = BNode4;
#endif

// 128 bytes (one cache line): an 8-wide node of the search, collapsed from the
// binary BVH (same leaves), with child boxes quantised to bytes on a per-node
// grid.  Child k's face on axis a is decoded as fmaf(q, scale[a], org[a]) (one
// correctly rounded operation, the same on the host and the device); the build
// picks each q so that the decoded box CONTAINS the binary tree's box, bit for
// bit checked, so the search's boxes only grow and every argument about its
// margins holds unchanged.  Layout (float4 words):
//   [0] org.xyz, scale.x   [1] scale.y, scale.z, n (children), 0
//   [2] c[0..3]            [3] c[4..7]          (links as in BNode; slots >= n unused)
//   [4] qlo.x[0..7], qlo.y[0..7]   [5] qlo.z[0..7], qhi.x[0..7]
//   [6] qhi.y[0..7], qhi.z[0..7]   [7] unused
struct BNode8 {
  float org[3];
  float scale[3];
  int32_t n, pad0;
  int32_t c[8];
  uint8_t qlo[3][8];
  uint8_t qhi[3][8];
  uint8_t pad1[16];
};
static_assert(sizeof(BNode8) == 128, "8-wide BVH node is 128 bytes");

// 48 bytes per triangle, in BVH leaf order, laid out as the KD refs
// (wr_traverse.h): (p0.xyz, A), (B, C, D, E), (F, prim, lb, ln) with A..F =
// p0 - p1, p0 - p2 exactly as Triangle::hit forms them and [lb, lb + ln) the
// primitive's range of prim_leaf.  A sphere: (centre, r), 0, (0, -(prim + 1),
// lb, ln) -- Sphere::hit reads its geometry from the primitive arrays.
struct TriRec {
  float a[4], b[4], c[4];
};
static_assert(sizeof(TriRec) == 48, "BVH triangle record is 48 bytes");

// KD membership data.  Leaf path record at path[off] (off even: 16-byte
// aligned): header (n, 0), (cell lo.x, lo.y), (lo.z, hi.x), (hi.y, hi.z) -- the
// leaf's cell, which orders the replays -- then n entries (split bits,
// axis | went_right << 2) from the root down; 8 zero entries pad the array's end.
// prim_leaf[prim_leaf_off[p] .. prim_leaf_off[p+1]) = path offsets of the KD
// leaves that hold primitive p (ascending), prim_leaf_pos = its index in each
// leaf's list; node_path maps a KD leaf node to its record.
// 128 bytes per primitive (one cache line): the cells and path record offsets
// of its first four KD leaves, for the membership test of a winning primitive
// without index lookups.  Unused cells are empty (lo = +inf, hi = -inf).
struct PrimRec {
  float cell[4][6];  // lo.xyz, hi.xyz
  int32_t off[4];    // path record offsets (-1: none)
  int32_t ln;        // the primitive's KD leaf count (> 4: only the first four here)
  int32_t pad[3];
};
static_assert(sizeof(PrimRec) == 128, "primitive membership record is 128 bytes");

#ifndef WR_BVH_WIDE
#define WR_BVH_WIDE 2  // the search's tree: 2 = BNode, 4 = BNode4, 8 = BNode8
#endif
#ifndef WR_BVH_LEAF
// 2: the search keeps 2 instead of 4 triangle records in flight per leaf
// (79 instead of 95 VGPRs, 6 waves per SIMD); the SAH build rarely makes
// larger leaves anyway (torus: none).  Measured at 64 iterations, BVH mode,
// leaf 4 -> 2: C2 2,370 -> 2,411, VCM 1,670 -> 1,694, C4 759 -> 809, C3
// 2,432 -> 2,480 Mrays/s
#define WR_BVH_LEAF 2
#endif
#ifndef WR_BVH_BOX_GROW
#define WR_BVH_BOX_GROW 0.002f
#endif
#ifndef WR_BVH_RAY_GROW
#define WR_BVH_RAY_GROW 1e-4f
#endif
constexpr int kMaxLeaf = WR_BVH_LEAF;  // triangles per BVH leaf (<= 8)
constexpr int kMaxBvhDepth = 62;       // deeper builds disable the fast path
constexpr float kBoxGrow = WR_BVH_BOX_GROW;  // x (|p0 - p1| + |p0 - p2|): 2x the EPS fattening (0.01: C2 -6 %)
constexpr float kRayGrow = WR_BVH_RAY_GROW;  // x (ray length to the search bound + 1), per ray
static_assert(kMaxLeaf >= 1 && kMaxLeaf <= 8, "leaf links hold count - 1 in 3 bits");

}  // namespace wrf

// host build (declared in both HIP compile passes; defined in wr_bvh.cpp)
#include <string>
#include <vector>
namespace wr {
struct Scene;
}
namespace wrf {
struct FastHost {
  std::vector<BNode> nodes;
  std::vector<BNode4S> nodes4;  // the search's tree (root 0)
  int depth4 = 0;              // deepest 4-wide node chain
  std::vector<BNode8> nodes8;  // WR_BVH_WIDE 8: the search's tree (root 0)
  int depth8 = 0;              // deepest 8-wide node chain
  std::vector<TriRec> tris;
  std::vector<int32_t> prim_leaf_off, prim_leaf, prim_leaf_pos;
  std::vector<int32_t> node_path;  // KD leaf node -> its path record offset (-1: inner node)
  std::vector<float> node_cell;    // per KD node: cell lo.xyz, 0, hi.xyz, 0
  std::vector<uint32_t> path;  // pairs
  std::vector<PrimRec> prim_rec;  // per primitive
  int depth = 0;               // deepest node chain (stack bound)
  int leaves = 0;
  int spheres = 0;             // sphere primitives in the tree
  float org_lo[3] = {0.f, 0.f, 0.f}, org_hi[3] = {0.f, 0.f, 0.f};  // where rays start (scene box + camera):
                                                                 // sphere boxes are grown for origins in it
  bool ok = false;
  std::string why;  // when !ok: why the fast path is off for this scene
};
// Build the BVH over the scene's triangles and spheres and the KD membership
// data.
// wide: the search tree built beside the binary one (4: nodes4, 8: nodes8);
// with4: the 4-wide one as well (a binary-tree scene's latency-bound renders)
void build_fast(const wr::Scene& s, FastHost& out, int wide = WR_BVH_WIDE, bool with4 = false);
// scenes of at least this many triangles search the 4-wide tree (a binary
// tree of 2^18 triangles is ~28 MB of nodes and records: past the 4 MB L2)
#ifndef WR_BVH4_MIN_TRIS
#define WR_BVH4_MIN_TRIS (1 << 18)
#endif
constexpr size_t kWide4MinTris = WR_BVH4_MIN_TRIS;
}  // namespace wrf
