// Host build of the verified-BVH fast path (wr_bvh.h): a binned-SAH BVH over the
// scene's triangles and spheres, and for every primitive the root-to-leaf paths of the
// reference KD leaves that hold it (KDtreeAccel::buildTree,
// src/scene/KDtreeAccel.cpp:118-307, as restated in wr_scene.cpp).
#include "wr_bvh.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <future>

#include "wr_scene.h"

namespace wrf {
namespace {

struct Box {
  float lo[3] = {INFINITY, INFINITY, INFINITY};
  float hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  void grow(const Box& b) {
    for (int k = 0; k < 3; ++k) {
      lo[k] = std::min(lo[k], b.lo[k]);
      hi[k] = std::max(hi[k], b.hi[k]);
    }
  }
  void grow(const float* p) {
    for (int k = 0; k < 3; ++k) {
      lo[k] = std::min(lo[k], p[k]);
      hi[k] = std::max(hi[k], p[k]);
    }
  }
  bool empty() const { return !(lo[0] <= hi[0]); }
  double area() const {
    if (empty()) return 0.0;
    const double x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
    return 2.0 * (x * y + x * z + y * z);
  }
};

constexpr int kMaxBins = 256;

// build knobs (measurement only; the defaults are the measured best):
//   WR_BVH_BINS   SAH bins over the centroids of ranges above the sweep size
//   WR_BVH_SWEEP  ranges of at most this many triangles take the exact SAH sweep
//   WR_BVH_CT     cost of one node visit relative to one triangle test
//   WR_BVH_SERIAL 1: no helper threads for subtrees and splits (the same tree)
// Round 6 re-sweep on the current kernels (profiles/r6/bvh_knobs/): 64 bins
// and a node visit priced as one triangle test (was 16 and 0.5) take C2 at 20
// iterations from 3,002 to 3,107 Mrays/s (6 runs each), C3 +2.8 %, VCM
// +1.3 %, C4 and one iteration unchanged; 20.55 -> 20.12 nodes per ray
struct BuildKnobs {
  int bins = 64;
  int sweep = 0;
  double ct = 1.0;
  bool serial = false;
  BuildKnobs() {
    if (const char* e = std::getenv("WR_BVH_SERIAL")) serial = std::atoi(e) != 0;
    if (const char* e = std::getenv("WR_BVH_BINS")) bins = std::max(2, std::min(kMaxBins, std::atoi(e)));
    if (const char* e = std::getenv("WR_BVH_SWEEP")) sweep = std::max(0, std::atoi(e));
    if (const char* e = std::getenv("WR_BVH_CT")) ct = std::max(0.0, std::atof(e));
  }
};

// The right child of a split whose halves both hold >= kParallelMin
// triangles is built on its own thread (at most kMaxThreads at once) into a
// separate output, spliced after the left subtree: the layout is the serial
// build's (node, left subtree, right subtree), bit for bit.  By size, not
// depth: the SAH's top splits peel small parts (floor, glass) off the scene.
constexpr int kParallelMin = 8192;
constexpr int kMaxThreads = 32;

// relocate a child link of a subtree built into its own output
int relocate(int link, int nbase, int tbase) {
  if (link >= 0) return link + nbase;
  const int l = ~link;
  return ~((((l >> 3) + tbase) << 3) | (l & 7));
}

struct Builder {
  const std::vector<Box>& box;
  const std::vector<float>& cen;  // 3 per triangle
  std::vector<int>& idx;
  FastHost& out;
  const wr::Scene& s;
  const std::vector<int>& tri_prim;
  const std::vector<int32_t>& leaf_off;  // prim_leaf_off of the whole build
  std::atomic<int>& threads;             // helper threads running
  BuildKnobs K;
  std::vector<int> tmp;
  std::vector<double> rarea;
  std::vector<Box> bins;  // 2 x K.bins: the bins, then the right-side prefixes
  std::vector<int> bcount;

  int leaf_link(int b, int e) {
    const int first = static_cast<int>(out.tris.size());
    for (int i = b; i < e; ++i) {
      const wr::Prim& p = s.prims[tri_prim[idx[i]]];
      TriRec r;
      const int32_t prim = tri_prim[idx[i]];
      if (p.type == wr::kTri) {
        // A..F exactly as Triangle::hit forms them (triangle.cpp:24-30)
        r.a[0] = p.p0.x;
        r.a[1] = p.p0.y;
        r.a[2] = p.p0.z;
        r.a[3] = p.p0.x - p.p1.x;
        r.b[0] = p.p0.y - p.p1.y;
        r.b[1] = p.p0.z - p.p1.z;
        r.b[2] = p.p0.x - p.p2.x;
        r.b[3] = p.p0.y - p.p2.y;
        r.c[0] = p.p0.z - p.p2.z;
        std::memcpy(&r.c[1], &prim, 4);
      } else {
        // a sphere: -(prim + 1) as in the KD refs (wr_traverse.h); Sphere::hit
        // reads its centre, radius and box from the primitive arrays
        r.a[0] = p.c.x;
        r.a[1] = p.c.y;
        r.a[2] = p.c.z;
        r.a[3] = p.r;
        r.b[0] = r.b[1] = r.b[2] = r.b[3] = 0.f;
        r.c[0] = 0.f;
        const int32_t code = -(prim + 1);
        std::memcpy(&r.c[1], &code, 4);
      }
      // the primitive's KD leaf list (prim_leaf range): no extra lookup when it wins
      const int32_t lb = leaf_off[static_cast<size_t>(prim)];
      const int32_t ln = leaf_off[static_cast<size_t>(prim) + 1] - lb;
      std::memcpy(&r.c[2], &lb, 4);
      std::memcpy(&r.c[3], &ln, 4);
      out.tris.push_back(r);
    }
    ++out.leaves;
    return ~((first << 3) | (e - b - 1));
  }

  Box bounds(int b, int e) const {
    Box r;
    for (int i = b; i < e; ++i) r.grow(box[idx[i]]);
    return r;
  }

  // exact SAH sweep: every split position of the centroid order on each axis
  int split_sweep(int b, int e, const Box& nb) {
    const int n = e - b;
    double best = INFINITY;
    int bax = -1, bk = 0;
    tmp.assign(idx.begin() + b, idx.begin() + e);
    rarea.resize(static_cast<size_t>(n) + 1);
    for (int ax = 0; ax < 3; ++ax) {
      std::sort(tmp.begin(), tmp.end(), [&](int x, int y) {
        const float cx = cen[3 * x + ax], cy = cen[3 * y + ax];
        return cx < cy || (cx == cy && x < y);
      });
      Box acc;
      for (int k = n - 1; k > 0; --k) {
        acc.grow(box[tmp[static_cast<size_t>(k)]]);
        rarea[static_cast<size_t>(k)] = acc.area();
      }
      Box la;
      for (int k = 1; k < n; ++k) {
        la.grow(box[tmp[static_cast<size_t>(k - 1)]]);
        const double cost = la.area() * k + rarea[static_cast<size_t>(k)] * (n - k);
        if (cost < best) {
          best = cost;
          bax = ax;
          bk = k;
        }
      }
    }
    if (n <= kMaxLeaf && (bax < 0 || best + K.ct * nb.area() >= nb.area() * n)) return -1;
    if (bax < 0) return b + n / 2;
    std::sort(idx.begin() + b, idx.begin() + e, [&](int x, int y) {
      const float cx = cen[3 * x + bax], cy = cen[3 * y + bax];
      return cx < cy || (cx == cy && x < y);
    });
    return b + bk;
  }

  // the binned SAH over one axis: the cheapest split bin (first of equals)
  void axis_best(int b, int e, const Box& cb, int ax, Box* bb, int* bc, double& best, int& bbin) const {
    const int kBins = K.bins;
    const float ext = cb.hi[ax] - cb.lo[ax];
    best = INFINITY;
    bbin = -1;
    if (!(ext > 0.f)) return;
    Box* rb = bb + kBins;
    int* rc = bc + kBins;
    for (int k = 0; k < 2 * kBins; ++k) {  // only the bins in use are cleared
      bb[k] = Box();
      bc[k] = 0;
    }
    const float sc = kBins / ext;
    for (int i = b; i < e; ++i) {
      int k = static_cast<int>((cen[3 * idx[i] + ax] - cb.lo[ax]) * sc);
      k = std::min(kBins - 1, std::max(0, k));
      bb[k].grow(box[idx[i]]);
      ++bc[k];
    }
    Box acc;
    int an = 0;
    for (int k = kBins - 1; k > 0; --k) {
      acc.grow(bb[k]);
      an += bc[k];
      rb[k] = acc;
      rc[k] = an;
    }
    Box la;
    int ln = 0;
    for (int k = 0; k < kBins - 1; ++k) {
      la.grow(bb[k]);
      ln += bc[k];
      if (ln == 0 || rc[k + 1] == 0) continue;
      const double cost = la.area() * ln + rb[k + 1].area() * rc[k + 1];
      if (cost < best) {
        best = cost;
        bbin = k + 1;
      }
    }
  }

  // split [b, e) by SAH over the centroids (binned, or swept for small ranges);
  // returns the split position (b < m < e) or -1 when a leaf is cheaper (only
  // allowed for e - b <= kMaxLeaf)
  int split(int b, int e, const Box& nb) {
    const int n = e - b;
    if (n <= K.sweep) return split_sweep(b, e, nb);
    const int kBins = K.bins;
    Box cb;
    for (int i = b; i < e; ++i) cb.grow(&cen[3 * idx[i]]);
    double cost[3];
    int cbin[3];
    bins.resize(6 * static_cast<size_t>(kBins));
    bcount.resize(6 * static_cast<size_t>(kBins));
    auto axis = [&](int ax) {
      axis_best(b, e, cb, ax, bins.data() + 2 * kBins * ax, bcount.data() + 2 * kBins * ax, cost[ax], cbin[ax]);
    };
    if (n >= 8 * kParallelMin && !K.serial) {  // the top splits: one axis per thread
      auto f1 = std::async(std::launch::async, axis, 1);
      auto f2 = std::async(std::launch::async, axis, 2);
      axis(0);
      f1.get();
      f2.get();
    } else {
      for (int ax = 0; ax < 3; ++ax) axis(ax);
    }
    double best = INFINITY;
    int bax = -1, bbin = 0;
    for (int ax = 0; ax < 3; ++ax)
      if (cbin[ax] >= 0 && cost[ax] < best) {
        best = cost[ax];
        bax = ax;
        bbin = cbin[ax];
      }
    if (n <= kMaxLeaf) {
      // leaf cost n tests vs 1 node + the children's tests
      const double leaf = nb.area() * n;
      if (bax < 0 || best + K.ct * nb.area() >= leaf) return -1;
    }
    if (bax < 0) return b + n / 2;  // all centroids equal: split by index
    const float ext = cb.hi[bax] - cb.lo[bax];
    const float sc = kBins / ext;
    auto mid = std::partition(idx.begin() + b, idx.begin() + e, [&](int t) {
      int k = static_cast<int>((cen[3 * t + bax] - cb.lo[bax]) * sc);
      k = std::min(kBins - 1, std::max(0, k));
      return k < bbin;
    });
    int m = static_cast<int>(mid - idx.begin());
    if (m <= b || m >= e) m = b + n / 2;
    return m;
  }

  // child link for [b, e) with bounds cb
  int child(int b, int e, const Box& cb, int depth) {
    if (e - b <= kMaxLeaf) {
      const int m = split(b, e, cb);
      if (m < 0) return leaf_link(b, e);
      return inner(b, e, m, depth);
    }
    return inner(b, e, split(b, e, cb), depth);
  }

  int inner(int b, int e, int m, int depth) {
    out.depth = std::max(out.depth, depth);
    if (depth > kMaxBvhDepth) {
      out.ok = false;
      out.why = "BVH deeper than the traversal stack";
      return leaf_link(b, std::min(e, b + kMaxLeaf));
    }
    const int at = static_cast<int>(out.nodes.size());
    out.nodes.emplace_back();
    const Box l = bounds(b, m), r = bounds(m, e);
    int cl, cr;
    bool spawn = !K.serial && m - b >= kParallelMin && e - m >= kParallelMin;
    if (spawn && threads.fetch_add(1) >= kMaxThreads) {
      threads.fetch_sub(1);
      spawn = false;
    }
    if (spawn) {
      // [b, m) and [m, e) are disjoint ranges of idx: independent subtrees
      FastHost sub;
      sub.ok = true;
      Builder rb{box, cen, idx, sub, s, tri_prim, leaf_off, threads};
      int rl = 0;
      auto fut = std::async(std::launch::async, [&] { rl = rb.child(m, e, r, depth + 1); });
      cl = child(b, m, l, depth + 1);
      fut.get();
      threads.fetch_sub(1);
      const int nbase = static_cast<int>(out.nodes.size()), tbase = static_cast<int>(out.tris.size());
      for (BNode n : sub.nodes) {
        n.c[0] = relocate(n.c[0], nbase, tbase);
        n.c[1] = relocate(n.c[1], nbase, tbase);
        out.nodes.push_back(n);
      }
      out.tris.insert(out.tris.end(), sub.tris.begin(), sub.tris.end());
      out.leaves += sub.leaves;
      out.depth = std::max(out.depth, sub.depth);
      if (!sub.ok && out.ok) {
        out.ok = false;
        out.why = sub.why;
      }
      cr = relocate(rl, nbase, tbase);
    } else {
      cl = child(b, m, l, depth + 1);
      cr = child(m, e, r, depth + 1);
    }
    BNode& nd = out.nodes[static_cast<size_t>(at)];
    for (int k = 0; k < 3; ++k) {
      nd.b[k] = l.lo[k];
      nd.b[3 + k] = l.hi[k];
      nd.b[6 + k] = r.lo[k];
      nd.b[9 + k] = r.hi[k];
    }
    nd.c[0] = cl;
    nd.c[1] = cr;
    nd.c[2] = nd.c[3] = 0;
    return at;
  }
};

void kd_paths(const wr::Scene& s, FastHost& out) {
  const size_t np = s.prims.size();
  // every (primitive, leaf record, position in the leaf) in walk order; grouped
  // by primitive afterwards by a stable counting sort (the walk is pre-order,
  // so each primitive's records come out ascending)
  struct Ref {
    int32_t prim, off, pos;
  };
  std::vector<Ref> refs;
  refs.reserve(s.refs.size());
  std::vector<uint32_t> cur;  // entries of the current path
  struct Item {
    int node;
    int depth;            // entries on the path to this node
    uint32_t e0, e1;      // the entry that led here (valid if depth > 0)
    float lo[3], hi[3];   // the node's cell: the root box cut by the splits above
  };
  std::vector<Item> st;
  out.node_path.assign(s.nodes.size(), -1);
  out.node_cell.assign(8 * s.nodes.size(), 0.f);
  st.push_back({0, 0, 0u, 0u, {s.root_l.x, s.root_l.y, s.root_l.z}, {s.root_r.x, s.root_r.y, s.root_r.z}});
  while (!st.empty()) {
    const Item it = st.back();
    st.pop_back();
    cur.resize(2 * static_cast<size_t>(it.depth));
    if (it.depth > 0) {
      cur[2 * (it.depth - 1)] = it.e0;
      cur[2 * (it.depth - 1) + 1] = it.e1;
    }
    const wr::KdNode& k = s.nodes[static_cast<size_t>(it.node)];
    for (int a = 0; a < 3; ++a) {  // the node's cell (targeted walks prune by it)
      out.node_cell[8 * static_cast<size_t>(it.node) + a] = it.lo[a];
      out.node_cell[8 * static_cast<size_t>(it.node) + 4 + a] = it.hi[a];
    }
    if (k.axis >= 0) {
      uint32_t bits;
      std::memcpy(&bits, &k.split, 4);
      Item r = {k.right, it.depth + 1, bits, static_cast<uint32_t>(k.axis) | 4u, {}, {}};
      Item l = {it.node + 1, it.depth + 1, bits, static_cast<uint32_t>(k.axis), {}, {}};
      for (int a = 0; a < 3; ++a) {
        l.lo[a] = r.lo[a] = it.lo[a];
        l.hi[a] = r.hi[a] = it.hi[a];
      }
      l.hi[k.axis] = std::min(l.hi[k.axis], k.split);
      r.lo[k.axis] = std::max(r.lo[k.axis], k.split);
      st.push_back(r);
      st.push_back(l);
    } else {
      // records start on 16-byte boundaries (even entries): read as uint4
      if ((out.path.size() / 2) & 1) {
        out.path.push_back(0u);
        out.path.push_back(0u);
      }
      const int32_t off = static_cast<int32_t>(out.path.size() / 2);
      out.node_path[static_cast<size_t>(it.node)] = off;
      out.path.push_back(static_cast<uint32_t>(it.depth));
      out.path.push_back(0u);
      for (int a = 0; a < 3; ++a) {  // the leaf's cell (orders the replays)
        uint32_t b;
        std::memcpy(&b, &it.lo[a], 4);
        out.path.push_back(b);
      }
      for (int a = 0; a < 3; ++a) {
        uint32_t b;
        std::memcpy(&b, &it.hi[a], 4);
        out.path.push_back(b);
      }
      out.path.insert(out.path.end(), cur.begin(), cur.end());
      for (int i = 0; i < k.count; ++i) refs.push_back({s.refs[static_cast<size_t>(k.first + i)], off, i});
    }
  }
  // a primitive listed twice in one leaf keeps its first position (the leaf
  // tests it there first)
  std::vector<int32_t> last(np, -1);
  std::vector<int32_t> cnt(np + 1, 0);
  size_t kept = 0;
  for (Ref& r : refs) {
    if (last[static_cast<size_t>(r.prim)] == r.off) {
      r.prim = -1;
      continue;
    }
    last[static_cast<size_t>(r.prim)] = r.off;
    ++cnt[static_cast<size_t>(r.prim) + 1];
    ++kept;
  }
  out.prim_leaf_off.assign(np + 1, 0);
  for (size_t p = 0; p < np; ++p) out.prim_leaf_off[p + 1] = out.prim_leaf_off[p] + cnt[p + 1];
  out.prim_leaf.assign(kept, 0);
  out.prim_leaf_pos.assign(kept, 0);
  {
    std::vector<int32_t> at(out.prim_leaf_off.begin(), out.prim_leaf_off.end() - 1);
    for (const Ref& r : refs) {
      if (r.prim < 0) continue;
      const int32_t j = at[static_cast<size_t>(r.prim)]++;
      out.prim_leaf[static_cast<size_t>(j)] = r.off;
      out.prim_leaf_pos[static_cast<size_t>(j)] = r.pos;
    }
  }
  // the replay reads 8 entries at a time: pad past the last record
  out.path.resize(out.path.size() + 2 * 8, 0u);
  // per primitive: its first four leaves' cells and records in one line
  out.prim_rec.assign(np, PrimRec{});
  for (size_t p = 0; p < np; ++p) {
    PrimRec& r = out.prim_rec[p];
    const int32_t lb = out.prim_leaf_off[p];
    r.ln = out.prim_leaf_off[p + 1] - lb;
    for (int k = 0; k < 4; ++k) {
      const bool have = k < r.ln;
      const int32_t off = have ? out.prim_leaf[static_cast<size_t>(lb + k)] : -1;
      r.off[k] = off;
      for (int a = 0; a < 6; ++a) {
        float v = a < 3 ? INFINITY : -INFINITY;
        if (have) std::memcpy(&v, &out.path[2 * static_cast<size_t>(off) + 2 + static_cast<size_t>(a)], 4);
        r.cell[k][a] = v;
      }
    }
  }
}

// One axis of a quantised node (BNode4Q, BNode8): the grid (org, scale) and
// each child's bytes, with the decoded faces fmaf(q, scale, org) holding the
// child's [lo, hi] -- checked with the same correctly rounded fmaf the device
// decodes with.
void quantise_axis(const float* clo, const float* chi, int n, float& org, float& scale, uint8_t* qlo, uint8_t* qhi) {
  float lo = INFINITY, hi = -INFINITY;
  for (int i = 0; i < n; ++i) {
    lo = std::min(lo, clo[i]);
    hi = std::max(hi, chi[i]);
  }
  if (n == 0) {
    org = 0.f;
    scale = 1.f;
    return;
  }
  // the smallest power of two with (hi - lo) / scale <= 254 (one step spare
  // for the outward corrections below)
  int e = -126;
  const double ext = static_cast<double>(hi) - static_cast<double>(lo);
  while (std::ldexp(254.0, e) < ext) ++e;
  for (;; ++e) {
    const float sc = std::ldexp(1.f, e);
    bool ok = true;
    for (int i = 0; i < n && ok; ++i) {
      double ql = std::floor((static_cast<double>(clo[i]) - lo) / sc);
      double qh = std::ceil((static_cast<double>(chi[i]) - lo) / sc);
      ql = std::max(0.0, ql);
      while (ql > 0 && std::fma(static_cast<float>(ql), sc, lo) > clo[i]) ql -= 1;
      while (qh <= 255 && std::fma(static_cast<float>(qh), sc, lo) < chi[i]) qh += 1;
      if (std::fma(static_cast<float>(ql), sc, lo) > clo[i] || qh > 255) {
        ok = false;
        break;
      }
      qlo[i] = static_cast<uint8_t>(ql);
      qhi[i] = static_cast<uint8_t>(qh);
    }
    if (ok) {
      org = lo;
      scale = sc;
      return;
    }
  }
}

// The 4-wide tree: each node takes its binary node's children and opens the
// inner child of largest area until it holds four (or only leaves remain).
struct Collapse {
  FastHost& out;
  struct Kid {
    float lo[3], hi[3];
    int link;
    double area() const {
      if (!(lo[0] <= hi[0])) return 0.0;
      const double x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
      return 2.0 * (x * y + x * z + y * z);
    }
  };
  Kid kid(int n2, int side) const {
    const BNode& b = out.nodes[static_cast<size_t>(n2)];
    Kid k;
    for (int a = 0; a < 3; ++a) {
      k.lo[a] = b.b[6 * side + a];
      k.hi[a] = b.b[6 * side + 3 + a];
    }
    k.link = b.c[side];
    return k;
  }
  int node(int n2, int depth) {
    out.depth4 = std::max(out.depth4, depth);
    Kid ks[4] = {kid(n2, 0), kid(n2, 1), {}, {}};
    int n = 2;
    while (n < 4) {
      int best = -1;
      double ba = -1.0;
      for (int i = 0; i < n; ++i)
        if (ks[i].link >= 0 && ks[i].area() > ba) {
          ba = ks[i].area();
          best = i;
        }
      if (best < 0) break;
      const int open = ks[best].link;
      ks[best] = kid(open, 0);
      ks[n++] = kid(open, 1);
    }
#if WR_BVH4_QUANT
    int m = 0;  // drop empty children (the binary root of a tiny scene)
    for (int i = 0; i < n; ++i)
      if (!(!(ks[i].lo[0] <= ks[i].hi[0]) || (ks[i].lo[0] == 3e38f && ks[i].hi[0] == 3e38f))) ks[m++] = ks[i];
    n = m;
#endif
    const int at = static_cast<int>(out.nodes4.size());
    out.nodes4.emplace_back();
    int links[4];
    for (int i = 0; i < 4; ++i) links[i] = i < n && ks[i].link >= 0 ? node(ks[i].link, depth + 1) : (i < n ? ks[i].link : ~0);
#if WR_BVH4_QUANT
    BNode4Q& q = out.nodes4[static_cast<size_t>(at)];
    std::memset(&q, 0, sizeof q);
    for (int i = 0; i < 4; ++i) q.c[i] = i < n ? links[i] : kEmptyLink;
    float lo[4], hi[4];
    for (int a = 0; a < 3; ++a) {
      for (int i = 0; i < n; ++i) {
        lo[i] = ks[i].lo[a];
        hi[i] = ks[i].hi[a];
      }
      quantise_axis(lo, hi, n, q.org[a], q.scale[a], q.qlo[a], q.qhi[a]);
    }
    return at;
#else
    BNode4& d = out.nodes4[static_cast<size_t>(at)];
    for (int i = 0; i < 4; ++i) {
      // an empty slot is a point far outside every scene: its slab interval is
      // empty for every direction (an inverted [inf, -inf] box is not: its
      // min / max per axis span the whole line, and the slot's link -1 would
      // then test triangle 0 as a leaf)
      for (int a = 0; a < 3; ++a) {
        d.lo[a][i] = i < n ? ks[i].lo[a] : 3e38f;
        d.hi[a][i] = i < n ? ks[i].hi[a] : 3e38f;
      }
      d.c[i] = links[i];
      d.pad[i] = 0;
    }
    return at;
#endif
  }
};

// The 8-wide tree: as Collapse, up to eight children, their boxes quantised
// outward to bytes on a per-node power-of-two grid (BNode8).
struct Collapse8 {
  FastHost& out;
  struct Kid {
    float lo[3], hi[3];
    int link;
    double area() const {
      if (!(lo[0] <= hi[0])) return 0.0;
      const double x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
      return 2.0 * (x * y + x * z + y * z);
    }
  };
  Kid kid(int n2, int side) const {
    const BNode& b = out.nodes[static_cast<size_t>(n2)];
    Kid k;
    for (int a = 0; a < 3; ++a) {
      k.lo[a] = b.b[6 * side + a];
      k.hi[a] = b.b[6 * side + 3 + a];
    }
    k.link = b.c[side];
    return k;
  }
  static bool empty(const Kid& k) { return !(k.lo[0] <= k.hi[0]) || (k.lo[0] == 3e38f && k.hi[0] == 3e38f); }
  // one axis of a node: the grid (org, scale) and each child's bytes, with the
  // decoded faces fmaf(q, scale, org) holding the child's [lo, hi]
  static void quantise(const Kid* ks, int n, int a, BNode8& d) {
    float lo = INFINITY, hi = -INFINITY;
    for (int i = 0; i < n; ++i) {
      lo = std::min(lo, ks[i].lo[a]);
      hi = std::max(hi, ks[i].hi[a]);
    }
    // the smallest power of two with (hi - lo) / scale <= 254 (one step spare
    // for the outward corrections below)
    int e = -126;
    const double ext = static_cast<double>(hi) - static_cast<double>(lo);
    while (std::ldexp(254.0, e) < ext) ++e;
    for (;; ++e) {
      const float sc = std::ldexp(1.f, e);
      bool ok = true;
      for (int i = 0; i < n && ok; ++i) {
        double ql = std::floor((static_cast<double>(ks[i].lo[a]) - lo) / sc);
        double qh = std::ceil((static_cast<double>(ks[i].hi[a]) - lo) / sc);
        ql = std::max(0.0, ql);
        while (ql > 0 && std::fma(static_cast<float>(ql), sc, lo) > ks[i].lo[a]) ql -= 1;
        while (qh <= 255 && std::fma(static_cast<float>(qh), sc, lo) < ks[i].hi[a]) qh += 1;
        if (std::fma(static_cast<float>(ql), sc, lo) > ks[i].lo[a] || qh > 255) {
          ok = false;
          break;
        }
        d.qlo[a][i] = static_cast<uint8_t>(ql);
        d.qhi[a][i] = static_cast<uint8_t>(qh);
      }
      if (ok) {
        d.org[a] = lo;
        d.scale[a] = sc;
        return;
      }
    }
  }
  int node(int n2, int depth) {
    out.depth8 = std::max(out.depth8, depth);
    Kid ks[8] = {kid(n2, 0), kid(n2, 1)};
    int n = 2;
    while (n < 8) {
      int best = -1;
      double ba = -1.0;
      for (int i = 0; i < n; ++i)
        if (ks[i].link >= 0 && ks[i].area() > ba) {
          ba = ks[i].area();
          best = i;
        }
      if (best < 0) break;
      const int open = ks[best].link;
      ks[best] = kid(open, 0);
      ks[n++] = kid(open, 1);
    }
    int m = 0;  // drop empty children (the binary root of a tiny scene)
    for (int i = 0; i < n; ++i)
      if (!empty(ks[i])) ks[m++] = ks[i];
    n = m;
    const int at = static_cast<int>(out.nodes8.size());
    out.nodes8.emplace_back();
    int links[8];
    for (int i = 0; i < n; ++i) links[i] = ks[i].link >= 0 ? node(ks[i].link, depth + 1) : ks[i].link;
    BNode8& d = out.nodes8[static_cast<size_t>(at)];
    std::memset(&d, 0, sizeof d);
    d.n = n;
    for (int i = 0; i < 8; ++i) d.c[i] = i < n ? links[i] : 0;
    for (int a = 0; a < 3; ++a) quantise(ks, n, a, d);
    return at;
  }
};

}  // namespace

// Sphere::hit (sphere.cpp:17-78) forms t = t_ca -+ sqrt(t_hc), t_hc = r^2 -
// |oc|^2 + t_ca^2 with oc = centre - origin: a sum of terms of magnitude up to
// M^2 (M = |oc| or r) whose float rounding moves t_hc by up to ~1.2e-6 M^2.
// The square root turns that into an error of t of at most 2.7e-5 M^2 when the
// accepted t_hc (> EPS) is far above the noise, and of up to ~2 sqrt(1.2e-6) M
// where the noise decides (a ray at the sphere's rim; there the "hit" lies
// within r + 2.2e-3 M of the centre).  So every t Sphere::hit accepts lies on
// the ray within sphere_grow(M) of the sphere's box, with M bounded by the
// distance of the ray's origin from the centre plus r: the BVH boxes of
// spheres are grown by that for every origin in the region the render's rays
// start from (the scene's box and the camera: FastHost::org_lo / org_hi), and
// the search sends a ray from outside it to the KD walk (wr_fast.h).
double sphere_grow(double M) { return 3e-5 * M * M + 2.5e-3 * M + 2.0 * 1e-3; }

void build_fast(const wr::Scene& s, FastHost& out, int wide, bool with4) {
  out = FastHost();
  if (s.prims.empty() || s.nodes.empty()) {
    out.why = "empty scene";
    return;
  }
  const size_t n = s.prims.size();
  if (n >= (size_t(1) << 29)) {  // the search marks near-ties and grazing rays in bits 30, 29 of a primitive (wr_fast.h)
    out.why = "2^29 primitives or more";
    return;
  }
  std::vector<Box> box(n);
  std::vector<float> cen(3 * n);
  std::vector<int> tri_prim(n), idx(n);
  // where the renderer's rays start: the scene (its KD root box) and the camera
  {
    const float rl[3] = {s.root_l.x, s.root_l.y, s.root_l.z}, rr[3] = {s.root_r.x, s.root_r.y, s.root_r.z};
    const float cp[3] = {s.cam.pos.x, s.cam.pos.y, s.cam.pos.z};
    float ext = 0.f;
    for (int k = 0; k < 3; ++k) {
      out.org_lo[k] = std::min(rl[k], cp[k]);
      out.org_hi[k] = std::max(rr[k], cp[k]);
      ext = std::max(ext, out.org_hi[k] - out.org_lo[k]);
    }
    // slack: extension rays start EPS past a surface point, which may lie on the box
    const float slack = 0.01f * ext + 0.01f;
    for (int k = 0; k < 3; ++k) {
      out.org_lo[k] -= slack;
      out.org_hi[k] += slack;
    }
  }
  for (const auto& p : s.prims) out.spheres += p.type != wr::kTri ? 1 : 0;
  auto prep = [&](size_t i0, size_t i1) {
    for (size_t i = i0; i < i1; ++i) {
      const wr::Prim& p = s.prims[i];
      tri_prim[i] = static_cast<int>(i);
      idx[i] = static_cast<int>(i);
      if (p.type != wr::kTri) {
        // the reference's box (AABB::extend, as box.hit tests it) grown by the
        // reach of Sphere::hit's rounding for the farthest ray origin
        const float c[3] = {p.c.x, p.c.y, p.c.z};
        double M2 = 0.0;
        for (int k = 0; k < 3; ++k) {
          const double a = std::max(std::fabs(static_cast<double>(out.org_lo[k]) - c[k]),
                                    std::fabs(static_cast<double>(out.org_hi[k]) - c[k]));
          M2 += a * a;
        }
        const double M = std::sqrt(M2) + std::fabs(static_cast<double>(p.r));
        const double g = sphere_grow(M) + 1e-6 * (1.0 + std::max({std::fabs(p.bl.x), std::fabs(p.bl.y),
            std::fabs(p.bl.z), std::fabs(p.br.x), std::fabs(p.br.y), std::fabs(p.br.z)}));
        Box b;
        const float bl[3] = {p.bl.x, p.bl.y, p.bl.z}, br[3] = {p.br.x, p.br.y, p.br.z};
        for (int k = 0; k < 3; ++k) {
          b.lo[k] = std::nextafter(static_cast<float>(std::min(bl[k], c[k] - std::fabs(p.r)) - g), -INFINITY);
          b.hi[k] = std::nextafter(static_cast<float>(std::max(br[k], c[k] + std::fabs(p.r)) + g), INFINITY);
          cen[3 * i + k] = 0.5f * (b.lo[k] + b.hi[k]);
        }
        box[i] = b;
        continue;
      }
      const float v[3][3] = {{p.p0.x, p.p0.y, p.p0.z}, {p.p1.x, p.p1.y, p.p1.z}, {p.p2.x, p.p2.y, p.p2.z}};
      Box b;
      for (auto& q : v) b.grow(q);
      // the EPS-fattened triangle of Triangle::hit (hits lie within EPS x (|e1| + |e2|)
      // of it), twice over; the float error of the solve is the per-ray margin's
      auto len = [](const float* a, const float* c) {
        const double x = a[0] - c[0], y = a[1] - c[1], z = a[2] - c[2];
        return std::sqrt(x * x + y * y + z * z);
      };
      const double m = kBoxGrow * (len(v[0], v[1]) + len(v[0], v[2])) + 1e-6 * (1.0 + std::max({std::fabs(b.lo[0]),
          std::fabs(b.lo[1]), std::fabs(b.lo[2]), std::fabs(b.hi[0]), std::fabs(b.hi[1]), std::fabs(b.hi[2])}));
      for (int k = 0; k < 3; ++k) {
        b.lo[k] = std::nextafter(static_cast<float>(b.lo[k] - m), -INFINITY);
        b.hi[k] = std::nextafter(static_cast<float>(b.hi[k] + m), INFINITY);
        cen[3 * i + k] = 0.5f * (b.lo[k] + b.hi[k]);
      }
      box[i] = b;
    }
  };
  // the KD membership data first (the triangle records carry their
  // prim_leaf range), beside the boxes in chunks of one thread each
  auto kd = std::async(std::launch::async, [&] { kd_paths(s, out); });
  const size_t chunk = 1 << 16;
  std::vector<std::future<void>> parts;
  for (size_t i0 = chunk; i0 < n; i0 += chunk)
    parts.push_back(std::async(std::launch::async, prep, i0, std::min(n, i0 + chunk)));
  prep(0, std::min(n, chunk));
  for (auto& f : parts) f.get();
  kd.get();
  out.ok = true;
  out.tris.reserve(n);
  out.nodes.reserve(2 * n / kMaxLeaf + 8);
  std::atomic<int> threads{0};
  Builder B{box, cen, idx, out, s, tri_prim, out.prim_leaf_off, threads};
  // node 0 is always inner (the traversal starts from its two children)
  const int nn = static_cast<int>(n);
  if (nn <= kMaxLeaf) {
    out.nodes.emplace_back();
    Box all = B.bounds(0, nn);
    const int l = B.leaf_link(0, nn);
    BNode& nd = out.nodes[0];
    for (int k = 0; k < 3; ++k) {
      nd.b[k] = all.lo[k];
      nd.b[3 + k] = all.hi[k];
      nd.b[6 + k] = 3e38f;  // a point far outside the scene: never hit (see Collapse)
      nd.b[9 + k] = 3e38f;
    }
    nd.c[0] = l;
    nd.c[1] = ~0;  // never reached: empty box
    nd.c[2] = nd.c[3] = 0;
    out.depth = 1;
  } else {
    const Box all = B.bounds(0, nn);
    int m = B.split(0, nn, all);
    if (m < 0) m = nn / 2;
    B.inner(0, nn, m, 1);
  }
  if (out.ok && (wide == 4 || with4)) {
    out.nodes4.reserve(out.nodes.size() / 2 + 4);
    Collapse{out}.node(0, 1);
  }
  if (out.ok && wide == 8) {
    out.nodes8.reserve(out.nodes.size() / 4 + 4);
    Collapse8{out}.node(0, 1);
  }
}

}  // namespace wrf
