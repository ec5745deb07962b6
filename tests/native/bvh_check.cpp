// Structural check of the verified-BVH data (wr_bvh.cpp) on a scene, CPU only:
// built and run by tests/test_bvh_host.py.  Prints "OK <stats>" or the first
// violated property and exits non-zero.
#include <algorithm>
#include <map>
#include <functional>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "wr_bvh.h"
#include "wr_scene.h"

// an empty child slot: a point box far outside every scene (wr_bvh.cpp) or an inverted box
static bool empty_slot(float lo0, float hi0) { return !(lo0 <= hi0) || (lo0 == 3e38f && hi0 == 3e38f); }

static int fail(const std::string& m) {
  std::printf("FAIL %s\n", m.c_str());
  return 1;
}

int main(int argc, char** argv) {
  if (argc < 2) return fail("usage: bvh_check scene");
  wr::Scene s;
  std::string err;
  if (!wr::load_scene(argv[1], s, err)) return fail("load: " + err);
  wrf::FastHost f;
  wrf::build_fast(s, f);
  if (!f.ok) return fail("build refused: " + f.why);
  const size_t np = s.prims.size();
  // 1. every triangle exactly once, records = Triangle::hit's A..F
  std::vector<int> seen(np, 0);
  for (const auto& r : f.tris) {
    int p;
    std::memcpy(&p, &r.c[1], 4);
    const bool sph = p < 0;  // a sphere's record: -(prim + 1)
    if (sph) p = -p - 1;
    if (p < 0 || static_cast<size_t>(p) >= np) return fail("bad prim id in a record");
    ++seen[static_cast<size_t>(p)];
    const wr::Prim& q = s.prims[static_cast<size_t>(p)];
    if (sph != (q.type != wr::kTri)) return fail("record type differs from the primitive's");
    if (sph) {
      const float want[4] = {q.c.x, q.c.y, q.c.z, q.r};
      if (std::memcmp(want, r.a, sizeof want) != 0) return fail("record differs from the sphere");
    } else {
      const float want[10] = {q.p0.x, q.p0.y, q.p0.z, q.p0.x - q.p1.x, q.p0.y - q.p1.y, q.p0.z - q.p1.z,
                              q.p0.x - q.p2.x, q.p0.y - q.p2.y, q.p0.z - q.p2.z};
      const float got[9] = {r.a[0], r.a[1], r.a[2], r.a[3], r.b[0], r.b[1], r.b[2], r.b[3], r.c[0]};
      if (std::memcmp(want, got, sizeof got) != 0) return fail("record differs from the triangle");
    }
    int lb, ln;
    std::memcpy(&lb, &r.c[2], 4);
    std::memcpy(&ln, &r.c[3], 4);
    if (lb != f.prim_leaf_off[static_cast<size_t>(p)] || ln != f.prim_leaf_off[static_cast<size_t>(p) + 1] - lb)
      return fail("record leaf range");
  }
  for (size_t p = 0; p < np; ++p)
    if (seen[p] != 1) return fail("triangle " + std::to_string(p) + " appears " + std::to_string(seen[p]) + " times");
  // 2. child boxes contain their subtree's triangles (vertices)
  size_t leaves = 0, leaf_hist[9] = {};
  int maxdepth = 0;
  struct It {
    int link, depth;
    float lo[3], hi[3];
  };
  std::vector<It> st;
  for (int c = 0; c < 2; ++c) {
    const wrf::BNode& n = f.nodes[0];
    It it{n.c[c], 1, {n.b[6 * c], n.b[6 * c + 1], n.b[6 * c + 2]}, {n.b[6 * c + 3], n.b[6 * c + 4], n.b[6 * c + 5]}};
    if (!empty_slot(it.lo[0], it.hi[0])) st.push_back(it);
  }
  while (!st.empty()) {
    const It it = st.back();
    st.pop_back();
    maxdepth = std::max(maxdepth, it.depth);
    if (it.link >= 0) {
      const wrf::BNode& n = f.nodes[static_cast<size_t>(it.link)];
      for (int c = 0; c < 2; ++c) {
        It ch{n.c[c], it.depth + 1, {n.b[6 * c], n.b[6 * c + 1], n.b[6 * c + 2]},
              {n.b[6 * c + 3], n.b[6 * c + 4], n.b[6 * c + 5]}};
        for (int a = 0; a < 3; ++a)
          if (ch.lo[a] < it.lo[a] || ch.hi[a] > it.hi[a]) return fail("child box outside its parent's");
        st.push_back(ch);
      }
    } else {
      ++leaves;
      const int l = ~it.link, first = l >> 3, cnt = (l & 7) + 1;
      ++leaf_hist[cnt];
      if (cnt > wrf::kMaxLeaf) return fail("leaf too large");
      for (int j = 0; j < cnt; ++j) {
        int p;
        std::memcpy(&p, &f.tris[static_cast<size_t>(first + j)].c[1], 4);
        if (p < 0) {  // a sphere: its reference box and centre +- r inside the leaf box
          const wr::Prim& q = s.prims[static_cast<size_t>(-p - 1)];
          const float c[3] = {q.c.x, q.c.y, q.c.z}, bl[3] = {q.bl.x, q.bl.y, q.bl.z}, br[3] = {q.br.x, q.br.y, q.br.z};
          for (int a = 0; a < 3; ++a)
            if (bl[a] < it.lo[a] || br[a] > it.hi[a] || c[a] - q.r < it.lo[a] || c[a] + q.r > it.hi[a])
              return fail("sphere outside its leaf box");
          continue;
        }
        const wr::Prim& q = s.prims[static_cast<size_t>(p)];
        const float v[3][3] = {{q.p0.x, q.p0.y, q.p0.z}, {q.p1.x, q.p1.y, q.p1.z}, {q.p2.x, q.p2.y, q.p2.z}};
        for (auto& w : v)
          for (int a = 0; a < 3; ++a)
            if (w[a] < it.lo[a] || w[a] > it.hi[a]) return fail("triangle outside its leaf box");
      }
    }
  }
  if (leaves != static_cast<size_t>(f.leaves)) return fail("leaf count");
  if (maxdepth > f.depth + 1) return fail("depth bound");
  // 2b. the 4-wide tree: the same leaves with the same boxes (bit for bit),
  //     each once, inner boxes holding their children's, depth within depth4
  //     (built with -DWR_BVH_WIDE=4 only)
  if (!f.nodes4.empty()) {
    std::vector<std::pair<int, std::vector<float>>> want, got;
    std::vector<It> s2;
    for (int c = 0; c < 2; ++c) {
      const wrf::BNode& n = f.nodes[0];
      s2.push_back(It{n.c[c], 1, {n.b[6 * c], n.b[6 * c + 1], n.b[6 * c + 2]}, {n.b[6 * c + 3], n.b[6 * c + 4], n.b[6 * c + 5]}});
    }
    while (!s2.empty()) {
      const It it = s2.back();
      s2.pop_back();
      if (empty_slot(it.lo[0], it.hi[0])) continue;
      if (it.link >= 0) {
        const wrf::BNode& n = f.nodes[static_cast<size_t>(it.link)];
        for (int c = 0; c < 2; ++c)
          s2.push_back(It{n.c[c], 0, {n.b[6 * c], n.b[6 * c + 1], n.b[6 * c + 2]}, {n.b[6 * c + 3], n.b[6 * c + 4], n.b[6 * c + 5]}});
      } else {
        want.push_back({it.link, {it.lo[0], it.lo[1], it.lo[2], it.hi[0], it.hi[1], it.hi[2]}});
      }
    }
    struct It4 {
      int node, depth;
      float lo[3], hi[3];
    };
    std::vector<It4> s4{{0, 1, {-INFINITY, -INFINITY, -INFINITY}, {INFINITY, INFINITY, INFINITY}}};
    int maxd4 = 0;
    size_t visits = 0;
    while (!s4.empty()) {
      const It4 it = s4.back();
      s4.pop_back();
      if (++visits > f.nodes4.size()) return fail("4-wide tree has a cycle");
      maxd4 = std::max(maxd4, it.depth);
      const auto& n = f.nodes4[static_cast<size_t>(it.node)];
      for (int k = 0; k < 4; ++k) {
#if WR_BVH4_QUANT
        // BNode4Q: the decoded box fmaf(q, scale, org) of the slot (unused
        // slots: kEmptyLink); containment of the binary boxes is checked below
        if (n.c[k] == wrf::kEmptyLink) continue;
        float lo[3], hi[3];
        for (int a = 0; a < 3; ++a) {
          if (!(n.scale[a] > 0.f)) return fail("4-wide quantised scale");
          lo[a] = std::fma(static_cast<float>(n.qlo[a][k]), n.scale[a], n.org[a]);
          hi[a] = std::fma(static_cast<float>(n.qhi[a][k]), n.scale[a], n.org[a]);
          if (lo[a] > hi[a]) return fail("4-wide decoded box inverted");
        }
#else
        const float lo[3] = {n.lo[0][k], n.lo[1][k], n.lo[2][k]}, hi[3] = {n.hi[0][k], n.hi[1][k], n.hi[2][k]};
        if (empty_slot(lo[0], hi[0])) continue;
        for (int a = 0; a < 3; ++a)
          if (lo[a] < it.lo[a] || hi[a] > it.hi[a]) return fail("4-wide child box outside its parent's");
#endif
        if (n.c[k] >= 0) {
          if (static_cast<size_t>(n.c[k]) >= f.nodes4.size()) return fail("4-wide link out of range");
          s4.push_back(It4{n.c[k], it.depth + 1, {lo[0], lo[1], lo[2]}, {hi[0], hi[1], hi[2]}});
        } else {
          got.push_back({n.c[k], {lo[0], lo[1], lo[2], hi[0], hi[1], hi[2]}});
        }
      }
    }
    if (maxd4 > f.depth4) return fail("4-wide depth bound");
    std::sort(want.begin(), want.end());
    std::sort(got.begin(), got.end());
    if (want.size() != got.size()) return fail("4-wide tree leaf count");
#if WR_BVH4_QUANT
    // the same leaves, each decoded leaf box CONTAINING the binary one; each
    // decoded inner box containing every binary leaf box beneath it
    for (size_t i = 0; i < want.size(); ++i) {
      if (want[i].first != got[i].first) return fail("4-wide tree leaves differ from the binary tree's");
      for (int a = 0; a < 3; ++a)
        if (got[i].second[a] > want[i].second[a] || got[i].second[3 + a] < want[i].second[3 + a])
          return fail("4-wide decoded leaf box does not contain the binary box");
    }
    {
      std::map<int, std::vector<float>> leaf_box(want.begin(), want.end());
      // union of the binary leaf boxes under a 4-wide node, checked against the
      // decoded box of every inner slot on the way
      std::function<bool(int, float*)> sub = [&](int node, float* u) -> bool {
        for (int a = 0; a < 3; ++a) {
          u[a] = INFINITY;
          u[3 + a] = -INFINITY;
        }
        const auto& n = f.nodes4[static_cast<size_t>(node)];
        for (int k = 0; k < 4; ++k) {
          if (n.c[k] == wrf::kEmptyLink) continue;
          float b[6];
          if (n.c[k] >= 0) {
            if (!sub(n.c[k], b)) return false;
            for (int a = 0; a < 3; ++a) {
              const float lo = std::fma(static_cast<float>(n.qlo[a][k]), n.scale[a], n.org[a]);
              const float hi = std::fma(static_cast<float>(n.qhi[a][k]), n.scale[a], n.org[a]);
              if (lo > b[a] || hi < b[3 + a]) return false;
            }
          } else {
            const std::vector<float>& lb = leaf_box[n.c[k]];
            for (int a = 0; a < 6; ++a) b[a] = lb[static_cast<size_t>(a)];
          }
          for (int a = 0; a < 3; ++a) {
            u[a] = std::min(u[a], b[a]);
            u[3 + a] = std::max(u[3 + a], b[3 + a]);
          }
        }
        return true;
      };
      float u[6];
      if (!sub(0, u)) return fail("4-wide decoded inner box does not contain its subtree's leaf boxes");
    }
#else
    for (size_t i = 0; i < want.size(); ++i)
      if (want[i].first != got[i].first || std::memcmp(want[i].second.data(), got[i].second.data(), 24) != 0)
        return fail("4-wide tree leaves differ from the binary tree's");
#endif
  }
  // 2c. the 8-wide tree (built with -DWR_BVH_WIDE=8 only): the same leaves,
  //     each once, every decoded child box fmaf(q, scale, org) CONTAINING the
  //     binary tree's box of that child (the search's boxes only grow), inner
  //     nodes' boxes holding their children's decoded boxes, depth <= depth8
  if (!f.nodes8.empty()) {
    std::vector<std::pair<int, std::vector<float>>> want, got;
    std::vector<It> s2;
    for (int c = 0; c < 2; ++c) {
      const wrf::BNode& n = f.nodes[0];
      s2.push_back(It{n.c[c], 1, {n.b[6 * c], n.b[6 * c + 1], n.b[6 * c + 2]}, {n.b[6 * c + 3], n.b[6 * c + 4], n.b[6 * c + 5]}});
    }
    while (!s2.empty()) {
      const It it = s2.back();
      s2.pop_back();
      if (empty_slot(it.lo[0], it.hi[0])) continue;
      if (it.link >= 0) {
        const wrf::BNode& n = f.nodes[static_cast<size_t>(it.link)];
        for (int c = 0; c < 2; ++c)
          s2.push_back(It{n.c[c], 0, {n.b[6 * c], n.b[6 * c + 1], n.b[6 * c + 2]}, {n.b[6 * c + 3], n.b[6 * c + 4], n.b[6 * c + 5]}});
      } else {
        want.push_back({it.link, {it.lo[0], it.lo[1], it.lo[2], it.hi[0], it.hi[1], it.hi[2]}});
      }
    }
    // every binary inner node's box by link, to check the decoded inner boxes too
    std::vector<std::vector<float>> bin_box(f.nodes.size());
    for (size_t i = 0; i < f.nodes.size(); ++i)
      for (int c = 0; c < 2; ++c)
        if (f.nodes[i].c[c] >= 0)
          bin_box[static_cast<size_t>(f.nodes[i].c[c])] = {f.nodes[i].b[6 * c], f.nodes[i].b[6 * c + 1], f.nodes[i].b[6 * c + 2],
                                                           f.nodes[i].b[6 * c + 3], f.nodes[i].b[6 * c + 4], f.nodes[i].b[6 * c + 5]};
    struct It8 {
      int node, depth;
      float lo[3], hi[3];
    };
    std::vector<It8> s8{{0, 1, {-INFINITY, -INFINITY, -INFINITY}, {INFINITY, INFINITY, INFINITY}}};
    int maxd8 = 0;
    size_t visits = 0;
    std::vector<std::pair<int, std::vector<float>>> leaf_dec;  // leaf link -> decoded box
    bool bad_inner = false;
    while (!s8.empty()) {
      const It8 it = s8.back();
      s8.pop_back();
      if (++visits > f.nodes8.size()) return fail("8-wide tree has a cycle");
      maxd8 = std::max(maxd8, it.depth);
      const wrf::BNode8& n = f.nodes8[static_cast<size_t>(it.node)];
      if (n.n < 1 || n.n > 8) return fail("8-wide child count");
      for (int k = 0; k < n.n; ++k) {
        float lo[3], hi[3];
        for (int a = 0; a < 3; ++a) {
          if (!(n.scale[a] > 0.f)) return fail("8-wide scale");
          lo[a] = std::fma(static_cast<float>(n.qlo[a][k]), n.scale[a], n.org[a]);
          hi[a] = std::fma(static_cast<float>(n.qhi[a][k]), n.scale[a], n.org[a]);
          if (lo[a] > hi[a]) return fail("8-wide decoded box inverted");
        }
        (void)it;
        if (n.c[k] >= 0) {
          if (static_cast<size_t>(n.c[k]) >= f.nodes8.size()) return fail("8-wide link out of range");
          s8.push_back(It8{n.c[k], it.depth + 1, {lo[0], lo[1], lo[2]}, {hi[0], hi[1], hi[2]}});
        } else {
          got.push_back({n.c[k], {}});
          leaf_dec.push_back({n.c[k], {lo[0], lo[1], lo[2], hi[0], hi[1], hi[2]}});
        }
      }
    }
    if (maxd8 > f.depth8) return fail("8-wide depth bound");
    std::sort(want.begin(), want.end());
    std::sort(leaf_dec.begin(), leaf_dec.end());
    if (want.size() != leaf_dec.size()) return fail("8-wide tree leaf count");
    for (size_t i = 0; i < want.size(); ++i) {
      if (want[i].first != leaf_dec[i].first) return fail("8-wide tree leaves differ from the binary tree's");
      for (int a = 0; a < 3; ++a)
        if (leaf_dec[i].second[a] > want[i].second[a] || leaf_dec[i].second[3 + a] < want[i].second[3 + a])
          return fail("8-wide decoded leaf box does not contain the binary box");
    }
    // inner children: each decoded box contains every binary leaf box beneath
    // it (the union of its subtree's geometry); decoded boxes need not nest
    std::map<int, std::vector<float>> leaf_box(want.begin(), want.end());
    std::vector<std::array<float, 6>> sub(f.nodes8.size());
    std::vector<char> done(f.nodes8.size(), 0);
    std::function<std::array<float, 6>(int)> uni = [&](int nd) -> std::array<float, 6> {
      if (done[static_cast<size_t>(nd)]) return sub[static_cast<size_t>(nd)];
      std::array<float, 6> u{INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
      const wrf::BNode8& n = f.nodes8[static_cast<size_t>(nd)];
      for (int k = 0; k < n.n; ++k) {
        std::array<float, 6> c;
        if (n.c[k] >= 0) {
          c = uni(n.c[k]);
        } else {
          const std::vector<float>& b = leaf_box[n.c[k]];
          for (int a = 0; a < 6; ++a) c[static_cast<size_t>(a)] = b[static_cast<size_t>(a)];
        }
        for (int a = 0; a < 3; ++a) {
          const float lo = std::fma(static_cast<float>(n.qlo[a][k]), n.scale[a], n.org[a]);
          const float hi = std::fma(static_cast<float>(n.qhi[a][k]), n.scale[a], n.org[a]);
          if (lo > c[static_cast<size_t>(a)] || hi < c[static_cast<size_t>(3 + a)]) bad_inner = true;
          u[static_cast<size_t>(a)] = std::min(u[static_cast<size_t>(a)], c[static_cast<size_t>(a)]);
          u[static_cast<size_t>(3 + a)] = std::max(u[static_cast<size_t>(3 + a)], c[static_cast<size_t>(3 + a)]);
        }
      }
      done[static_cast<size_t>(nd)] = 1;
      return sub[static_cast<size_t>(nd)] = u;
    };
    uni(0);
    if (bad_inner) return fail("8-wide decoded box does not contain its subtree's leaf boxes");
    (void)bin_box;
  }
  // 3. KD membership: each primitive's leaves (ascending), its position in
  //    each, and the leaf paths lead from the root to that leaf
  std::vector<std::vector<std::pair<int, int>>> per(np);
  for (size_t i = 0; i < s.nodes.size(); ++i) {
    const wr::KdNode& k = s.nodes[i];
    if (k.axis >= 0) {
      if (f.node_path[i] != -1) return fail("inner node mapped to a path");
      continue;
    }
    const int off = f.node_path[i];
    if (off < 0 || (off & 1)) return fail("leaf without an aligned path record");
    const uint32_t* rec = f.path.data() + 2 * static_cast<size_t>(off);
    const uint32_t n = rec[0];
    size_t node = 0;  // follow the entries from the root, cutting the root box
    float lo[3] = {s.root_l.x, s.root_l.y, s.root_l.z}, hi[3] = {s.root_r.x, s.root_r.y, s.root_r.z};
    for (uint32_t e = 0; e < n; ++e) {
      const uint32_t bits = rec[2 * (4 + e)], w = rec[2 * (4 + e) + 1];
      const wr::KdNode& a = s.nodes[node];
      uint32_t sb;
      std::memcpy(&sb, &a.split, 4);
      if (a.axis < 0 || sb != bits || static_cast<uint32_t>(a.axis) != (w & 3u)) return fail("path entry mismatch");
      if (w & 4u) lo[a.axis] = std::max(lo[a.axis], a.split);
      else hi[a.axis] = std::min(hi[a.axis], a.split);
      node = (w & 4u) ? static_cast<size_t>(a.right) : node + 1;
    }
    if (node != i) return fail("path does not lead to its leaf");
    // the record's cell (the membership witnesses' box) is the leaf's region
    const float want_cell[6] = {lo[0], lo[1], lo[2], hi[0], hi[1], hi[2]};
    if (std::memcmp(want_cell, rec + 2, sizeof want_cell) != 0) return fail("leaf cell differs from its region");
    for (int j = 0; j < k.count; ++j) per[static_cast<size_t>(s.refs[static_cast<size_t>(k.first + j)])].emplace_back(off, j);
  }
  for (size_t p = 0; p < np; ++p) {
    const int lb = f.prim_leaf_off[p], le = f.prim_leaf_off[p + 1];
    if (static_cast<size_t>(le - lb) != per[p].size()) return fail("leaf list length of prim " + std::to_string(p));
    for (int k = lb; k < le; ++k) {
      if (f.prim_leaf[static_cast<size_t>(k)] != per[p][static_cast<size_t>(k - lb)].first ||
          f.prim_leaf_pos[static_cast<size_t>(k)] != per[p][static_cast<size_t>(k - lb)].second)
        return fail("leaf list of prim " + std::to_string(p));
      if (k > lb && f.prim_leaf[static_cast<size_t>(k)] <= f.prim_leaf[static_cast<size_t>(k - 1)])
        return fail("leaf list not ascending");
    }
    // the primitive's record: leaf count, first four leaves' offsets and cells
    const wrf::PrimRec& r = f.prim_rec[p];
    if (r.ln != le - lb) return fail("record leaf count of prim " + std::to_string(p));
    for (int k = 0; k < 4; ++k) {
      const int off = k < r.ln ? f.prim_leaf[static_cast<size_t>(lb + k)] : -1;
      if (r.off[k] != off) return fail("record offsets of prim " + std::to_string(p));
      float want_cell[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
      if (off >= 0) std::memcpy(want_cell, f.path.data() + 2 * static_cast<size_t>(off) + 2, sizeof want_cell);
      if (std::memcmp(want_cell, r.cell[k], sizeof want_cell) != 0) return fail("record cells of prim " + std::to_string(p));
    }
  }
  std::printf("OK prims %zu nodes %zu leaves %zu depth %d refs %zu leaf sizes", np, f.nodes.size(), leaves, f.depth,
              f.prim_leaf.size());
  for (int k = 1; k <= wrf::kMaxLeaf; ++k) std::printf(" %d:%zu", k, leaf_hist[k]);
  // KD leaves per primitive (the membership / tie resolution's list lengths)
  size_t big16 = 0, big256 = 0;
  int maxln = 0;
  for (size_t p = 0; p < np; ++p) {
    const int ln = f.prim_leaf_off[p + 1] - f.prim_leaf_off[p];
    maxln = std::max(maxln, ln);
    big16 += ln > 16;
    big256 += ln > 256;
  }
  std::printf(" kd leaves per prim: max %d, >16: %zu, >256: %zu", maxln, big16, big256);
  // content hash (FNV-1a) of everything the device reads: equal builds, equal data
  uint64_t h = 1469598103934665603ull;
  auto mix = [&h](const void* data, size_t n) {
    const unsigned char* c = static_cast<const unsigned char*>(data);
    for (size_t i = 0; i < n; ++i) h = (h ^ c[i]) * 1099511628211ull;
  };
  mix(f.nodes.data(), f.nodes.size() * sizeof(f.nodes[0]));
  mix(f.tris.data(), f.tris.size() * sizeof(f.tris[0]));
  mix(f.prim_leaf_off.data(), f.prim_leaf_off.size() * 4);
  mix(f.prim_leaf.data(), f.prim_leaf.size() * 4);
  mix(f.prim_leaf_pos.data(), f.prim_leaf_pos.size() * 4);
  mix(f.prim_rec.data(), f.prim_rec.size() * sizeof(f.prim_rec[0]));
  mix(f.path.data(), f.path.size() * 4);
  mix(f.node_path.data(), f.node_path.size() * 4);
  mix(f.node_cell.data(), f.node_cell.size() * 4);
  std::printf(" hash %016llx\n", static_cast<unsigned long long>(h));
  return 0;
}
