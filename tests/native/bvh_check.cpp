// Structural check of the verified-BVH data (wr_bvh.cpp) on a scene, CPU only:
// built and run by tests/test_bvh_host.py.  Prints "OK <stats>" or the first
// violated property and exits non-zero.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "wr_bvh.h"
#include "wr_scene.h"

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
    if (p < 0 || static_cast<size_t>(p) >= np) return fail("bad prim id in a record");
    ++seen[static_cast<size_t>(p)];
    const wr::Prim& q = s.prims[static_cast<size_t>(p)];
    const float want[10] = {q.p0.x, q.p0.y, q.p0.z, q.p0.x - q.p1.x, q.p0.y - q.p1.y, q.p0.z - q.p1.z,
                            q.p0.x - q.p2.x, q.p0.y - q.p2.y, q.p0.z - q.p2.z};
    const float got[9] = {r.a[0], r.a[1], r.a[2], r.a[3], r.b[0], r.b[1], r.b[2], r.b[3], r.c[0]};
    if (std::memcmp(want, got, sizeof got) != 0) return fail("record differs from the triangle");
    int lb, ln;
    std::memcpy(&lb, &r.c[2], 4);
    std::memcpy(&ln, &r.c[3], 4);
    if (lb != f.prim_leaf_off[static_cast<size_t>(p)] || ln != f.prim_leaf_off[static_cast<size_t>(p) + 1] - lb)
      return fail("record leaf range");
  }
  for (size_t p = 0; p < np; ++p)
    if (seen[p] != 1) return fail("triangle " + std::to_string(p) + " appears " + std::to_string(seen[p]) + " times");
  // 2. child boxes contain their subtree's triangles (vertices)
  size_t leaves = 0;
  int maxdepth = 0;
  struct It {
    int link, depth;
    float lo[3], hi[3];
  };
  std::vector<It> st;
  for (int c = 0; c < 2; ++c) {
    const wrf::BNode& n = f.nodes[0];
    It it{n.c[c], 1, {n.b[6 * c], n.b[6 * c + 1], n.b[6 * c + 2]}, {n.b[6 * c + 3], n.b[6 * c + 4], n.b[6 * c + 5]}};
    if (it.lo[0] <= it.hi[0]) st.push_back(it);
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
      if (cnt > wrf::kMaxLeaf) return fail("leaf too large");
      for (int j = 0; j < cnt; ++j) {
        int p;
        std::memcpy(&p, &f.tris[static_cast<size_t>(first + j)].c[1], 4);
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
    size_t node = 0;  // follow the entries from the root
    for (uint32_t e = 0; e < n; ++e) {
      const uint32_t bits = rec[2 * (4 + e)], w = rec[2 * (4 + e) + 1];
      const wr::KdNode& a = s.nodes[node];
      uint32_t sb;
      std::memcpy(&sb, &a.split, 4);
      if (a.axis < 0 || sb != bits || static_cast<uint32_t>(a.axis) != (w & 3u)) return fail("path entry mismatch");
      node = (w & 4u) ? static_cast<size_t>(a.right) : node + 1;
    }
    if (node != i) return fail("path does not lead to its leaf");
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
  }
  std::printf("OK prims %zu nodes %zu leaves %zu depth %d refs %zu\n", np, f.nodes.size(), leaves, f.depth,
              f.prim_leaf.size());
  return 0;
}
