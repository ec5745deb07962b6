// CPU estimate of the BVH search's work per ray (node visits, triangle tests)
// for a scene, used to compare build variants (WR_BVH_BINS / WR_BVH_SWEEP /
// WR_BVH_CT) before spending GPU time.  The walk mirrors k_trace_fast's
// (wr_fast.h trace_fast): ordered descent, nearer child first, window t1 + 2 EPS,
// popped entries kept when their entry t is inside the window; no per-ray
// margins (relative comparisons only).
// Rays: camera rays through random film points (the scene's camera), and
// secondary rays from random surface points in cosine directions about either
// side's normal (the BDPT mix is ~1/4 primaries, ~3/4 bounces).
// Build: g++ -O2 -std=c++17 -I winmad-s-raytracer-v1.0_amd/csrc -I include
//   scripts/bvh_cost.cpp winmad-s-raytracer-v1.0_amd/csrc/{wr_scene,wr_bvh}.cpp -lpthread
// Usage: bvh_cost scene [rays]
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "wr_bvh.h"
#include "wr_scene.h"

namespace {
constexpr float kEps = 1e-3f;

struct V {
  float x, y, z;
};
V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V add(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
V mul(V a, float s) { return {a.x * s, a.y * s, a.z * s}; }
float dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
V cross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
V norm(V a) { return mul(a, 1.f / std::sqrt(dot(a, a))); }
V f3(wr::F3 p) { return {p.x, p.y, p.z}; }

bool tri(const wrf::TriRec& r, V o, V d, float& t) {
  const V p0{r.a[0], r.a[1], r.a[2]};
  const V e1{-r.a[3], -r.b[0], -r.b[1]}, e2{-r.b[2], -r.b[3], -r.c[0]};
  const V pv = cross(d, e2);
  const float det = dot(e1, pv);
  if (std::fabs(det) < 1e-12f) return false;
  const float inv = 1.f / det;
  const V tv = sub(o, p0);
  const float u = dot(tv, pv) * inv;
  if (u < -kEps || u > 1.f) return false;
  const V qv = cross(tv, e1);
  const float v = dot(d, qv) * inv;
  if (v < -kEps || u + v > 1.f) return false;
  t = dot(e2, qv) * inv;
  return t > kEps;
}

struct Cost {
  double nodes = 0, tests = 0;
};

void walk(const wrf::FastHost& F, V o, V d, Cost& c) {
  const V inv{1.f / d.x, 1.f / d.y, 1.f / d.z};
  float t1 = INFINITY;
  struct E {
    int link;
    float t;
  } st[128];
  int sp = 0, cur = 0;
  auto hi = [&]() { return t1 + 2.f * kEps; };
  auto slab = [&](const float* b, float& tn) {
    const float x0 = (b[0] - o.x) * inv.x, x1 = (b[3] - o.x) * inv.x;
    const float y0 = (b[1] - o.y) * inv.y, y1 = (b[4] - o.y) * inv.y;
    const float z0 = (b[2] - o.z) * inv.z, z1 = (b[5] - o.z) * inv.z;
    tn = std::fmax(std::fmax(std::fmin(x0, x1), std::fmin(y0, y1)), std::fmax(std::fmin(z0, z1), 0.f));
    const float tf = std::fmin(std::fmin(std::fmax(x0, x1), std::fmax(y0, y1)), std::fmin(std::fmax(z0, z1), hi()));
    return tn <= tf;
  };
  for (;;) {
    if (cur >= 0) {
      c.nodes += 1;
      const wrf::BNode& n = F.nodes[static_cast<size_t>(cur)];
      float ta, tb;
      const bool ha = slab(n.b, ta), hb = slab(n.b + 6, tb);
      if (ha && hb) {
        const bool af = ta <= tb;
        st[sp++] = {af ? n.c[1] : n.c[0], af ? tb : ta};
        cur = af ? n.c[0] : n.c[1];
        continue;
      }
      if (ha || hb) {
        cur = ha ? n.c[0] : n.c[1];
        continue;
      }
    } else {
      const int l = ~cur, first = l >> 3, cnt = (l & 7) + 1;
      for (int j = 0; j < cnt; ++j) {
        c.tests += 1;
        float t;
        if (tri(F.tris[static_cast<size_t>(first + j)], o, d, t) && t < t1) t1 = t;
      }
    }
    cur = 0x7fffffff;
    while (sp > 0) {
      --sp;
      if (st[sp].t <= hi()) {
        cur = st[sp].link;
        break;
      }
    }
    if (cur == 0x7fffffff) return;
  }
}
// W-wide trees collapsed from the binary one (as wr_bvh.cpp's Collapse does
// for W = 4: open the inner child of largest area until W children), walked
// the same way: children hit sorted by entry t, nearest next, the rest pushed
struct Wide {
  struct Node {
    float b[8][6];
    int c[8];
    int n;
  };
  std::vector<Node> nodes;
  int W;
  const wrf::FastHost& F;
  Wide(const wrf::FastHost& f, int w) : W(w), F(f) { build(0); }
  static double area(const float* b) {
    if (!(b[0] <= b[3])) return 0.0;
    const double x = b[3] - b[0], y = b[4] - b[1], z = b[5] - b[2];
    return 2.0 * (x * y + x * z + y * z);
  }
  int build(int n2) {
    struct K {
      float b[6];
      int link;
    };
    std::vector<K> ks;
    auto kid = [&](int n, int side) {
      K k;
      std::memcpy(k.b, F.nodes[static_cast<size_t>(n)].b + 6 * side, sizeof k.b);
      k.link = F.nodes[static_cast<size_t>(n)].c[side];
      return k;
    };
    ks.push_back(kid(n2, 0));
    ks.push_back(kid(n2, 1));
    while (static_cast<int>(ks.size()) < W) {
      int best = -1;
      double ba = -1;
      for (size_t i = 0; i < ks.size(); ++i)
        if (ks[i].link >= 0 && area(ks[i].b) > ba) {
          ba = area(ks[i].b);
          best = static_cast<int>(i);
        }
      if (best < 0) break;
      const int open = ks[static_cast<size_t>(best)].link;
      ks[static_cast<size_t>(best)] = kid(open, 0);
      ks.push_back(kid(open, 1));
    }
    const int at = static_cast<int>(nodes.size());
    nodes.emplace_back();
    std::vector<int> links;
    for (const K& k : ks) links.push_back(k.link >= 0 ? build(k.link) : k.link);
    Node& d = nodes[static_cast<size_t>(at)];
    d.n = static_cast<int>(ks.size());
    for (int i = 0; i < d.n; ++i) {
      std::memcpy(d.b[i], ks[static_cast<size_t>(i)].b, sizeof d.b[i]);
      d.c[i] = links[static_cast<size_t>(i)];
    }
    return at;
  }
  mutable std::vector<long> sp_hist = std::vector<long>(64, 0);  // rays by their deepest stack
  void walk(V o, V d, Cost& c, double& leaves) const {
    int spmax = 0;
    struct Rec {
      std::vector<long>& h;
      int& m;
      ~Rec() { ++h[static_cast<size_t>(std::min(m, 63))]; }
    } rec{sp_hist, spmax};
    const V inv{1.f / d.x, 1.f / d.y, 1.f / d.z};
    float t1 = INFINITY;
    struct E {
      int link;
      float t;
    } st[512];
    int sp = 0, cur = 0;
    auto hi = [&]() { return t1 + 2.f * kEps; };
    auto slab = [&](const float* b, float& tn) {
      const float x0 = (b[0] - o.x) * inv.x, x1 = (b[3] - o.x) * inv.x;
      const float y0 = (b[1] - o.y) * inv.y, y1 = (b[4] - o.y) * inv.y;
      const float z0 = (b[2] - o.z) * inv.z, z1 = (b[5] - o.z) * inv.z;
      tn = std::fmax(std::fmax(std::fmin(x0, x1), std::fmin(y0, y1)), std::fmax(std::fmin(z0, z1), 0.f));
      const float tf = std::fmin(std::fmin(std::fmax(x0, x1), std::fmax(y0, y1)), std::fmin(std::fmax(z0, z1), hi()));
      return tn <= tf;
    };
    for (;;) {
      if (cur >= 0) {
        c.nodes += 1;
        const Node& n = nodes[static_cast<size_t>(cur)];
        E hit[8];
        int nh = 0;
        for (int i = 0; i < n.n; ++i) {
          float t;
          if (slab(n.b[i], t)) hit[nh++] = {n.c[i], t};
        }
        std::sort(hit, hit + nh, [](const E& a, const E& b) { return a.t < b.t; });
        if (nh > 0) {
          for (int i = nh - 1; i >= 1; --i) st[sp++] = hit[i];
          spmax = std::max(spmax, sp);
          cur = hit[0].link;
          continue;
        }
      } else {
        leaves += 1;
        const int l = ~cur, first = l >> 3, cnt = (l & 7) + 1;
        for (int j = 0; j < cnt; ++j) {
          c.tests += 1;
          float t;
          if (tri(F.tris[static_cast<size_t>(first + j)], o, d, t) && t < t1) t1 = t;
        }
      }
      cur = 0x7fffffff;
      while (sp > 0) {
        --sp;
        if (st[sp].t <= hi()) {
          cur = st[sp].link;
          break;
        }
      }
      if (cur == 0x7fffffff) return;
    }
  }
};
}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: bvh_cost scene [rays]\n");
    return 2;
  }
  const int nrays = argc > 2 ? std::atoi(argv[2]) : 200000;
  wr::Scene s;
  std::string err;
  if (!wr::load_scene(argv[1], s, err)) {
    std::fprintf(stderr, "load: %s\n", err.c_str());
    return 1;
  }
  wrf::FastHost F;
  wrf::build_fast(s, F);
  if (!F.ok) {
    std::fprintf(stderr, "build refused: %s\n", F.why.c_str());
    return 1;
  }
  // SAH cost of the tree (ct 1 per node, 1 per triangle), relative to the root box
  double sah = 0;
  {
    const wrf::BNode& r = F.nodes[0];
    auto area = [](const float* b) {
      if (!(b[0] <= b[3])) return 0.0;
      const double x = b[3] - b[0], y = b[4] - b[1], z = b[5] - b[2];
      return 2.0 * (x * y + x * z + y * z);
    };
    float rb[6];
    for (int k = 0; k < 3; ++k) {
      rb[k] = std::fmin(r.b[k], r.b[6 + k]);
      rb[3 + k] = std::fmax(r.b[3 + k], r.b[9 + k]);
    }
    const double ra = area(rb);
    for (const auto& n : F.nodes)
      for (int c = 0; c < 2; ++c) {
        const double a = area(n.b + 6 * c) / ra;
        sah += n.c[c] >= 0 ? a : a * (((~n.c[c]) & 7) + 1);
      }
  }
  std::mt19937 rng(12345);
  std::uniform_real_distribution<float> U(0.f, 1.f);
  // area-weighted triangle pick
  std::vector<double> cdf(s.prims.size());
  double acc = 0;
  for (size_t i = 0; i < s.prims.size(); ++i) {
    const auto& p = s.prims[i];
    acc += 0.5 * std::sqrt(dot(cross(sub(f3(p.p1), f3(p.p0)), sub(f3(p.p2), f3(p.p0))),
                               cross(sub(f3(p.p1), f3(p.p0)), sub(f3(p.p2), f3(p.p0)))));
    cdf[i] = acc;
  }
  Cost cam, sec;
  std::vector<Wide> wides;
  for (int w : {4, 8}) wides.emplace_back(F, w);
  std::vector<Cost> wcam(wides.size()), wsec(wides.size());
  std::vector<double> wlv(wides.size(), 0.0);
  const V cpos = f3(s.cam.pos), cfwd = norm(f3(s.cam.fwd)), cup = norm(f3(s.cam.up));
  const V cright = norm(cross(cfwd, cup));
  const float th = std::tan(s.cam.fov * 0.5f * 3.14159265f / 180.f);
  for (int i = 0; i < nrays; ++i) {
    // camera ray: a random point of the image plane (same FOV scale on both axes)
    const float a = (2.f * U(rng) - 1.f) * th, b = (2.f * U(rng) - 1.f) * th * s.cam.yres / s.cam.xres;
    const V cd = norm(add(cfwd, add(mul(cright, a), mul(cup, b))));
    walk(F, cpos, cd, cam);
    for (size_t w = 0; w < wides.size(); ++w) wides[w].walk(cpos, cd, wcam[w], wlv[w]);
    // secondary ray: random surface point, cosine direction about a random side's normal
    const double x = U(rng) * acc;
    const size_t k = static_cast<size_t>(std::lower_bound(cdf.begin(), cdf.end(), x) - cdf.begin());
    const auto& p = s.prims[std::min(k, s.prims.size() - 1)];
    float u = U(rng), v = U(rng);
    if (u + v > 1.f) {
      u = 1.f - u;
      v = 1.f - v;
    }
    const V e1 = sub(f3(p.p1), f3(p.p0)), e2 = sub(f3(p.p2), f3(p.p0));
    V n = norm(cross(e1, e2));
    if (U(rng) < 0.5f) n = mul(n, -1.f);
    const V t1 = norm(std::fabs(n.x) > 0.5f ? cross(n, V{0, 1, 0}) : cross(n, V{1, 0, 0})), t2 = cross(n, t1);
    const float r1 = U(rng), r2 = U(rng), rr = std::sqrt(r1), ph = 6.2831853f * r2;
    const V dir = norm(add(mul(n, std::sqrt(1.f - r1)), add(mul(t1, rr * std::cos(ph)), mul(t2, rr * std::sin(ph)))));
    const V org = add(add(add(f3(p.p0), mul(e1, u)), mul(e2, v)), mul(dir, kEps));
    walk(F, org, dir, sec);
    for (size_t w = 0; w < wides.size(); ++w) wides[w].walk(org, dir, wsec[w], wlv[w]);
  }
  for (size_t w = 0; w < wides.size(); ++w) {
    std::printf("%d-wide: nodes %zu | mix(1:3) %.2f nodes %.2f tests %.2f leaves | rays whose stack exceeds",
                wides[w].W, wides[w].nodes.size(), (wcam[w].nodes + 3 * wsec[w].nodes) / (4.0 * nrays),
                (wcam[w].tests + 3 * wsec[w].tests) / (4.0 * nrays), wlv[w] / (2.0 * nrays));
    long tot = 0, above[4] = {0, 0, 0, 0};
    const int lim[4] = {8, 12, 16, 24};
    for (int k = 0; k < 64; ++k) {
      tot += wides[w].sp_hist[static_cast<size_t>(k)];
      for (int j = 0; j < 4; ++j) above[j] += k > lim[j] ? wides[w].sp_hist[static_cast<size_t>(k)] : 0;
    }
    for (int j = 0; j < 4; ++j) std::printf(" %d: %.2e", lim[j], double(above[j]) / double(tot));
    std::printf("\n");
  }
  std::printf("nodes %zu leaves %d depth %d sah %.2f | camera %.2f nodes %.2f tests | secondary %.2f nodes %.2f tests"
              " | mix(1:3) %.2f nodes %.2f tests\n",
              F.nodes.size(), F.leaves, F.depth, sah, cam.nodes / nrays, cam.tests / nrays, sec.nodes / nrays,
              sec.tests / nrays, (cam.nodes + 3 * sec.nodes) / (4.0 * nrays), (cam.tests + 3 * sec.tests) / (4.0 * nrays));
  return 0;
}
