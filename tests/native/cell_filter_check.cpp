// CPU check of cell_may_be_reached (csrc/wr_fast.h): is it conservative for
// the leaves the reference's KD walk actually reaches?  The walk here is
// KDtreeAccel::traverse (KDtreeAccel.cpp:309-388) as kd_walk states it (root
// clip, belowFirst near / far rule, the :323 stop, no early exit), over the
// tree wr_scene.cpp builds; every leaf it reaches is given to a host copy of
// cell_may_be_reached, float op for float op.  Rays: plane-grazing ones
// (origins on or just off a triangle, directions tilted out of its plane by
// 1e-8 .. 3e-3 rad) and random ones.  Prints every reached leaf the filter
// would drop.  Built and run by tests/test_cell_filter.py; CPU only.
//
//   cell_filter_check SCENE NRAYS SEED
//   cell_filter_check SCENE --rays RAYS.f32 [--list]
// Exit status 1 if any reached leaf would be dropped.
#include <cmath>
#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "wr_scene.h"

namespace {

struct V {
  float x, y, z;
};

float ax(const V& v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }
float smax(float a, float b) { return (a < b) ? b : a; }
float smin(float a, float b) { return (b < a) ? b : a; }

// AABB::hit (AABB.cpp:9-32), as wr_traverse.h box_hit
bool box_hit(V l, V r, V o, V d, float& t1, float& t2) {
  float tmin = -INFINITY, tmax = INFINITY;
  for (int i = 0; i < 3; ++i) {
    const float inv = 1.f / ax(d, i);
    float tn = (ax(l, i) - ax(o, i)) * inv;
    float tf = (ax(r, i) - ax(o, i)) * inv;
    if (tn > tf) std::swap(tn, tf);
    tmin = smax(tmin, tn);
    tmax = smin(tmax, tf);
    if (tmin > tmax) return false;
  }
  t1 = tmin;
  t2 = tmax;
  return true;
}

// wr_fast.h cell_may_be_reached, on a cell (lo, hi); tmax0: the root interval's end
bool cell_may_be_reached(V lo, V hi, V o, V d, float tmax0) {
  if (!(tmax0 > 0.f)) return true;
  if (!(std::fabs(d.x) > 1e-20f && std::fabs(d.y) > 1e-20f && std::fabs(d.z) > 1e-20f)) return true;
  const float mx = 1e-5f * (std::fabs(lo.x) + std::fabs(hi.x) + 2.f * std::fabs(o.x)) + 1e-30f;
  const float my = 1e-5f * (std::fabs(lo.y) + std::fabs(hi.y) + 2.f * std::fabs(o.y)) + 1e-30f;
  const float mz = 1e-5f * (std::fabs(lo.z) + std::fabs(hi.z) + 2.f * std::fabs(o.z)) + 1e-30f;
  const float ix = 1.f / d.x, iy = 1.f / d.y, iz = 1.f / d.z;
  const float x0 = (lo.x - mx - o.x) * ix, x1 = (hi.x + mx - o.x) * ix;
  const float y0 = (lo.y - my - o.y) * iy, y1 = (hi.y + my - o.y) * iy;
  const float z0 = (lo.z - mz - o.z) * iz, z1 = (hi.z + mz - o.z) * iz;
  const float tn = std::fmax(std::fmax(std::fmin(x0, x1), std::fmin(y0, y1)), std::fmin(z0, z1));
  const float tf = std::fmin(std::fmin(std::fmax(x0, x1), std::fmax(y0, y1)), std::fmax(z0, z1));
  return !(tn > tf);
}

// Triangle::hit (triangle.cpp:22-87) as tri_test's exact part: accept and t
int cmpf(float x) { return (x < -1e-3f) ? -1 : (x > 1e-3f); }
bool tri_hit(const wr::Prim& p, V o, V d, float& t) {
  const float A = p.p0.x - p.p1.x, B = p.p0.y - p.p1.y, C = p.p0.z - p.p1.z;
  const float D = p.p0.x - p.p2.x, E = p.p0.y - p.p2.y, F = p.p0.z - p.p2.z;
  const float G = d.x, H = d.y, I = d.z, J = p.p0.x - o.x, K = p.p0.y - o.y, L = p.p0.z - o.z;
  const float EIHF = E * I - H * F, GFDI = G * F - D * I, DHEG = D * H - E * G;
  const float denom = A * EIHF + B * GFDI + C * DHEG;
  const float bnum = J * EIHF + K * GFDI + L * DHEG;
  const float AKJB = A * K - J * B, JCAL = J * C - A * L, BLKC = B * L - K * C;
  const float gnum = I * AKJB + H * JCAL + G * BLKC;
  const float tnum = -(F * AKJB + E * JCAL + D * BLKC);
  const float beta = bnum / denom, gamma = gnum / denom;
  t = tnum / denom;
  return !(cmpf(beta) < 0 || beta > 1.f) && !(cmpf(gamma) < 0 || beta + gamma > 1.f) && cmpf(t) > 0;
}

struct Entry {
  int node;
  float tmin, tmax;
  V lo, hi;
};

// the walk; calls leaf(node, lo, hi, tmin, tmax) for every leaf reached
template <class F>
void walk(const wr::Scene& s, V o, V d, float rtmax, float& root_tmax, F leaf) {
  const V rl{s.root_l.x, s.root_l.y, s.root_l.z}, rr{s.root_r.x, s.root_r.y, s.root_r.z};
  float tmin, tmax;
  if (!box_hit(rl, rr, o, d, tmin, tmax) || rtmax < tmin) return;
  root_tmax = tmax;
  const V inv{1.f / d.x, 1.f / d.y, 1.f / d.z};
  std::vector<Entry> stk;
  Entry cur{0, tmin, tmax, rl, rr};
  for (;;) {
    const wr::KdNode& n = s.nodes[static_cast<size_t>(cur.node)];
    if (n.axis >= 0) {
      const int a = n.axis;
      const float oa = ax(o, a), da = ax(d, a), ia = ax(inv, a);
      const float t = (n.split - oa) * ia;
      const bool below = (oa < n.split) || (oa == n.split && da <= 0);
      Entry L = cur, R = cur;
      L.node = cur.node + 1;
      R.node = n.right;
      // the cells of the path records (wr_bvh.cpp): clipped to the parent's
      float& lh = a == 0 ? L.hi.x : a == 1 ? L.hi.y : L.hi.z;
      float& rl = a == 0 ? R.lo.x : a == 1 ? R.lo.y : R.lo.z;
      lh = std::min(lh, n.split);
      rl = std::max(rl, n.split);
      Entry nearc = below ? L : R, farc = below ? R : L;
      if (t > cur.tmax || t <= 0) {
        cur = nearc;
      } else if (t < cur.tmin) {
        cur = farc;
      } else {
        farc.tmin = t;
        stk.push_back(farc);
        nearc.tmax = t;
        cur = nearc;
      }
      continue;
    }
    leaf(cur);
    if (stk.empty()) return;
    cur = stk.back();
    stk.pop_back();
    if (rtmax < cur.tmin) return;
  }
}

V norm(double x, double y, double z) {
  const float fx = static_cast<float>(x), fy = static_cast<float>(y), fz = static_cast<float>(z);
  const float l = std::sqrt(fx * fx + fy * fy + fz * fz);
  return V{fx / l, fy / l, fz / l};
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    std::printf("usage: cell_filter_check SCENE NRAYS SEED\n");
    return 2;
  }
  wr::Scene s;
  std::string err;
  if (!wr::load_scene(argv[1], s, err)) {
    std::printf("load failed: %s\n", err.c_str());
    return 2;
  }
  // RAYS mode: argv[2] = "--rays", argv[3] = a raw float32 file of N x 8
  // (o, d, tmin, tmax; native.rays_from_arrays' layout)
  std::vector<float> file_rays;
  if (std::string(argv[2]) == "--rays") {
    FILE* f = std::fopen(argv[3], "rb");
    if (!f) return 2;
    float buf[8];
    while (std::fread(buf, sizeof(float), 8, f) == 8) file_rays.insert(file_rays.end(), buf, buf + 8);
    std::fclose(f);
  }
  const bool list = argc > 4 && std::string(argv[4]) == "--list";
  const long n = file_rays.empty() ? std::atol(argv[2]) : static_cast<long>(file_rays.size() / 8);
  std::mt19937_64 rng(file_rays.empty() ? static_cast<uint64_t>(std::atoll(argv[3])) : 1u);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  std::normal_distribution<double> N(0.0, 1.0);
  std::vector<int> tris;
  for (size_t i = 0; i < s.prims.size(); ++i)
    if (s.prims[i].type == wr::kTri) tris.push_back(static_cast<int>(i));
  double scale = 0;
  for (const auto& p : s.prims)
    for (const wr::F3& q : {p.p0, p.p1, p.p2})
      scale = std::max({scale, std::fabs(double(q.x)), std::fabs(double(q.y)), std::fabs(double(q.z))});
  long leaves = 0, bad = 0, bad_rays = 0, grazing = 0, neg_hit = 0;
  for (long k = 0; k < n; ++k) {
    V o, d;
    if (!file_rays.empty()) {
      const float* r = &file_rays[static_cast<size_t>(k) * 8];
      o = V{r[0], r[1], r[2]};
      d = V{r[3], r[4], r[5]};
    } else if (k % 4 != 3 && !tris.empty()) {  // plane-grazing
      const wr::Prim& p = s.prims[static_cast<size_t>(tris[static_cast<size_t>(rng() % tris.size())])];
      double a = U(rng), b = U(rng);
      if (a + b > 1) a = 1 - a, b = 1 - b;
      const double e1[3] = {double(p.p1.x) - p.p0.x, double(p.p1.y) - p.p0.y, double(p.p1.z) - p.p0.z};
      const double e2[3] = {double(p.p2.x) - p.p0.x, double(p.p2.y) - p.p0.y, double(p.p2.z) - p.p0.z};
      double nn[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
      const double nl = std::sqrt(nn[0] * nn[0] + nn[1] * nn[1] + nn[2] * nn[2]);
      if (!(nl > 0)) continue;
      for (double& c : nn) c /= nl;
      const double r[3] = {N(rng), N(rng), N(rng)};
      double u[3] = {nn[1] * r[2] - nn[2] * r[1], nn[2] * r[0] - nn[0] * r[2], nn[0] * r[1] - nn[1] * r[0]};
      const double ul = std::sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
      for (double& c : u) c /= ul;
      const double ang = std::pow(10.0, -8 + U(rng) * (std::log10(3e-3) + 8)) * (U(rng) < 0.5 ? 1 : -1);
      const double lift = U(rng) < 0.5 ? 0.0 : std::pow(10.0, -7 + 4 * U(rng)) * scale * (U(rng) < 0.5 ? 1 : -1);
      const double pt[3] = {p.p0.x + a * e1[0] + b * e2[0], p.p0.y + a * e1[1] + b * e2[1],
                            p.p0.z + a * e1[2] + b * e2[2]};
      o = V{float(pt[0] + nn[0] * lift), float(pt[1] + nn[1] * lift), float(pt[2] + nn[2] * lift)};
      d = norm(u[0] * std::cos(ang) + nn[0] * std::sin(ang), u[1] * std::cos(ang) + nn[1] * std::sin(ang),
               u[2] * std::cos(ang) + nn[2] * std::sin(ang));
      ++grazing;
    } else {
      o = V{float((U(rng) * 2 - 1) * scale), float((U(rng) * 2 - 1) * scale), float((U(rng) * 2 - 1) * scale)};
      d = norm(N(rng), N(rng), N(rng));
    }
    if (!std::isfinite(d.x) || !std::isfinite(d.y) || !std::isfinite(d.z)) continue;
    bool rb = false;
    float root_tmax = 0.f;
    walk(s, o, d, 1e7f, root_tmax, [&](const Entry& e) {
      ++leaves;
      if (!(e.tmax > 0.f)) {
        // a leaf reached with an all-negative interval (an origin outside the
        // root box, the ray pointing away): counted when one of its triangles
        // is hit at t > EPS all the same (the walk tests it like any leaf)
        const wr::KdNode& nd = s.nodes[static_cast<size_t>(e.node)];
        for (int r = 0; r < nd.count; ++r) {
          float t;
          const wr::Prim& p = s.prims[static_cast<size_t>(s.refs[static_cast<size_t>(nd.first + r)])];
          if (p.type == wr::kTri && tri_hit(p, o, d, t)) {
            ++neg_hit;
            if (list) std::printf("NEG %ld\n", k);
            break;
          }
        }
      }
      if (!cell_may_be_reached(e.lo, e.hi, o, d, root_tmax)) {
        ++bad;
        if (!rb && bad_rays < 20)
          std::printf("DROP ray %ld o=(%.9g %.9g %.9g) d=(%.9g %.9g %.9g) leaf %d cell (%.9g %.9g %.9g)-(%.9g %.9g %.9g) "
                      "t=[%.9g %.9g]\n",
                      k, o.x, o.y, o.z, d.x, d.y, d.z, e.node, e.lo.x, e.lo.y, e.lo.z, e.hi.x, e.hi.y, e.hi.z, e.tmin,
                      e.tmax);
        rb = true;
      }
    });
    bad_rays += rb ? 1 : 0;
  }
  std::printf("rays %ld (grazing %ld) leaves %ld dropped %ld rays_with_drops %ld; hits in all-negative leaves %ld\n",
              n, grazing, leaves, bad, bad_rays, neg_hit);
  return bad == 0 ? 0 : 1;
}
