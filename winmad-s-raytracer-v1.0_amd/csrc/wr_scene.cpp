// Host scene ingestion + KD build (see wr_scene.h).  Compiled with
// -ffp-contract=off: every float expression keeps the reference's rounding.
#include "wr_scene.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <future>
#include <memory>
#include <utility>

namespace wr {
namespace {

constexpr float kEps = 1e-3f;  // math/math.h:17
constexpr float kInf = 1e7f;   // math/math.h:18
const float kPi = static_cast<float>(std::acos(-1.0));

inline int fcmp(float x) { return (x < -kEps) ? -1 : (x > kEps); }        // math.cpp:8-11
inline float smax(float a, float b) { return (a < b) ? b : a; }           // std::max
inline float smin(float a, float b) { return (b < a) ? b : a; }           // std::min

inline F3 f3(float x, float y, float z) { return F3{x, y, z}; }
inline F3 operator+(F3 a, F3 b) { return f3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline F3 operator-(F3 a, F3 b) { return f3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline F3 operator-(F3 a) { return f3(-a.x, -a.y, -a.z); }
inline F3 operator*(F3 a, float s) { return f3(a.x * s, a.y * s, a.z * s); }
inline float dot(F3 a, F3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline F3 cross(F3 a, F3 b) {
  return f3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
inline float sqr_len(F3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
inline F3 normalized(F3 a) {
  float l = std::sqrt(sqr_len(a));
  return f3(a.x / l, a.y / l, a.z / l);
}
inline float comp(const F3& a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

// ---------------------------------------------------------------- 4x4 algebra
// (transform.cpp).  Only the forward matrices of worldToRaster / rasterToWorld
// reach the device, but their values depend on the inverses taken on the way.
struct M4 {
  float v[16];
};
M4 ident() {
  M4 r{};
  r.v[0] = r.v[5] = r.v[10] = r.v[15] = 1.f;
  return r;
}
M4 mul(const M4& a, const M4& b) {  // transform.cpp:24-35
  M4 r;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      r.v[4 * i + j] = a.v[4 * i] * b.v[j] + a.v[4 * i + 1] * b.v[4 + j] +
                       a.v[4 * i + 2] * b.v[8 + j] + a.v[4 * i + 3] * b.v[12 + j];
  return r;
}
// Adjugate inverse (transform.cpp:46-176).  Cofactor k is a signed sum of six
// triple products, accumulated left to right in the order listed.
struct Term {
  int8_t s, a, b, c;
};
constexpr Term kCof[16][6] = {
    {{+1, 5, 10, 15}, {-1, 5, 11, 14}, {-1, 9, 6, 15}, {+1, 9, 7, 14}, {+1, 13, 6, 11}, {-1, 13, 7, 10}},
    {{-1, 1, 10, 15}, {+1, 1, 11, 14}, {+1, 9, 2, 15}, {-1, 9, 3, 14}, {-1, 13, 2, 11}, {+1, 13, 3, 10}},
    {{+1, 1, 6, 15}, {-1, 1, 7, 14}, {-1, 5, 2, 15}, {+1, 5, 3, 14}, {+1, 13, 2, 7}, {-1, 13, 3, 6}},
    {{-1, 1, 6, 11}, {+1, 1, 7, 10}, {+1, 5, 2, 11}, {-1, 5, 3, 10}, {-1, 9, 2, 7}, {+1, 9, 3, 6}},
    {{-1, 4, 10, 15}, {+1, 4, 11, 14}, {+1, 8, 6, 15}, {-1, 8, 7, 14}, {-1, 12, 6, 11}, {+1, 12, 7, 10}},
    {{+1, 0, 10, 15}, {-1, 0, 11, 14}, {-1, 8, 2, 15}, {+1, 8, 3, 14}, {+1, 12, 2, 11}, {-1, 12, 3, 10}},
    {{-1, 0, 6, 15}, {+1, 0, 7, 14}, {+1, 4, 2, 15}, {-1, 4, 3, 14}, {-1, 12, 2, 7}, {+1, 12, 3, 6}},
    {{+1, 0, 6, 11}, {-1, 0, 7, 10}, {-1, 4, 2, 11}, {+1, 4, 3, 10}, {+1, 8, 2, 7}, {-1, 8, 3, 6}},
    {{+1, 4, 9, 15}, {-1, 4, 11, 13}, {-1, 8, 5, 15}, {+1, 8, 7, 13}, {+1, 12, 5, 11}, {-1, 12, 7, 9}},
    {{-1, 0, 9, 15}, {+1, 0, 11, 13}, {+1, 8, 1, 15}, {-1, 8, 3, 13}, {-1, 12, 1, 11}, {+1, 12, 3, 9}},
    {{+1, 0, 5, 15}, {-1, 0, 7, 13}, {-1, 4, 1, 15}, {+1, 4, 3, 13}, {+1, 12, 1, 7}, {-1, 12, 3, 5}},
    {{-1, 0, 5, 11}, {+1, 0, 7, 9}, {+1, 4, 1, 11}, {-1, 4, 3, 9}, {-1, 8, 1, 7}, {+1, 8, 3, 5}},
    {{-1, 4, 9, 14}, {+1, 4, 10, 13}, {+1, 8, 5, 14}, {-1, 8, 6, 13}, {-1, 12, 5, 10}, {+1, 12, 6, 9}},
    {{+1, 0, 9, 14}, {-1, 0, 10, 13}, {-1, 8, 1, 14}, {+1, 8, 2, 13}, {+1, 12, 1, 10}, {-1, 12, 2, 9}},
    {{-1, 0, 5, 14}, {+1, 0, 6, 13}, {+1, 4, 1, 14}, {-1, 4, 2, 13}, {-1, 12, 1, 6}, {+1, 12, 2, 5}},
    {{+1, 0, 5, 10}, {-1, 0, 6, 9}, {-1, 4, 1, 10}, {+1, 4, 2, 9}, {+1, 8, 1, 6}, {-1, 8, 2, 5}},
};
M4 inverse(const M4& m) {
  float inv[16];
  for (int k = 0; k < 16; ++k) {
    float acc = 0.f;
    for (int t = 0; t < 6; ++t) {
      const Term& e = kCof[k][t];
      float lead = e.s > 0 ? m.v[e.a] : -m.v[e.a];
      float p = lead * m.v[e.b] * m.v[e.c];
      acc = t == 0 ? p : acc + p;
    }
    inv[k] = acc;
  }
  float det = m.v[0] * inv[0] + m.v[1] * inv[4] + m.v[2] * inv[8] + m.v[3] * inv[12];
  det = 1.f / det;
  M4 r;
  for (int i = 0; i < 16; ++i) r.v[i] = inv[i] * det;
  return r;
}
struct Xf {  // Transform: forward + inverse (transform.h)
  M4 m, mi;
};
Xf xf(const M4& m) { return Xf{m, inverse(m)}; }
Xf operator*(const Xf& a, const Xf& b) { return Xf{mul(a.m, b.m), mul(b.mi, a.mi)}; }
Xf inv(const Xf& t) { return Xf{t.mi, t.m}; }
Xf translate(F3 d) {
  return Xf{M4{{1, 0, 0, d.x, 0, 1, 0, d.y, 0, 0, 1, d.z, 0, 0, 0, 1}},
            M4{{1, 0, 0, -d.x, 0, 1, 0, -d.y, 0, 0, 1, -d.z, 0, 0, 0, 1}}};
}
Xf scale(float x, float y, float z) {
  return Xf{M4{{x, 0, 0, 0, 0, y, 0, 0, 0, 0, z, 0, 0, 0, 0, 1}},
            M4{{1.0f / x, 0, 0, 0, 0, 1.0f / y, 0, 0, 0, 0, 1.0f / z, 0, 0, 0, 0, 1}}};
}
Xf look_at(F3 pos, F3 look, F3 up) {  // transform.cpp:353-370
  F3 dir = normalized(look - pos);
  F3 u = normalized(cross(up, -dir));
  F3 left = cross(u, dir);
  F3 p = f3(dot(u, pos), dot(left, pos), dot(-dir, pos));
  M4 w = ident();
  F3 nd = -dir;
  const F3 rows[3] = {u, left, nd};
  const float tr[3] = {-p.x, -p.y, -p.z};
  for (int r = 0; r < 3; ++r) {
    w.v[4 * r] = rows[r].x;
    w.v[4 * r + 1] = rows[r].y;
    w.v[4 * r + 2] = rows[r].z;
    w.v[4 * r + 3] = tr[r];
  }
  return xf(w);
}
Xf perspective(float fov, float zn, float zf) {  // transform.cpp:379-387
  M4 p{{1, 0, 0, 0, 0, -1, 0, 0, 0, 0, (zn + zf) / (zf - zn), 2 * zf * zn / (zf - zn), 0, 0, -1, 0}};
  float it = 1.0f / std::tan(fov / 360.0f * kPi);
  return scale(it, it, 1) * xf(p);
}

// ------------------------------------------------------------- primitives
Prim make_tri(F3 a, F3 b, F3 c, int mat) {  // triangle.h:14-31
  Prim p{};
  p.type = kTri;
  p.mat = mat;
  p.p0 = a;
  p.p1 = b;
  p.p2 = c;
  p.bl = f3(smin(a.x, smin(b.x, c.x)), smin(a.y, smin(b.y, c.y)), smin(a.z, smin(b.z, c.z)));
  p.br = f3(smax(a.x, smax(b.x, c.x)), smax(a.y, smax(b.y, c.y)), smax(a.z, smax(b.z, c.z)));
  return p;
}
Prim make_sphere(F3 c, float r, int mat) {  // sphere.h:16-21
  Prim p{};
  p.type = kSphere;
  p.mat = mat;
  p.c = c;
  p.r = r;
  p.bl = f3(c.x - r, c.y - r, c.z - r);
  p.br = f3(c.x + r, c.y + r, c.z + r);
  return p;
}
void extend_box(Prim& p) {  // AABB::extend (AABB.h:13-21)
  if (fcmp(p.bl.x - p.br.x) == 0) p.br.x += 10 * kEps;
  if (fcmp(p.bl.y - p.br.y) == 0) p.br.y += 10 * kEps;
  if (fcmp(p.bl.z - p.br.z) == 0) p.br.z += 10 * kEps;
}
Light make_light(F3 p0, F3 p1, F3 p2, F3 le);
void add_prim(Scene& s, Prim p) {  // Scene::addGeometry (scene.cpp:5-9)
  extend_box(p);
  if (p.type == kTri) {
    F3 n = cross(p.p1 - p.p0, p.p2 - p.p0);
    s.tot_area += 0.5f * std::sqrt(sqr_len(n));
  } else {
    s.tot_area += 4 * kPi * (p.r * p.r);
  }
  s.prims.push_back(p);
}

struct Frame {
  F3 x, y, z;
};
Frame frame_from_z(F3 z0) {  // frame.cpp:3-11
  Frame f;
  f.z = normalized(z0);
  F3 tx = (std::fabs(f.z.x) > 0.99f) ? f3(0.0f, 1.0f, 0.0f) : f3(1.0f, 0.0f, 0.0f);
  f.y = normalized(cross(f.z, tx));
  f.x = cross(f.y, f.z);
  return f;
}
Light make_light(F3 p0, F3 p1, F3 p2, F3 le) {  // light.h:90-103
  Light l{};
  l.le = le;
  l.p0 = p0;
  l.d1 = p1 - p0;
  l.d2 = p2 - p0;
  F3 n = cross(l.d1, l.d2);
  float len = std::sqrt(sqr_len(n));
  l.inv_area = 2.f / len;
  n = normalized(n);
  Frame fr = frame_from_z(n);
  l.fx = fr.x;
  l.fy = fr.y;
  l.fz = fr.z;
  return l;
}

// ------------------------------------------------------------------ .obj
// tinyobjloader 0.9.x semantics (tiny_obj_loader.cpp:461-661): v lines parsed
// with (float)atof, faces fan-triangulated (f0, f[k-1], f[k]), a shape flushed
// at every g / o line, negative indices relative to the vertices seen so far.
struct ObjShape {
  std::string name;
  std::vector<int> tri;  // 3 vertex indices per triangle (into verts)
};
struct ObjFile {
  std::vector<float> verts;
  std::vector<ObjShape> shapes;
};

bool read_file(const char* path, std::string& out) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  out.resize(n > 0 ? static_cast<size_t>(n) : 0);
  size_t got = n > 0 ? std::fread(&out[0], 1, out.size(), f) : 0;
  out.resize(got);
  std::fclose(f);
  return true;
}

inline bool is_ws(char c) { return c == ' ' || c == '\t'; }

// returns 0 ok / 1 missing file / -1 malformed
int parse_obj(const char* path, ObjFile& of) {
  std::string text;
  if (!read_file(path, text)) return 1;
  // lines are parsed in place: each '\n' becomes the line's terminator
  for (char& c : text)
    if (c == '\n') c = 0;
  // faces of the current group, flat: face f is fidx[fbeg[f] .. fbeg[f + 1])
  std::vector<int> fidx, fbeg(1, 0);
  std::string name;
  auto flush = [&]() -> bool {
    if (fbeg.size() == 1) return true;
    ObjShape sh;
    sh.name = name;
    const int nv = static_cast<int>(of.verts.size() / 3);
    for (size_t f = 0; f + 1 < fbeg.size(); ++f) {
      const int* face = fidx.data() + fbeg[f];
      const int fn = fbeg[f + 1] - fbeg[f];
      for (int k = 2; k < fn; ++k) {
        int i0 = face[0], i1 = face[k - 1], i2 = face[k];
        if (i0 < 0 || i1 < 0 || i2 < 0 || i0 >= nv || i1 >= nv || i2 >= nv) return false;
        sh.tri.push_back(i0);
        sh.tri.push_back(i1);
        sh.tri.push_back(i2);
      }
    }
    of.shapes.push_back(std::move(sh));
    fidx.clear();
    fbeg.assign(1, 0);
    return true;
  };
  size_t pos = 0;
  const size_t len = text.size();
  while (pos < len) {
    const char* t = text.c_str() + pos;
    pos += std::strlen(t) + 1;
    t += std::strspn(t, " \t");
    if (!*t || *t == '#') continue;
    if (t[0] == 'v' && is_ws(t[1])) {
      t += 2;
      for (int k = 0; k < 3; ++k) {
        t += std::strspn(t, " \t");
        of.verts.push_back(static_cast<float>(std::atof(t)));
        t += std::strcspn(t, " \t\r");
      }
      continue;
    }
    if (t[0] == 'f' && is_ws(t[1])) {
      t += 2;
      t += std::strspn(t, " \t");
      const int vcount = static_cast<int>(of.verts.size() / 3);
      while (!(*t == '\r' || *t == '\n' || *t == 0)) {
        int raw = std::atoi(t);
        fidx.push_back(raw > 0 ? raw - 1 : (raw == 0 ? 0 : vcount + raw));
        // skip the i / i/j / i//k / i/j/k triple (only the position index is used)
        for (int part = 0; part < 3; ++part) {
          t += std::strcspn(t, "/ \t\r");
          if (*t != '/') break;
          ++t;
          if (*t == '/') ++t, part = 1;
        }
        t += std::strspn(t, " \t\r");
      }
      fbeg.push_back(static_cast<int>(fidx.size()));
      continue;
    }
    if ((t[0] == 'g' || t[0] == 'o') && is_ws(t[1])) {
      if (!flush()) return -1;
      const char* q = t + 1;
      q += std::strspn(q, " \t\r");
      size_t n = std::strcspn(q, t[0] == 'g' ? " \t\r" : " \t\r\n\v\f");
      name.assign(q, n);
      continue;
    }
  }
  if (!flush()) return -1;
  return 0;
}

// ------------------------------------------------------------------ XML
struct XNode {
  std::string tag;
  std::vector<std::pair<std::string, std::string>> attrs;
  std::vector<std::unique_ptr<XNode>> kids;
  const char* attr(const char* k) const {
    for (const auto& a : attrs)
      if (a.first == k) return a.second.c_str();
    return nullptr;
  }
  const XNode* kid(size_t i) const { return i < kids.size() ? kids[i].get() : nullptr; }
};

class XmlReader {
 public:
  explicit XmlReader(const std::string& s) : s_(s) {}
  std::unique_ptr<XNode> root() {
    skip_misc();
    return element();
  }

 private:
  const std::string& s_;
  size_t p_ = 0;
  bool at(const char* lit) const { return s_.compare(p_, std::strlen(lit), lit) == 0; }
  void skip_misc() {  // text, comments, <?...?>, <!...>
    for (;;) {
      while (p_ < s_.size() && s_[p_] != '<') ++p_;
      if (p_ >= s_.size()) return;
      if (at("<!--")) {
        size_t e = s_.find("-->", p_);
        p_ = e == std::string::npos ? s_.size() : e + 3;
      } else if (at("<?") || at("<!")) {
        size_t e = s_.find('>', p_);
        p_ = e == std::string::npos ? s_.size() : e + 1;
      } else {
        return;
      }
    }
  }
  static std::string decode(const std::string& v) {
    static const char* ent[5] = {"&amp;", "&lt;", "&gt;", "&quot;", "&apos;"};
    static const char rep[5] = {'&', '<', '>', '"', '\''};
    std::string o;
    for (size_t i = 0; i < v.size(); ++i) {
      bool done = false;
      if (v[i] == '&')
        for (int k = 0; k < 5 && !done; ++k)
          if (v.compare(i, std::strlen(ent[k]), ent[k]) == 0) {
            o += rep[k];
            i += std::strlen(ent[k]) - 1;
            done = true;
          }
      if (!done) o += v[i];
    }
    return o;
  }
  std::unique_ptr<XNode> element() {
    if (p_ >= s_.size() || s_[p_] != '<' || (p_ + 1 < s_.size() && s_[p_ + 1] == '/')) return nullptr;
    ++p_;
    auto n = std::make_unique<XNode>();
    size_t e = s_.find_first_of(" \t\r\n/>", p_);
    if (e == std::string::npos) return nullptr;
    n->tag = s_.substr(p_, e - p_);
    p_ = e;
    for (;;) {
      while (p_ < s_.size() && std::strchr(" \t\r\n", s_[p_])) ++p_;
      if (p_ >= s_.size()) return n;
      if (at("/>")) {
        p_ += 2;
        return n;
      }
      if (s_[p_] == '>') {
        ++p_;
        break;
      }
      size_t ke = s_.find_first_of(" \t\r\n=/>", p_);
      if (ke == std::string::npos) return n;
      std::string key = s_.substr(p_, ke - p_);
      p_ = ke;
      while (p_ < s_.size() && std::strchr(" \t\r\n", s_[p_])) ++p_;
      if (p_ >= s_.size() || s_[p_] != '=') {
        ++p_;
        continue;
      }
      ++p_;
      while (p_ < s_.size() && std::strchr(" \t\r\n", s_[p_])) ++p_;
      if (p_ >= s_.size() || (s_[p_] != '"' && s_[p_] != '\'')) continue;
      char q = s_[p_++];
      size_t ve = s_.find(q, p_);
      if (ve == std::string::npos) ve = s_.size();
      n->attrs.emplace_back(decode(key), decode(s_.substr(p_, ve - p_)));
      p_ = ve + 1;
    }
    for (;;) {
      skip_misc();
      if (p_ >= s_.size()) return n;
      if (at("</")) {
        size_t e2 = s_.find('>', p_);
        p_ = e2 == std::string::npos ? s_.size() : e2 + 1;
        return n;
      }
      auto k = element();
      if (!k) return n;
      n->kids.push_back(std::move(k));
    }
  }
};

// TiXmlElement::Attribute(name, double*) / (name, int*): atof / atoi, 0 if absent
double att_d(const XNode* e, const char* k) {
  const char* v = e ? e->attr(k) : nullptr;
  return v ? std::atof(v) : 0.0;
}
int att_i(const XNode* e, const char* k) {
  const char* v = e ? e->attr(k) : nullptr;
  return v ? std::atoi(v) : 0;
}
F3 att_xyz(const XNode* e) {
  return f3(static_cast<float>(att_d(e, "x")), static_cast<float>(att_d(e, "y")),
            static_cast<float>(att_d(e, "z")));
}
F3 att_rgb(const XNode* e) {
  return f3(static_cast<float>(att_d(e, "r")), static_cast<float>(att_d(e, "g")),
            static_cast<float>(att_d(e, "b")));
}

// ------------------------------------------------------------------ KD build
struct Ev {
  float pos;
  int type;  // End = 0, Planar = 1, Start = 2 (KDtreeAccel.h:9-18)
  int idx;
};
inline int ev_order(const Ev& a, const Ev& b) {  // KDtreeAccel.cpp:3-10
  int c = fcmp(a.pos - b.pos);
  return c != 0 ? c : a.type - b.type;
}
// The reference sorts with qsort(); glibc 2.35's qsort is a top-down merge sort
// (n1 = n/2, left run wins ties: cmp <= 0).  The comparator is EPS-tolerant
// and not transitive, so that exact merge tree is reproduced.
void merge_sort(Ev* b, size_t n, Ev* tmp) {
  if (n <= 1) return;
  size_t n1 = n / 2, n2 = n - n1;
  Ev *l = b, *r = b + n1;
  merge_sort(l, n1, tmp);
  merge_sort(r, n2, tmp);
  Ev* o = tmp;
  while (n1 && n2) {
    if (ev_order(*l, *r) <= 0) {
      *o++ = *l++;
      --n1;
    } else {
      *o++ = *r++;
      --n2;
    }
  }
  std::copy(l, l + n1, o);
  std::copy(tmp, tmp + (n - n2), b);
}

struct Work {
  std::vector<int> obj;
  F3 bl{}, br{};
  std::vector<Ev> ev[3];
};

struct Sub {
  std::vector<KdNode> nodes;
  std::vector<int> refs;
  int max_stack = 0;
};

inline float surface(F3 v) { return 2 * (v.x * v.y + v.x * v.z + v.y * v.z); }

class Builder {
 public:
  Builder(const Scene& s, int dep_max) : s_(s), dep_max_(dep_max) {}

  void build(Work&& w, int dep, Sub& out) {
    const int me = static_cast<int>(out.nodes.size());
    out.nodes.push_back(KdNode{-1, 0.f, 0, 0, 0});
    const int nobj = static_cast<int>(w.obj.size());
    float split = 0.f;
    int axis = -1;
    if (dep <= dep_max_ && nobj > 1) axis = find_split(w, split);
    if (axis < 0) {  // leaf (buildTree returns early, :120-123)
      out.nodes[me].first = static_cast<int>(out.refs.size());
      out.nodes[me].count = nobj;
      out.refs.insert(out.refs.end(), w.obj.begin(), w.obj.end());
      out.max_stack = std::max(out.max_stack, dep - 1);
      return;
    }
    Work L, R;
    partition(w, axis, split, L, R);
    out.nodes[me].axis = axis;
    out.nodes[me].split = split;
    out.nodes[me].count = nobj;
    // independent subtrees: the right one on another thread when both sides are
    // large (by size, not depth: the SAH's top splits peel small parts off),
    // spliced after the left one -- the serial layout
    bool spawn = L.obj.size() >= kParallelMin && R.obj.size() >= kParallelMin;
    if (spawn && threads_.fetch_add(1) >= kMaxThreads) {
      threads_.fetch_sub(1);
      spawn = false;
    }
    if (spawn) {
      Sub rs;
      auto fut = std::async(std::launch::async, [&] { build(std::move(R), dep + 1, rs); });
      build(std::move(L), dep + 1, out);
      fut.get();
      threads_.fetch_sub(1);
      const int nbase = static_cast<int>(out.nodes.size());
      const int rbase = static_cast<int>(out.refs.size());
      out.nodes[me].right = nbase;
      for (KdNode n : rs.nodes) {
        if (n.axis >= 0) n.right += nbase;
        else n.first += rbase;
        out.nodes.push_back(n);
      }
      out.refs.insert(out.refs.end(), rs.refs.begin(), rs.refs.end());
      out.max_stack = std::max(out.max_stack, rs.max_stack);
    } else {
      build(std::move(L), dep + 1, out);
      out.nodes[me].right = static_cast<int>(out.nodes.size());
      build(std::move(R), dep + 1, out);
    }
  }

 private:
  static constexpr size_t kParallelMin = 4096;
  static constexpr int kMaxThreads = 32;
  const Scene& s_;
  int dep_max_;
  std::atomic<int> threads_{0};

  float sah(const Work& w, int axis, float plane, int nl, int nr) const {  // :64-80
    F3 v = w.br - w.bl, vl = v, vr = v;
    if (axis == 0) vl.x = plane - w.bl.x, vr.x = w.br.x - plane;
    if (axis == 1) vl.y = plane - w.bl.y, vr.y = w.br.y - plane;
    if (axis == 2) vl.z = plane - w.bl.z, vr.z = w.br.z - plane;
    float lambda = (nl == 0 || nr == 0) ? 0.8f : 1.0f;
    return (lambda / surface(v)) * (surface(vl) * static_cast<float>(nl) +
                                    surface(vr) * static_cast<float>(nr));
  }

  int find_split(const Work& w, float& split) const {  // :82-116
    float cost = kInf;
    int best = -1;
    const int nobj = static_cast<int>(w.obj.size());
    for (int axis = 0; axis < 3; ++axis) {
      const std::vector<Ev>& ev = w.ev[axis];
      int nl = 0, nr = nobj;
      size_t i = 0;
      while (i < ev.size()) {
        const float now = ev[i].pos;
        int ends = 0, starts = 0;
        for (; i < ev.size() && ev[i].pos == now; ++i) {
          ends += ev[i].type == 0;
          starts += ev[i].type == 2;
        }
        nr -= ends;
        float c = sah(w, axis, now, nl, nr);
        if (fcmp(c - cost) < 0) {
          cost = c;
          split = now;
          best = axis;
        }
        nl += starts;
      }
    }
    return best;
  }

  void partition(Work& w, int axis, float split, Work& L, Work& R) const {  // :125-298
    const int nobj = static_cast<int>(w.obj.size());
    std::vector<int8_t> side(nobj);   // 0 left only, 1 right only, 2 both
    std::vector<int> to_l(nobj, -1), to_r(nobj, -1);
    for (int i = 0; i < nobj; ++i) {
      const Prim& p = s_.prims[w.obj[i]];
      float st = comp(p.bl, axis), ed = comp(p.br, axis);
      side[i] = fcmp(ed - split) <= 0 ? 0 : (fcmp(split - st) <= 0 ? 1 : 2);
      if (side[i] != 1) {
        to_l[i] = static_cast<int>(L.obj.size());
        L.obj.push_back(w.obj[i]);
      }
      if (side[i] != 0) {
        to_r[i] = static_cast<int>(R.obj.size());
        R.obj.push_back(w.obj[i]);
      }
    }
    for (int a = 0; a < 3; ++a) {
      L.ev[a].reserve(2 * L.obj.size());
      R.ev[a].reserve(2 * R.obj.size());
      for (const Ev& e : w.ev[a]) {
        const int sd = side[e.idx];
        if (sd != 1) {
          Ev x{e.pos, e.type, to_l[e.idx]};
          if (sd == 2 && a == axis && e.type == 0) x.pos = split;  // End clipped left
          L.ev[a].push_back(x);
        }
        if (sd != 0) {
          Ev x{e.pos, e.type, to_r[e.idx]};
          if (sd == 2 && a == axis && e.type == 2) x.pos = split;  // Start clipped right
          R.ev[a].push_back(x);
        }
      }
      std::vector<Ev>().swap(w.ev[a]);
    }
    for (Work* c : {&L, &R}) {
      if (c->obj.empty()) continue;
      c->bl = f3(c->ev[0].front().pos, c->ev[1].front().pos, c->ev[2].front().pos);
      c->br = f3(c->ev[0].back().pos, c->ev[1].back().pos, c->ev[2].back().pos);
    }
    std::vector<int>().swap(w.obj);
  }
};

}  // namespace

void setup_camera(Camera& c, F3 pos, F3 fwd, F3 up, float xres, float yres, float fov) {
  c.pos = pos;  // camera.cpp:3-29
  c.fwd = normalized(fwd);
  c.up = normalized(up);
  c.xres = xres;
  c.yres = yres;
  c.fov = fov;
  Xf w2c = look_at(c.pos, c.pos + c.fwd, c.up);
  Xf w2n = perspective(fov, 0.1f, 10000.f) * w2c;
  Xf w2r = scale(xres * 0.5f, yres * 0.5f, 0) * translate(f3(1.0f, 1.0f, 0.0f)) * w2n;
  Xf r2w = inv(w2n) * translate(f3(-1.0f, -1.0f, 0.0f)) * scale(2.0f / xres, 2.0f / yres, 0);
  std::memcpy(c.w2r, w2r.m.v, sizeof c.w2r);
  std::memcpy(c.r2w, r2w.m.v, sizeof c.r2w);
  c.plane_dist = xres / (2.0f * std::tan(fov * kPi / 360.0f));
}

void build_kdtree(Scene& s) {  // KDtreeAccel::init (:12-57) + buildTree
  const int n = static_cast<int>(s.prims.size());
  s.nodes.clear();
  s.refs.clear();
  if (n == 0) return;
  s.dep_max = static_cast<int>(1.2 * std::log(static_cast<double>(n)) + 2.0);
  Work root;
  root.obj.resize(n);
  for (int i = 0; i < n; ++i) root.obj[i] = i;
  std::future<void> sorts[3];
  for (int a = 0; a < 3; ++a) {
    sorts[a] = std::async(std::launch::async, [&, a] {
      std::vector<Ev>& ev = root.ev[a];
      ev.resize(2 * static_cast<size_t>(n));
      for (int j = 0; j < n; ++j) {
        ev[2 * j] = Ev{comp(s.prims[j].bl, a), 2, j};
        ev[2 * j + 1] = Ev{comp(s.prims[j].br, a), 0, j};
      }
      std::vector<Ev> tmp(ev.size());
      merge_sort(ev.data(), ev.size(), tmp.data());
    });
  }
  for (auto& f : sorts) f.get();
  root.bl = f3(root.ev[0].front().pos, root.ev[1].front().pos, root.ev[2].front().pos);
  root.br = f3(root.ev[0].back().pos, root.ev[1].back().pos, root.ev[2].back().pos);
  s.root_l = root.bl;
  s.root_r = root.br;
  Sub out;
  Builder(s, s.dep_max).build(std::move(root), 1, out);
  s.nodes = std::move(out.nodes);
  s.refs = std::move(out.refs);
  s.max_stack = out.max_stack;
  // scene sphere (scene.cpp:483-487)
  F3 diag = s.root_r - s.root_l;
  float d2 = sqr_len(diag);
  s.sph_c = (s.root_l + s.root_r) * 0.5f;
  s.sph_r = std::sqrt(d2) * 0.5f;
  s.sph_inv_r2 = 1.f / d2;
}

bool load_scene(const char* path, Scene& s, std::string& err) {
  std::string text;
  if (!read_file(path, text)) {
    err = std::string("cannot open scene file ") + path;
    return false;
  }
  auto root = XmlReader(text).root();
  if (!root) {
    err = std::string("no root element in ") + path;
    return false;
  }
  s = Scene();
  for (const auto& kp : root->kids) {
    const XNode* it = kp.get();
    if (it->tag == "camera") {  // scene.cpp:276-304 (children read by position)
      const XNode *pos = it->kid(0), *fwd = it->kid(1), *up = it->kid(2), *res = it->kid(3),
                  *fov = it->kid(4);
      if (!fov) {
        err = "camera element needs 5 children";
        return false;
      }
      setup_camera(s.cam, att_xyz(pos), att_xyz(fwd), att_xyz(up), static_cast<float>(att_d(res, "height")),
                   static_cast<float>(att_d(res, "width")), static_cast<float>(att_d(fov, "horizontalFOV")));
      s.has_camera = true;
    } else if (it->tag == "material") {  // scene.cpp:305-332
      if (!it->kid(4)) {
        err = "material element needs 5 children";
        return false;
      }
      Material m;
      m.diffuse = att_rgb(it->kid(0));
      m.phong = att_rgb(it->kid(1));
      m.specular = att_rgb(it->kid(2));
      m.phong_exp = static_cast<float>(att_d(it->kid(3), "phongExp"));
      m.index = static_cast<float>(att_d(it->kid(4), "refracIndex"));
      s.mats.push_back(m);
    } else if (it->tag == "object" || it->tag == "area_light") {  // scene.cpp:333-374, 397-432
      const char* file = it->kid(0) ? it->kid(0)->attr("path") : nullptr;
      if (!file || !it->kid(1)) {
        err = "<" + it->tag + "> needs a file_path and a second child";
        return false;
      }
      ObjFile of;
      int rc = parse_obj(file, of);
      if (rc < 0) {
        err = std::string("vertex index out of range in ") + file;
        return false;
      }
      if (rc == 1) ++s.missing_files;
      const bool light = it->tag == "area_light";
      const int mat = light ? 0 : att_i(it->kid(1), "matid");
      const F3 le = light ? att_rgb(it->kid(1)) : F3{};
      auto vert = [&](int i) { return f3(of.verts[3 * i], of.verts[3 * i + 1], of.verts[3 * i + 2]); };
      for (const ObjShape& sh : of.shapes) {
        const size_t nt = sh.tri.size() / 3;
        for (size_t f = 0; f < nt; ++f) {
          F3 a = vert(sh.tri[3 * f]), b = vert(sh.tri[3 * f + 1]), c = vert(sh.tri[3 * f + 2]);
          if (light) {  // one AreaLight + one emitter triangle per face, matId -(f+1)
            s.lights.push_back(make_light(a, b, c, le));
            add_prim(s, make_tri(a, b, c, -static_cast<int>(f + 1)));
          } else {
            if (sh.name == "water") {  // scene.cpp:360-368
              F3 nn = cross(b - a, c - a);
              if (nn.y < kEps) std::swap(a, c);
            }
            add_prim(s, make_tri(a, b, c, mat));
          }
        }
      }
    } else if (it->tag == "sphere") {  // scene.cpp:375-396
      add_prim(s, make_sphere(att_xyz(it->kid(0)), static_cast<float>(att_d(it->kid(1), "radius")),
                              att_i(it->kid(2), "matid")));
    }
    // homo_media: participating media are outside the surface hot path
  }
  build_kdtree(s);
  return true;
}

bool scene_from_arrays(const SceneArrays& a, Scene& s, std::string& err) {
  if (a.n_prims < 0 || a.n_lights < 0 || a.n_materials < 0) {
    err = "negative count";
    return false;
  }
  if ((a.n_prims && (!a.prim_type || !a.prim_data || !a.prim_mat)) || (a.n_lights && (!a.light_tri || !a.light_le)) ||
      (a.n_materials && !a.materials)) {
    err = "null array with a nonzero count";
    return false;
  }
  s = Scene();
  auto v = [](const float* q) { return f3(q[0], q[1], q[2]); };
  for (int i = 0; i < a.n_materials; ++i) {  // scene.cpp:305-332
    const float* m = a.materials + 11 * static_cast<size_t>(i);
    s.mats.push_back(Material{v(m), v(m + 3), v(m + 6), m[9], m[10]});
  }
  for (int i = 0; i < a.n_lights; ++i) {  // AreaLight(p0, p1, p2, intensity) (light.h:90-103)
    const float* t = a.light_tri + 9 * static_cast<size_t>(i);
    s.lights.push_back(make_light(v(t), v(t + 3), v(t + 6), v(a.light_le + 3 * static_cast<size_t>(i))));
  }
  for (int i = 0; i < a.n_prims; ++i) {  // Scene::addGeometry in objs order (scene.cpp:5-9)
    const float* q = a.prim_data + 9 * static_cast<size_t>(i);
    const int mat = a.prim_mat[i];
    if (mat < 0 && -mat - 1 >= a.n_lights) {
      err = "primitive " + std::to_string(i) + ": emitter matId " + std::to_string(mat) + " names no area light";
      return false;
    }
    if (a.prim_type[i] == kTri) {
      add_prim(s, make_tri(v(q), v(q + 3), v(q + 6), mat));
    } else if (a.prim_type[i] == kSphere) {
      if (!(q[3] > 0.f)) {
        err = "primitive " + std::to_string(i) + ": sphere radius must be > 0";
        return false;
      }
      add_prim(s, make_sphere(v(q), q[3], mat));
    } else {
      err = "primitive " + std::to_string(i) + ": type must be 0 (triangle) or 1 (sphere)";
      return false;
    }
  }
  setup_camera(s.cam, v(a.cam_pos), v(a.cam_fwd), v(a.cam_up), a.cam_xres, a.cam_yres, a.cam_hfov);
  s.has_camera = true;
  build_kdtree(s);
  return true;
}

namespace {
void hx(std::string& o, float v) {
  char b[40];
  std::snprintf(b, sizeof b, " %a", static_cast<double>(v));
  o += b;
}
void hx3(std::string& o, F3 v) {
  hx(o, v.x);
  hx(o, v.y);
  hx(o, v.z);
}
void dump_node(const Scene& s, int id, std::string& o) {
  const KdNode& n = s.nodes[id];
  char b[64];
  if (n.axis < 0) {
    std::snprintf(b, sizeof b, "L %d", n.count);
    o += b;
    for (int i = 0; i < n.count; ++i) {
      std::snprintf(b, sizeof b, " %d", s.refs[n.first + i]);
      o += b;
    }
    o += "\n";
    return;
  }
  std::snprintf(b, sizeof b, "I %d", n.axis);
  o += b;
  hx(o, n.split);
  std::snprintf(b, sizeof b, " %d\n", n.count);
  o += b;
  dump_node(s, id + 1, o);
  dump_node(s, n.right, o);
}
}  // namespace

std::string dump_scene(const Scene& s) {
  std::string o;
  char b[64];
  std::snprintf(b, sizeof b, "nobjs %d\n", static_cast<int>(s.prims.size()));
  o += b;
  for (const Prim& p : s.prims) {
    std::snprintf(b, sizeof b, p.type == kTri ? "tri %d" : "sph %d", p.mat);
    o += b;
    if (p.type == kTri) {
      hx3(o, p.p0);
      hx3(o, p.p1);
      hx3(o, p.p2);
    } else {
      hx3(o, p.c);
      hx(o, p.r);
    }
    o += "\n";
  }
  std::snprintf(b, sizeof b, "nlights %d\n", static_cast<int>(s.lights.size()));
  o += b;
  for (const Light& l : s.lights) {
    o += "light";
    for (F3 v : {l.p0, l.d1, l.d2, l.fx, l.fy, l.fz, l.le}) hx3(o, v);
    hx(o, l.inv_area);
    o += "\n";
  }
  std::snprintf(b, sizeof b, "nmat %d\n", static_cast<int>(s.mats.size()));
  o += b;
  for (const Material& m : s.mats) {
    o += "mat";
    hx3(o, m.diffuse);
    hx3(o, m.phong);
    hx(o, m.phong_exp);
    hx3(o, m.specular);
    hx(o, m.index);
    o += "\n";
  }
  const Camera& c = s.cam;
  o += "camera";
  hx3(o, c.pos);
  hx3(o, c.fwd);
  hx3(o, c.up);
  hx(o, c.xres);
  hx(o, c.yres);
  hx(o, c.plane_dist);
  o += "\nw2r";
  for (float v : c.w2r) hx(o, v);
  o += "\nr2w";
  for (float v : c.r2w) hx(o, v);
  o += "\nsphere";
  hx3(o, s.sph_c);
  hx(o, s.sph_r);
  hx(o, s.sph_inv_r2);
  o += "\ntotarea";
  hx(o, s.tot_area);
  o += "\n";
  if (s.prims.empty()) return o;
  std::snprintf(b, sizeof b, "kd %d", s.dep_max);
  o += b;
  hx3(o, s.root_l);
  hx3(o, s.root_r);
  o += "\n";
  dump_node(s, 0, o);
  return o;
}

namespace {
thread_local std::string g_err;
}
int set_error(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
const char* last_error() { return g_err.c_str(); }

uint64_t scene_fingerprint(const Scene& s) {
  uint64_t h = 1469598103934665603ull;
  auto mix = [&h](const void* p, size_t n) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
  };
  const uint64_t n[3] = {s.prims.size(), s.lights.size(), s.mats.size()};
  mix(n, sizeof n);
  // all-4-byte-field records: no padding bytes enter the hash
  static_assert(sizeof(Prim) % 4 == 0 && sizeof(Light) % 4 == 0 && sizeof(Material) % 4 == 0, "packed records");
  if (!s.prims.empty()) mix(s.prims.data(), s.prims.size() * sizeof(Prim));
  if (!s.lights.empty()) mix(s.lights.data(), s.lights.size() * sizeof(Light));
  if (!s.mats.empty()) mix(s.mats.data(), s.mats.size() * sizeof(Material));
  mix(&s.cam, sizeof s.cam);
  return h;
}

}  // namespace wr
