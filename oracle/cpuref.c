/* cpuref.c -- CPU restatement of the reference BDPT / PT hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see cpuref.h).  Never linked by the product.
 *
 * Every function cites the reference statement range it restates; paths are
 * relative to /root/reference/Winmad-s-raytracer-v1.0/src/.  Arithmetic keeps the
 * reference's float evaluation order; compile with -ffp-contract=off.
 */
#define _GNU_SOURCE
#include "cpuref.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------------- */
/* math.h / math.cpp                                                          */
/* ------------------------------------------------------------------------- */
#define R_EPS 1e-3f /* math/math.h:17 */
#define R_INF 1e7f  /* math/math.h:18 */
static float R_PI, R_INV_PI;   /* math/math.h:15-16: acos(-1.0f), 1/PI */

static void init_consts(void) {
    if (R_PI == 0.f) {
        R_PI = (float)acos(-1.0);
        R_INV_PI = 1.0f / R_PI;
    }
}

static char g_err[512];
const char* cr_last_error(void) { return g_err; }
static void set_err(const char* m, const char* a) {
    snprintf(g_err, sizeof g_err, "%s%s%s", m, a ? ": " : "", a ? a : "");
}

/* math.cpp:8-11 */
static inline int cmpf(float x) { return (x < -R_EPS) ? -1 : (x > R_EPS); }
/* std::max / std::min semantics (second argument wins only on strict order) */
static inline float fmaxs(float a, float b) { return (a < b) ? b : a; }
static inline float fmins(float a, float b) { return (b < a) ? b : a; }
/* math.cpp:3-6 */
static inline float clampv(float v, float lo, float hi) { return fmins(hi, fmaxs(v, lo)); }

typedef struct { float x, y, z; } v3;
typedef struct { float r, g, b; } c3;

static inline v3 mk(float x, float y, float z) { v3 v = {x, y, z}; return v; }
static inline c3 mkc(float r, float g, float b) { c3 c = {r, g, b}; return c; }
/* vector.cpp:3-34 */
static inline v3 vadd(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vneg(v3 a) { return mk(-a.x, -a.y, -a.z); }
static inline float vdot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline v3 vmul3(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 vcross(v3 a, v3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline v3 vscale(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
/* vector.cpp:36-41: division by a near-zero scalar yields the INF vector */
static inline v3 vdiv(v3 a, float s) {
    if (cmpf(s) == 0) return mk(R_INF, R_INF, R_INF);
    return mk(a.x / s, a.y / s, a.z / s);
}
/* vector.cpp:43-47 */
static inline int veq(v3 a, v3 b) {
    return cmpf(a.x - b.x) == 0 && cmpf(a.y - b.y) == 0 && cmpf(a.z - b.z) == 0;
}
/* vector.h:55-68 */
static inline float vsqr(v3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
static inline float vlen(v3 a) { return sqrtf(vsqr(a)); }
static inline v3 vnorm(v3 a) {
    float l = sqrtf(vsqr(a));
    return mk(a.x / l, a.y / l, a.z / l);
}
static inline float vget(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

/* color.cpp / color.h */
static inline c3 cadd(c3 a, c3 b) { return mkc(a.r + b.r, a.g + b.g, a.b + b.b); }
static inline c3 cmul(c3 a, c3 b) { return mkc(a.r * b.r, a.g * b.g, a.b * b.b); }
static inline c3 cscale(c3 a, float s) { return mkc(a.r * s, a.g * s, a.b * s); }
static inline c3 cdivs(c3 a, float s) { return mkc(a.r / s, a.g / s, a.b / s); }
static inline int cblack(c3 a) { return cmpf(a.r) == 0 && cmpf(a.g) == 0 && cmpf(a.b) == 0; }
static inline float clum(c3 a) { return 0.2126f * a.r + 0.7152f * a.g + 0.0722f * a.b; }
static inline float cmaxc(c3 a) { return fmaxs(a.r, fmaxs(a.g, a.b)); }
static const c3 C0 = {0.f, 0.f, 0.f};

/* ------------------------------------------------------------------------- */
/* rng.cpp (MT19937) and the counter RNG                                      */
/* ------------------------------------------------------------------------- */
typedef struct { uint32_t mt[624]; int mti; } mt_state;

static void mt_seed(mt_state* s, uint32_t seed) { /* rng.cpp:8-16 */
    s->mt[0] = seed;
    for (s->mti = 1; s->mti < 624; s->mti++)
        s->mt[s->mti] = 1812433253u * (s->mt[s->mti - 1] ^ (s->mt[s->mti - 1] >> 30)) + (uint32_t)s->mti;
}

static uint32_t mt_next(mt_state* s) { /* rng.cpp:24-62 */
    static const uint32_t mag[2] = {0u, 0x9908b0dfu};
    uint32_t y;
    if (s->mti >= 624) {
        int k;
        for (k = 0; k < 624 - 397; k++) {
            y = (s->mt[k] & 0x80000000u) | (s->mt[k + 1] & 0x7fffffffu);
            s->mt[k] = s->mt[k + 397] ^ (y >> 1) ^ mag[y & 1u];
        }
        for (; k < 623; k++) {
            y = (s->mt[k] & 0x80000000u) | (s->mt[k + 1] & 0x7fffffffu);
            s->mt[k] = s->mt[k + 397 - 624] ^ (y >> 1) ^ mag[y & 1u];
        }
        y = (s->mt[623] & 0x80000000u) | (s->mt[0] & 0x7fffffffu);
        s->mt[623] = s->mt[396] ^ (y >> 1) ^ mag[y & 1u];
        s->mti = 0;
    }
    y = s->mt[s->mti++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

void cr_mt_outputs(uint32_t seed, int n, uint32_t* out) {
    mt_state s;
    mt_seed(&s, seed);
    for (int i = 0; i < n; i++) out[i] = mt_next(&s);
}

/* Counter RNG: stream key = mix(seed, iteration, subpath, path); draw j of a
 * stream = high 32 bits of mix(key + (j+1)*golden).  SplitMix64 finaliser. */
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
uint64_t cr_stream_key(uint32_t seed, uint32_t iteration, uint32_t subpath, uint32_t path) {
    uint64_t a = mix64(((uint64_t)seed << 32) | iteration);
    uint64_t b = mix64((((uint64_t)subpath << 32) | path) + 0x9E3779B97F4A7C15ull);
    return mix64(a ^ b);
}
uint32_t cr_stream_u32(uint64_t key, uint32_t index) {
    return (uint32_t)(mix64(key + (uint64_t)(index + 1u) * 0x9E3779B97F4A7C15ull) >> 32);
}

typedef struct {
    int mode;
    mt_state* mt;
    uint64_t key;
    uint32_t ctr;
} rng_t;

static inline uint32_t rng_u32(rng_t* r) {
    if (r->mode == CR_RNG_MT) return mt_next(r->mt);
    return cr_stream_u32(r->key, r->ctr++);
}
/* rng.cpp:18-22 */
static inline float rng_f(rng_t* r) { return (float)(rng_u32(r) & 0xffffffu) / (float)(1 << 24); }
/* rng.cpp:64-70: x, y, z drawn in order */
static inline v3 rng_v3(rng_t* r) {
    float a = rng_f(r);
    float b = rng_f(r);
    float c = rng_f(r);
    return mk(a, b, c);
}

/* ------------------------------------------------------------------------- */
/* transform.cpp (host-side camera matrices)                                  */
/* ------------------------------------------------------------------------- */
typedef struct { float m[4][4]; } m44;

static m44 m_ident(void) {
    m44 r;
    memset(&r, 0, sizeof r);
    r.m[0][0] = r.m[1][1] = r.m[2][2] = r.m[3][3] = 1.f;
    return r;
}
static m44 m_rows(const float* v) { m44 r; memcpy(r.m, v, sizeof r.m); return r; }

/* transform.cpp:24-35: sum of four products, left to right */
static m44 m_mul(const m44* a, const m44* b) {
    m44 r;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            r.m[i][j] = a->m[i][0] * b->m[0][j] + a->m[i][1] * b->m[1][j] +
                        a->m[i][2] * b->m[2][j] + a->m[i][3] * b->m[3][j];
    return r;
}

/* transform.cpp:46-176: cofactor (adjugate) inverse.  Each cofactor is a signed
 * sum of six triple products evaluated left to right; the table lists
 * (sign, a, b, c) per term in the reference's term order, for inv[0..15]. */
static const signed char COF[16][6][4] = {
    {{1,5,10,15},{-1,5,11,14},{-1,9,6,15},{1,9,7,14},{1,13,6,11},{-1,13,7,10}},
    {{-1,1,10,15},{1,1,11,14},{1,9,2,15},{-1,9,3,14},{-1,13,2,11},{1,13,3,10}},
    {{1,1,6,15},{-1,1,7,14},{-1,5,2,15},{1,5,3,14},{1,13,2,7},{-1,13,3,6}},
    {{-1,1,6,11},{1,1,7,10},{1,5,2,11},{-1,5,3,10},{-1,9,2,7},{1,9,3,6}},
    {{-1,4,10,15},{1,4,11,14},{1,8,6,15},{-1,8,7,14},{-1,12,6,11},{1,12,7,10}},
    {{1,0,10,15},{-1,0,11,14},{-1,8,2,15},{1,8,3,14},{1,12,2,11},{-1,12,3,10}},
    {{-1,0,6,15},{1,0,7,14},{1,4,2,15},{-1,4,3,14},{-1,12,2,7},{1,12,3,6}},
    {{1,0,6,11},{-1,0,7,10},{-1,4,2,11},{1,4,3,10},{1,8,2,7},{-1,8,3,6}},
    {{1,4,9,15},{-1,4,11,13},{-1,8,5,15},{1,8,7,13},{1,12,5,11},{-1,12,7,9}},
    {{-1,0,9,15},{1,0,11,13},{1,8,1,15},{-1,8,3,13},{-1,12,1,11},{1,12,3,9}},
    {{1,0,5,15},{-1,0,7,13},{-1,4,1,15},{1,4,3,13},{1,12,1,7},{-1,12,3,5}},
    {{-1,0,5,11},{1,0,7,9},{1,4,1,11},{-1,4,3,9},{-1,8,1,7},{1,8,3,5}},
    {{-1,4,9,14},{1,4,10,13},{1,8,5,14},{-1,8,6,13},{-1,12,5,10},{1,12,6,9}},
    {{1,0,9,14},{-1,0,10,13},{-1,8,1,14},{1,8,2,13},{1,12,1,10},{-1,12,2,9}},
    {{-1,0,5,14},{1,0,6,13},{1,4,1,14},{-1,4,2,13},{-1,12,1,6},{1,12,2,5}},
    {{1,0,5,10},{-1,0,6,9},{-1,4,1,10},{1,4,2,9},{1,8,1,6},{-1,8,2,5}},
};
/* COF rows above are ordered inv[0],inv[1],inv[2],inv[3],inv[4],... */

static m44 m_inv(const m44* a) {
    const float* m = &a->m[0][0];
    float inv[16];
    for (int k = 0; k < 16; k++) {
        float acc = 0.f;
        for (int t = 0; t < 6; t++) {
            const signed char* e = COF[k][t];
            float p = (e[0] > 0 ? m[e[1]] : -m[e[1]]) * m[e[2]] * m[e[3]];
            acc = (t == 0) ? p : acc + p;
        }
        inv[k] = acc;
    }
    float det = m[0] * inv[0] + m[1] * inv[4] + m[2] * inv[8] + m[3] * inv[12];
    det = 1.f / det;
    m44 r;
    for (int i = 0; i < 16; i++) (&r.m[0][0])[i] = inv[i] * det;
    return r;
}

typedef struct { m44 m, mi; } xform;

static xform x_make(m44 m, m44 mi) { xform t = {m, mi}; return t; }
static xform x_full(m44 m) { return x_make(m, m_inv(&m)); }
static xform x_mul(const xform* a, const xform* b) { /* transform.cpp:222-227 */
    return x_make(m_mul(&a->m, &b->m), m_mul(&b->mi, &a->mi));
}
static xform x_inverse(const xform* t) { return x_make(t->mi, t->m); }
static xform x_translate(v3 d) { /* transform.cpp:279-290 */
    float a[16] = {1, 0, 0, d.x, 0, 1, 0, d.y, 0, 0, 1, d.z, 0, 0, 0, 1};
    float b[16] = {1, 0, 0, -d.x, 0, 1, 0, -d.y, 0, 0, 1, -d.z, 0, 0, 0, 1};
    return x_make(m_rows(a), m_rows(b));
}
static xform x_scale(float x, float y, float z) { /* transform.cpp:292-303 */
    float a[16] = {x, 0, 0, 0, 0, y, 0, 0, 0, 0, z, 0, 0, 0, 0, 1};
    float b[16] = {1.0f / x, 0, 0, 0, 0, 1.0f / y, 0, 0, 0, 0, 1.0f / z, 0, 0, 0, 0, 1};
    return x_make(m_rows(a), m_rows(b));
}
static xform x_lookat(v3 pos, v3 look, v3 up) { /* transform.cpp:353-370 */
    v3 dir = vnorm(vsub(look, pos));
    v3 u = vnorm(vcross(up, vneg(dir)));
    v3 left = vcross(u, dir);
    v3 p = mk(vdot(u, pos), vdot(left, pos), vdot(vneg(dir), pos));
    m44 w = m_ident();
    w.m[0][0] = u.x; w.m[0][1] = u.y; w.m[0][2] = u.z; w.m[0][3] = -p.x;
    w.m[1][0] = left.x; w.m[1][1] = left.y; w.m[1][2] = left.z; w.m[1][3] = -p.y;
    v3 nd = vneg(dir);
    w.m[2][0] = nd.x; w.m[2][1] = nd.y; w.m[2][2] = nd.z; w.m[2][3] = -p.z;
    return x_full(w);
}
static xform x_perspective(float fov, float zn, float zf) { /* transform.cpp:379-387 */
    float a[16] = {1, 0, 0, 0, 0, -1, 0, 0, 0, 0, (zn + zf) / (zf - zn), 2 * zf * zn / (zf - zn),
                   0, 0, -1, 0};
    float inv_tan = 1.0f / tanf(fov / 360.0f * R_PI);
    xform s = x_scale(inv_tan, inv_tan, 1);
    xform p = x_full(m_rows(a));
    return x_mul(&s, &p);
}
/* transform.h:122-137 */
static v3 x_point(const m44* m, v3 p) {
    float xp = m->m[0][0] * p.x + m->m[0][1] * p.y + m->m[0][2] * p.z + m->m[0][3];
    float yp = m->m[1][0] * p.x + m->m[1][1] * p.y + m->m[1][2] * p.z + m->m[1][3];
    float zp = m->m[2][0] * p.x + m->m[2][1] * p.y + m->m[2][2] * p.z + m->m[2][3];
    float wp = m->m[3][0] * p.x + m->m[3][1] * p.y + m->m[3][2] * p.z + m->m[3][3];
    if (cmpf(wp - 1.0f) == 0) return mk(xp, yp, zp);
    return vdiv(mk(xp, yp, zp), wp);
}

/* ------------------------------------------------------------------------- */
/* camera.cpp                                                                 */
/* ------------------------------------------------------------------------- */
typedef struct {
    v3 pos, fwd, up;
    float xres, yres, fov, plane_dist;
    m44 w2r, r2w;
} camera_t;

static void cam_setup(camera_t* c, v3 pos, v3 fwd, v3 up, float xres, float yres, float fov) {
    c->pos = pos;                     /* camera.cpp:3-29 */
    c->fwd = vnorm(fwd);
    c->up = vnorm(up);
    c->xres = xres;
    c->yres = yres;
    c->fov = fov;
    xform w2c = x_lookat(c->pos, vadd(c->pos, c->fwd), c->up);
    xform persp = x_perspective(fov, 0.1f, 10000.f);
    xform w2n = x_mul(&persp, &w2c);
    xform n2w = x_inverse(&w2n);
    xform s1 = x_scale(xres * 0.5f, yres * 0.5f, 0);
    xform t1 = x_translate(mk(1.0f, 1.0f, 0.0f));
    xform a = x_mul(&s1, &t1);
    xform w2r = x_mul(&a, &w2n);
    xform t2 = x_translate(mk(-1.0f, -1.0f, 0.0f));
    xform s2 = x_scale(2.0f / xres, 2.0f / yres, 0);
    xform b = x_mul(&n2w, &t2);
    xform r2w = x_mul(&b, &s2);
    c->w2r = w2r.m;
    c->r2w = r2w.m;
    float th = tanf(fov * R_PI / 360.0f);
    c->plane_dist = xres / (2.0f * th);
}
static int cam_check(const camera_t* c, float x, float y) { /* camera.cpp:31-35 */
    return cmpf(x) >= 0 && cmpf(y) >= 0 && cmpf(x - c->xres) < 0 && cmpf(y - c->yres) < 0;
}

/* ------------------------------------------------------------------------- */
/* geometry: ray.h, AABB.cpp, triangle.cpp, sphere.cpp                         */
/* ------------------------------------------------------------------------- */
typedef struct { v3 o, d; float tmin, tmax; } ray_t;
/* ray.h:14-21: the constructor normalises the direction */
static inline ray_t mkray(v3 o, v3 d) { ray_t r = {o, vnorm(d), 0.f, R_INF}; return r; }
static inline v3 ray_at(const ray_t* r, float t) { return vadd(r->o, vscale(r->d, t)); }

typedef struct { v3 l, r; } aabb;

static aabb box_make(v3 l, v3 r) { /* AABB.h:13-21 (extend) */
    aabb b = {l, r};
    if (cmpf(b.l.x - b.r.x) == 0) b.r.x += 10 * R_EPS;
    if (cmpf(b.l.y - b.r.y) == 0) b.r.y += 10 * R_EPS;
    if (cmpf(b.l.z - b.r.z) == 0) b.r.z += 10 * R_EPS;
    return b;
}

static int box_hit(const aabb* b, const ray_t* ray, float* t1, float* t2) { /* AABB.cpp:9-32 */
    float tmin = -R_INF, tmax = R_INF;
    for (int i = 0; i < 3; i++) {
        float inv = 1.f / vget(ray->d, i);
        float tn = (vget(b->l, i) - vget(ray->o, i)) * inv;
        float tf = (vget(b->r, i) - vget(ray->o, i)) * inv;
        if (tn > tf) { float t = tn; tn = tf; tf = t; }
        tmin = fmaxs(tmin, tn);
        tmax = fmins(tmax, tf);
        if (tmin > tmax) return 0;
    }
    *t1 = tmin;
    *t2 = tmax;
    return 1;
}

typedef struct { float t; v3 p, n; int inside, matId; } hit_t;

enum { PRIM_TRI = 0, PRIM_SPH = 1 };
typedef struct {
    int type, matId;
    v3 p0, p1, p2;      /* triangle */
    v3 c; float rad;    /* sphere   */
    aabb box;
} prim_t;

static int tri_hit(const prim_t* g, const ray_t* ray, hit_t* h) { /* triangle.cpp:22-87 */
    float A = g->p0.x - g->p1.x, B = g->p0.y - g->p1.y, C = g->p0.z - g->p1.z;
    float D = g->p0.x - g->p2.x, E = g->p0.y - g->p2.y, F = g->p0.z - g->p2.z;
    float G = ray->d.x, H = ray->d.y, I = ray->d.z;
    float J = g->p0.x - ray->o.x, K = g->p0.y - ray->o.y, L = g->p0.z - ray->o.z;
    float EIHF = E * I - H * F, GFDI = G * F - D * I, DHEG = D * H - E * G;
    float denom = A * EIHF + B * GFDI + C * DHEG;
    float beta = (J * EIHF + K * GFDI + L * DHEG) / denom;
    if (cmpf(beta) < 0 || beta > 1.f) { h->t = R_INF; return 0; }
    float AKJB = A * K - J * B, JCAL = J * C - A * L, BLKC = B * L - K * C;
    float gamma = (I * AKJB + H * JCAL + G * BLKC) / denom;
    if (cmpf(gamma) < 0 || beta + gamma > 1.f) { h->t = R_INF; return 0; }
    h->t = -(F * AKJB + E * JCAL + D * BLKC) / denom;
    if (cmpf(h->t) <= 0) { h->t = R_INF; return 0; }
    if (h->t < ray->tmin || h->t > ray->tmax) { h->t = R_INF; return 0; }
    h->p = ray_at(ray, h->t);
    h->n = vnorm(vcross(vsub(g->p1, g->p0), vsub(g->p2, g->p0)));
    h->inside = (vdot(ray->d, h->n) < R_EPS) ? 0 : 1;
    h->matId = g->matId;
    return 1;
}

static int sph_hit(const prim_t* g, const ray_t* ray, hit_t* h) { /* sphere.cpp:17-78 */
    float a, b;
    if (!box_hit(&g->box, ray, &a, &b)) { h->t = R_INF; return 0; }
    v3 oc = vsub(g->c, ray->o);
    int inside = 0;
    if (vlen(oc) < g->rad + R_EPS) inside = 1;
    float l_oc = vdot(oc, oc);
    float t_ca = vdot(oc, ray->d);
    if (cmpf(t_ca) < 0 && !inside) { h->t = R_INF; return 0; }
    float t_hc = g->rad * g->rad - l_oc + t_ca * t_ca;
    if (cmpf(t_hc) <= 0) { h->t = R_INF; return 0; }
    float d = sqrtf(t_hc);
    float t1 = t_ca - d, t2 = t_ca + d;
    if (cmpf(t2) <= 0) { h->t = R_INF; return 0; }
    if (cmpf(t1) <= 0) { h->t = t2; h->inside = 1; }
    else { h->t = t1; h->inside = 0; }
    if (h->t < ray->tmin || h->t > ray->tmax) { h->t = R_INF; return 0; }
    h->p = ray_at(ray, h->t);
    h->n = vnorm(vsub(h->p, g->c));
    h->matId = g->matId;
    return 1;
}

static inline int prim_hit(const prim_t* g, const ray_t* r, hit_t* h) {
    return g->type == PRIM_TRI ? tri_hit(g, r, h) : sph_hit(g, r, h);
}

/* ------------------------------------------------------------------------- */
/* light.h / light.cpp (AreaLight), frame.cpp, sampler.cpp                    */
/* ------------------------------------------------------------------------- */
typedef struct { v3 x, y, z; } frame_t;

static frame_t frame_from_z(v3 z0) { /* frame.cpp:3-11 */
    frame_t f;
    f.z = vnorm(z0);
    v3 tx = (fabsf(f.z.x) > 0.99f) ? mk(0.0f, 1.0f, 0.0f) : mk(1.0f, 0.0f, 0.0f);
    f.y = vnorm(vcross(f.z, tx));
    f.x = vcross(f.y, f.z);
    return f;
}
static inline v3 to_world(const frame_t* f, v3 l) { /* frame.cpp:13-16 */
    return vadd(vadd(vscale(f->x, l.x), vscale(f->y, l.y)), vscale(f->z, l.z));
}
static inline v3 to_local(const frame_t* f, v3 w) { /* frame.cpp:18-21 */
    return mk(vdot(w, f->x), vdot(w, f->y), vdot(w, f->z));
}

static v3 sample_triangle(v3 s, v3 v1, v3 v2, v3 v3_) { /* sampler.cpp:3-13 */
    v3 p1 = vsub(v2, v1), p2 = vsub(v3_, v1);
    float u1 = sqrtf(s.x);
    float beta = 1.f - u1;
    float gamma = s.y * u1;
    return vadd(vadd(v1, vscale(p1, beta)), vscale(p2, gamma));
}
static v3 sample_rect_strat(v3 s, v3 v0, v3 v1, v3 v2, int cur, int tot) { /* sampler.cpp:28-42 */
    v3 p1 = vsub(v1, v0), p2 = vsub(v2, v0);
    int len = (int)sqrt((double)tot);
    int row = cur / len, col = cur % len;
    float a = (s.x + (float)row) / (float)len;
    float b = (s.y + (float)col) / (float)len;
    return vadd(vadd(v0, vscale(p1, a)), vscale(p2, b));
}
static v3 sample_cos_hemi(v3 s, float* pdf) { /* sampler.cpp:95-108 */
    float u1 = 2.f * R_PI * s.x;
    float u2 = sqrtf(1.f - s.y);
    v3 r = mk(cosf(u1) * u2, sinf(u1) * u2, sqrtf(s.y));
    if (pdf) *pdf = r.z * R_INV_PI;
    return vnorm(r);
}
static float cos_hemi_pdf(v3 n, v3 d) { return clampv(vdot(n, d), 0.f, 1.f) * R_INV_PI; } /* :110-113 */
static v3 sample_pow_cos_hemi(v3 s, float power, float* pdf) { /* sampler.cpp:115-129 */
    float u1 = 2.f * R_PI * s.x;
    float u2 = powf(s.y, 1.f / (power + 1.f));
    float u3 = sqrtf(1.f - u2 * u2);
    if (pdf) *pdf = (power + 1.f) * powf(u2, power) * (0.5f * R_INV_PI);
    v3 r = mk(cosf(u1) * u3, sinf(u1) * u3, u2);
    return vnorm(r);
}
static float pow_cos_hemi_pdf(v3 n, v3 d, float power) { /* sampler.cpp:131-136 */
    float c = clampv(vdot(n, d), 0.f, 1.f);
    return (power + 1.f) * powf(c, power) * (0.5f * R_INV_PI);
}

typedef struct {
    v3 p0, d1, d2;
    frame_t fr;
    c3 le;
    float inv_area;
} light_t;

static light_t light_make(v3 p0, v3 p1, v3 p2, c3 le) { /* light.h:90-103 */
    light_t l;
    l.le = le;
    l.p0 = p0;
    l.d1 = vsub(p1, p0);
    l.d2 = vsub(p2, p0);
    v3 n = vcross(l.d1, l.d2);
    float len = vlen(n);
    l.inv_area = 2.f / len;
    n = vnorm(n);
    l.fr = frame_from_z(n);
    return l;
}

typedef struct { v3 center; float radius, inv_r2; } sphere_t;

static c3 light_illum(const light_t* l, v3 pos, v3 r3, v3* dtl, float* dist, float* dpdf,
                      float* epdf, float* cal) { /* light.cpp:4-38 */
    if (epdf) *epdf = 0;
    if (cal) *cal = 0;
    v3 lp = sample_triangle(r3, l->p0, vadd(l->p0, l->d1), vadd(l->p0, l->d2));
    *dtl = vsub(lp, pos);
    *dist = vlen(*dtl);
    *dtl = vdiv(*dtl, *dist);
    float cn = vdot(l->fr.z, vneg(*dtl));
    if (cmpf(cn) <= 0) {
        *dpdf = 0;
        if (epdf) *epdf = 0;
        return C0;
    }
    *dpdf = l->inv_area * ((*dist) * (*dist)) / cn;
    if (cal) *cal = cn;
    if (epdf) *epdf = l->inv_area * cn * R_INV_PI;
    return l->le;
}
static c3 light_emit(const light_t* l, v3 dr, v3 pr, v3* pos, v3* dir, float* epdf,
                     float* dpa, float* cal) { /* light.cpp:40-67 */
    if (dpa) *dpa = 0;
    if (cal) *cal = 0;
    *pos = sample_triangle(pr, l->p0, vadd(l->p0, l->d1), vadd(l->p0, l->d2));
    v3 ld = sample_cos_hemi(dr, epdf);
    *epdf *= l->inv_area;
    ld.z = fmaxs(ld.z, R_EPS);
    *dir = to_world(&l->fr, ld);
    if (dpa) *dpa = l->inv_area;
    if (cal) *cal = ld.z;
    return cscale(l->le, ld.z);
}
static c3 light_radiance(const light_t* l, v3 rd, float* dpa, float* epdf) { /* light.cpp:69-100 */
    if (dpa) *dpa = 0;
    if (epdf) *epdf = 0;
    float cn = clampv(vdot(l->fr.z, vneg(rd)), 0.f, 1.f);
    if (cmpf(cn) == 0) {
        if (dpa) *dpa = 0;
        if (epdf) *epdf = 0;
        return C0;
    }
    if (dpa) *dpa = l->inv_area;
    if (epdf) {
        *epdf = cos_hemi_pdf(l->fr.z, vneg(rd));
        *epdf *= l->inv_area;
    }
    return l->le;
}

/* ------------------------------------------------------------------------- */
/* material.h, fresnel.cpp, bsdf.h / bsdf.cpp                                 */
/* ------------------------------------------------------------------------- */
typedef struct { c3 diffuse, phong, specular; float phong_exp, index; } mat_t;

static float fresnel(float cosI, float index) { /* fresnel.cpp:3-29 */
    if (cmpf(index) < 0) return 1.0f;
    float eta;
    if (cmpf(cosI) < 0) { cosI = -cosI; eta = index; }
    else eta = 1.0f / index;
    float sinT2 = (eta * eta) * (1.0f - cosI * cosI);
    float cosT = sqrtf(fmaxs(0.0f, 1.0f - sinT2));
    float term1 = eta * cosT;
    float par = (cosI - term1) / (cosI + term1);
    float term2 = eta * cosI;
    float perp = (term2 - cosT) / (term2 + cosT);
    return 0.5f * (par * par + perp * perp);
}

enum { T_REFL = 1, T_TRANS = 2, T_DIFF = 4, T_GLOSSY = 8, T_SPEC = 3 };

typedef struct {
    int matId;
    frame_t fr;
    v3 wi;          /* wiLocal */
    int delta;
    float cont, fres;
    float pd, pg, pr, pt;  /* componentProb */
} bsdf_t;

/* bsdf.h:66-89.  For emitter hits (matId < 0) the reference leaves
 * componentProb / continueProb / isDelta uninitialised; no film value depends
 * on them (f / sample return 0 first, bsdf.cpp:118-119,286-287).  Pinned here
 * as: probabilities 0, continueProb 0, isDelta false. */
static void bsdf_init(bsdf_t* b, v3 wi, const hit_t* h, const mat_t* mats) {
    b->matId = 0;
    b->fr = frame_from_z(h->n);
    b->wi = vnorm(to_local(&b->fr, wi));
    if (cmpf(b->wi.z) == 0) return;
    b->pd = b->pg = b->pr = b->pt = 0.f;
    b->cont = 0.f;
    b->fres = 1.f;
    b->delta = 0;
    if (h->matId > 0) {
        const mat_t* m = &mats[h->matId];
        /* bsdf.cpp:24-55 */
        b->fres = fresnel(b->wi.z, m->index);
        float pd = clum(m->diffuse);
        float pg = clum(m->phong);
        float pr = b->fres * clum(m->specular);
        float pt = (1.f - b->fres) * 1.0f;
        float tot = pd + pg + pr + pt;
        if (cmpf(tot) <= 0) {
            b->pd = b->pg = b->pr = b->pt = b->cont = 0.f;
        } else {
            b->pd = pd / tot;
            b->pg = pg / tot;
            b->pr = pr / tot;
            b->pt = pt / tot;
            c3 refl = cadd(cadd(m->diffuse, m->phong), cscale(m->specular, b->fres));
            b->cont = cmaxc(refl) + (1.f - b->fres);
            b->cont = clampv(b->cont, 0.f, 1.f);
        }
        b->delta = (cmpf(b->pd) == 0 && cmpf(b->pg) == 0);
    }
    b->matId = h->matId;
}

static c3 calc_diffuse(const bsdf_t* b, const mat_t* m, v3 wo, float* dp, float* rp) { /* :57-72 */
    if (cmpf(b->pd) == 0) return C0;
    if (cmpf(b->wi.z) <= 0 || cmpf(wo.z) <= 0) return C0;
    if (dp) *dp += b->pd * clampv(wo.z * R_INV_PI, 0.0f, 1.0f);
    if (rp) *rp += b->pd * clampv(b->wi.z * R_INV_PI, 0.0f, 1.0f);
    return cscale(m->diffuse, R_INV_PI);
}
static c3 calc_glossy(const bsdf_t* b, const mat_t* m, v3 wo, float* dp, float* rp) { /* :74-100 */
    if (cmpf(b->pg) == 0) return C0;
    if (cmpf(b->wi.z) <= 0 || cmpf(wo.z) <= 0) return C0;
    v3 refl = mk(-b->wi.x, -b->wi.y, b->wi.z);
    float c = vdot(refl, wo);
    if (cmpf(c) == 0) return C0;
    float pw = b->pg * pow_cos_hemi_pdf(refl, wo, m->phong_exp);
    if (dp) *dp += pw;
    if (rp) *rp += pw;
    c3 rho = cscale(cscale(cscale(m->phong, m->phong_exp + 2.f), 0.5f), R_INV_PI);
    return cscale(rho, powf(c, m->phong_exp));
}
static c3 bsdf_f(const bsdf_t* b, const mat_t* mats, v3 woW, float* cosWo, float* dp,
                 float* rp) { /* bsdf.cpp:102-126 */
    c3 res = C0;
    if (dp) *dp = 0.f;
    if (rp) *rp = 0.f;
    v3 wo = to_local(&b->fr, woW);
    if (cmpf(wo.z * b->wi.z) < 0) return res;
    *cosWo = fabsf(wo.z);
    if (b->matId < 0) return res;
    const mat_t* m = &mats[b->matId];
    res = cadd(res, calc_diffuse(b, m, wo, dp, rp));
    res = cadd(res, calc_glossy(b, m, wo, dp, rp));
    return res;
}
static void pdf_diffuse(const bsdf_t* b, v3 wo, float* dp, float* rp) { /* :128-141 */
    if (cmpf(b->pd) == 0) return;
    if (dp) *dp += b->pd * clampv(wo.z, 0.f, 1.f) * R_INV_PI;
    if (rp) *rp += b->pd * clampv(b->wi.z, 0.f, 1.f) * R_INV_PI;
}
static void pdf_glossy(const bsdf_t* b, const mat_t* m, v3 wo, float* dp, float* rp) { /* :143-163 */
    if (cmpf(b->pg) == 0) return;
    v3 refl = mk(-b->wi.x, -b->wi.y, b->wi.z);
    float c = vdot(refl, wo);
    if (cmpf(c) == 0) return;
    float pw = b->pg * pow_cos_hemi_pdf(refl, wo, m->phong_exp);
    if (dp) *dp += pw;
    if (rp) *rp += pw;
}
static float bsdf_pdf(const bsdf_t* b, const mat_t* mats, v3 woW, int rev) { /* :165-181 */
    v3 wo = to_local(&b->fr, woW);
    if (cmpf(wo.z * b->wi.z) < 0) return 0;
    const mat_t* m = &mats[b->matId];
    float dp = 0, rp = 0;
    pdf_diffuse(b, wo, &dp, &rp);
    pdf_glossy(b, m, wo, &dp, &rp);
    return rev ? rp : dp;
}
static c3 bsdf_sample(const bsdf_t* b, const mat_t* mats, v3 r3, v3* woW, float* pdf,
                      float* cosWo, int* type) { /* bsdf.cpp:183-334 */
    int comp;
    if (r3.z < b->pd) comp = T_DIFF;
    else if (r3.z < b->pd + b->pg) comp = T_GLOSSY;
    else if (r3.z < b->pd + b->pg + b->pr) comp = T_REFL;
    else comp = T_TRANS;
    if (type) *type = comp;
    if (b->matId < 0) return C0;
    const mat_t* m = &mats[b->matId];
    *pdf = 0;
    c3 res = C0;
    v3 wo = mk(0, 0, 0);
    if (comp == T_DIFF) {
        if (cmpf(b->wi.z) <= 0) return C0;                       /* :186-187 */
        float pw;
        wo = sample_cos_hemi(r3, &pw);
        *pdf += pw * b->pd;
        res = cadd(res, cscale(m->diffuse, R_INV_PI));
        if (cblack(res)) return C0;
        res = cadd(res, calc_glossy(b, m, wo, pdf, NULL));
    } else if (comp == T_GLOSSY) {
        wo = sample_pow_cos_hemi(r3, m->phong_exp, NULL);        /* :196-215 */
        v3 refl = mk(-b->wi.x, -b->wi.y, b->wi.z);
        frame_t f = frame_from_z(refl);
        wo = to_world(&f, wo);
        float c = vdot(refl, wo);
        c3 g = C0;
        if (cmpf(c) > 0) {
            pdf_glossy(b, m, wo, pdf, NULL);
            c3 rho = cscale(cscale(cscale(m->phong, m->phong_exp + 2.f), 0.5f), R_INV_PI);
            g = cscale(rho, powf(c, m->phong_exp));
        }
        res = cadd(res, g);
        if (cblack(res)) return C0;
        res = cadd(res, calc_diffuse(b, m, wo, pdf, NULL));
    } else if (comp == T_REFL) {
        wo = mk(-b->wi.x, -b->wi.y, b->wi.z);                    /* :217-223 */
        *pdf += b->pr;
        res = cadd(res, cdivs(cscale(m->specular, b->fres), fabsf(wo.z)));
        if (cblack(res)) return C0;
    } else {
        c3 t = C0;                                               /* :225-266 */
        if (!(cmpf(m->index) < 0)) {
            float cosI = b->wi.z, cosT, eta;
            if (cmpf(cosI) < 0) { eta = m->index; cosI = -cosI; cosT = 1.f; }
            else { eta = 1.f / m->index; cosT = -1.f; }
            float sinI2 = 1.f - cosI * cosI;
            float sinT2 = (eta * eta) * sinI2;
            if (sinT2 < 1.f) {
                cosT *= sqrtf(clampv(1.f - sinT2, 0.f, 1.f));
                wo = vnorm(mk(-eta * b->wi.x, -eta * b->wi.y, cosT));
                *pdf += b->pt;
                float tc = 1.f - b->fres;
                float v = tc / fabsf(cosT);
                t = mkc(v, v, v);
            } else {
                *pdf += 0.f;
            }
        }
        res = cadd(res, t);
        if (cblack(res)) return C0;
    }
    *cosWo = fabsf(wo.z);
    if (cmpf(*cosWo) == 0) return C0;
    *woW = to_world(&b->fr, wo);
    return res;
}

/* ------------------------------------------------------------------------- */
/* Scene: loader (scene.cpp:259-467 + tiny_obj_loader.cpp) and KD tree        */
/* ------------------------------------------------------------------------- */
typedef struct {
    int axis;          /* -1 leaf */
    float split;
    int left, right;   /* node indices */
    int first, count;  /* leaf: range in refs[] */
} node_t;

struct cr_scene {
    prim_t* prims; int nprims, cap_prims;
    light_t* lights; int nlights, cap_lights;
    mat_t* mats; int nmats, cap_mats;
    camera_t cam;
    sphere_t ssph;
    float tot_area;
    int dep_max;
    aabb root_box;
    node_t* nodes; int nnodes, cap_nodes;
    int* refs; int64_t nrefs, cap_refs;
};

#define GROW(ptr, n, cap, T) do { if ((n) >= (cap)) { (cap) = (cap) ? 2 * (cap) : 64; \
    (ptr) = (T*)realloc((ptr), (size_t)(cap) * sizeof(T)); } } while (0)

static void add_prim(cr_scene* s, prim_t p) {
    GROW(s->prims, s->nprims, s->cap_prims, prim_t);
    s->prims[s->nprims++] = p;
    /* Scene::addGeometry (scene.cpp:5-9): totArea += getArea() */
    if (p.type == PRIM_TRI) {
        v3 n = vcross(vsub(p.p1, p.p0), vsub(p.p2, p.p0));
        s->tot_area += 0.5f * vlen(n);
    } else {
        s->tot_area += 4 * R_PI * (p.rad * p.rad);
    }
}

static prim_t mk_tri(v3 a, v3 b, v3 c, int matId) { /* triangle.h:14-31 (setBox) */
    prim_t p;
    memset(&p, 0, sizeof p);
    p.type = PRIM_TRI; p.matId = matId; p.p0 = a; p.p1 = b; p.p2 = c;
    p.box = box_make(mk(fmins(a.x, fmins(b.x, c.x)), fmins(a.y, fmins(b.y, c.y)), fmins(a.z, fmins(b.z, c.z))),
                     mk(fmaxs(a.x, fmaxs(b.x, c.x)), fmaxs(a.y, fmaxs(b.y, c.y)), fmaxs(a.z, fmaxs(b.z, c.z))));
    return p;
}
static prim_t mk_sph(v3 c, float r, int matId) { /* sphere.h:16-21 */
    prim_t p;
    memset(&p, 0, sizeof p);
    p.type = PRIM_SPH; p.matId = matId; p.c = c; p.rad = r;
    p.box = box_make(mk(c.x - r, c.y - r, c.z - r), mk(c.x + r, c.y + r, c.z + r));
    return p;
}

/* ---- OBJ: tinyobjloader semantics (tiny_obj_loader.cpp:461-661) ---------- */
typedef struct { float* v; int nv, cap_v; } objbuf;

typedef void (*face_cb)(void* ctx, int shape_face, const char* shape_name, v3 a, v3 b, v3 c);

static int fix_index(int idx, int n) { return idx > 0 ? idx - 1 : (idx == 0 ? 0 : n + idx); }

/* Reads faces of one .obj; triangles are emitted per shape in file order as a
 * triangle fan (i0, f[k-1], f[k]).  Missing file => 0 shapes (LoadObj returns
 * after shapes.clear()).  Returns -1 on an out-of-range vertex index (the
 * reference asserts). */
static int load_obj(const char* path, face_cb cb, void* ctx) {
    FILE* f = fopen(path, "r");
    if (!f) return 0;
    float* v = NULL; int nv = 0, capv = 0;     /* floats */
    int* faces = NULL; int nf = 0, capf = 0;   /* flattened: count, idx... per face */
    char name[4096] = "", pending_name[4096] = "";
    char line[8192];
    int rc = 0;
    /* faceGroup flush (exportFaceGroupToShape) */
#define FLUSH() do { if (nf > 0) { int pos = 0, fi = 0; \
        while (pos < nf) { int cnt = faces[pos]; int* ix = faces + pos + 1; \
            for (int k = 2; k < cnt; k++) { int i0 = ix[0], i1 = ix[k-1], i2 = ix[k]; \
                if (i0 < 0 || i1 < 0 || i2 < 0 || 3*i0+2 >= nv || 3*i1+2 >= nv || 3*i2+2 >= nv) { rc = -1; } else { \
                cb(ctx, fi, pending_name, mk(v[3*i0], v[3*i0+1], v[3*i0+2]), mk(v[3*i1], v[3*i1+1], v[3*i1+2]), \
                   mk(v[3*i2], v[3*i2+1], v[3*i2+2])); } fi++; } \
            pos += cnt + 1; } } nf = 0; } while (0)
    while (fgets(line, sizeof line, f)) {
        size_t L = strlen(line);
        if (L > 0 && line[L - 1] == '\n') line[--L] = 0;
        if (L == 0) continue;
        const char* t = line + strspn(line, " \t");
        if (t[0] == 0 || t[0] == '#') continue;
        if (t[0] == 'v' && (t[1] == ' ' || t[1] == '\t')) {
            t += 2;
            for (int k = 0; k < 3; k++) {
                t += strspn(t, " \t");
                float x = (float)atof(t);
                t += strcspn(t, " \t\r");
                if (nv + 1 > capv) { capv = capv ? 2 * capv : 1024; v = (float*)realloc(v, capv * sizeof(float)); }
                v[nv++] = x;
            }
            continue;
        }
        if (t[0] == 'f' && (t[1] == ' ' || t[1] == '\t')) {
            t += 2;
            t += strspn(t, " \t");
            int start = nf;
            if (nf + 1 > capf) { capf = capf ? 2 * capf : 1024; faces = (int*)realloc(faces, capf * sizeof(int)); }
            faces[nf++] = 0;
            while (!(t[0] == '\r' || t[0] == '\n' || t[0] == 0)) {
                int vi = fix_index(atoi(t), nv / 3);
                t += strcspn(t, "/ \t\r");
                if (t[0] == '/') {  /* skip vt / vn parts (parseTriple) */
                    t++;
                    if (t[0] == '/') { t++; t += strcspn(t, "/ \t\r"); }
                    else {
                        t += strcspn(t, "/ \t\r");
                        if (t[0] == '/') { t++; t += strcspn(t, "/ \t\r"); }
                    }
                }
                if (nf + 1 > capf) { capf = 2 * capf; faces = (int*)realloc(faces, capf * sizeof(int)); }
                faces[nf++] = vi;
                faces[start]++;
                t += strspn(t, " \t\r");
            }
            continue;
        }
        if (t[0] == 'g' && (t[1] == ' ' || t[1] == '\t')) {
            FLUSH();
            /* names[0] is "g"; the shape name is names[1] (parseString, :582-599) */
            const char* q = t + 1;
            q += strspn(q, " \t\r");
            size_t e = strcspn(q, " \t\r");
            if (q[0] == 0) pending_name[0] = 0;
            else { memcpy(pending_name, q, e); pending_name[e] = 0; }
            continue;
        }
        if (t[0] == 'o' && (t[1] == ' ' || t[1] == '\t')) {
            FLUSH();
            if (sscanf(t + 2, "%4095s", name) != 1) name[0] = 0;
            strcpy(pending_name, name);
            continue;
        }
    }
    FLUSH();
#undef FLUSH
    fclose(f);
    free(v);
    free(faces);
    return rc;
}

typedef struct { cr_scene* s; int matId; } obj_ctx;
static void obj_face(void* vctx, int fi, const char* shape, v3 a, v3 b, v3 c) {
    obj_ctx* o = (obj_ctx*)vctx;
    (void)fi;
    if (strcmp(shape, "water") == 0) {  /* scene.cpp:360-368 */
        v3 n = vcross(vsub(b, a), vsub(c, a));
        if (n.y < R_EPS) { v3 t = c; c = a; a = t; }
    }
    add_prim(o->s, mk_tri(a, b, c, o->matId));
}
typedef struct { cr_scene* s; c3 le; } light_ctx;
static void light_face(void* vctx, int fi, const char* shape, v3 a, v3 b, v3 c) {
    light_ctx* o = (light_ctx*)vctx;
    (void)shape;
    GROW(o->s->lights, o->s->nlights, o->s->cap_lights, light_t);
    o->s->lights[o->s->nlights++] = light_make(a, b, c, o->le);  /* scene.cpp:421-428 */
    add_prim(o->s, mk_tri(a, b, c, -(fi + 1)));
}

/* ---- minimal XML DOM (elements + attributes; enough for .scene) ---------- */
typedef struct xel {
    char name[64];
    char* keys[16];
    char* vals[16];
    int nattr;
    struct xel* child[64];
    int nchild;
} xel;

static void xfree(xel* e) {
    if (!e) return;
    for (int i = 0; i < e->nattr; i++) { free(e->keys[i]); free(e->vals[i]); }
    for (int i = 0; i < e->nchild; i++) xfree(e->child[i]);
    free(e);
}
static char* xdecode(const char* s, size_t n) {
    char* o = (char*)malloc(n + 1);
    size_t j = 0;
    for (size_t i = 0; i < n; i++) {
        if (s[i] == '&') {
            static const char* ent[5] = {"&amp;", "&lt;", "&gt;", "&quot;", "&apos;"};
            static const char rep[5] = {'&', '<', '>', '"', '\''};
            int k;
            for (k = 0; k < 5; k++)
                if (strncmp(s + i, ent[k], strlen(ent[k])) == 0) break;
            if (k < 5) { o[j++] = rep[k]; i += strlen(ent[k]) - 1; continue; }
        }
        o[j++] = s[i];
    }
    o[j] = 0;
    return o;
}
static const char* xskip(const char* p) {
    for (;;) {
        while (*p && *p != '<') p++;
        if (!*p) return p;
        if (strncmp(p, "<!--", 4) == 0) { const char* e = strstr(p, "-->"); p = e ? e + 3 : p + strlen(p); continue; }
        if (p[1] == '?' || p[1] == '!') { const char* e = strchr(p, '>'); p = e ? e + 1 : p + strlen(p); continue; }
        return p;
    }
}
static xel* xparse(const char** pp) {
    const char* p = xskip(*pp);
    if (*p != '<' || p[1] == '/') { *pp = p; return NULL; }
    p++;
    xel* e = (xel*)calloc(1, sizeof(xel));
    size_t n = strcspn(p, " \t\r\n/>");
    if (n >= sizeof e->name) n = sizeof e->name - 1;
    memcpy(e->name, p, n);
    p += strcspn(p, " \t\r\n/>");
    for (;;) {
        p += strspn(p, " \t\r\n");
        if (*p == '/' && p[1] == '>') { *pp = p + 2; return e; }
        if (*p == '>') { p++; break; }
        if (!*p) { *pp = p; return e; }
        size_t kn = strcspn(p, " \t\r\n=/>");
        const char* k = p;
        p += kn;
        p += strspn(p, " \t\r\n");
        if (*p != '=') { p++; continue; }
        p++;
        p += strspn(p, " \t\r\n");
        char q = *p;
        if (q != '"' && q != '\'') continue;
        p++;
        const char* vs = p;
        while (*p && *p != q) p++;
        if (e->nattr < 16) {
            e->keys[e->nattr] = xdecode(k, kn);
            e->vals[e->nattr] = xdecode(vs, (size_t)(p - vs));
            e->nattr++;
        }
        if (*p) p++;
    }
    for (;;) {
        const char* q = xskip(p);
        if (!*q) { *pp = q; return e; }
        if (q[1] == '/') { const char* c = strchr(q, '>'); *pp = c ? c + 1 : q + strlen(q); return e; }
        xel* c = xparse(&q);
        p = q;
        if (c) { if (e->nchild < 64) e->child[e->nchild++] = c; else xfree(c); }
    }
}
static const char* xattr(const xel* e, const char* k) {
    if (!e) return NULL;
    for (int i = 0; i < e->nattr; i++) if (strcmp(e->keys[i], k) == 0) return e->vals[i];
    return NULL;
}
/* tinyxml.cpp:609-622: atof of the attribute, 0 if missing */
static double xd(const xel* e, const char* k) { const char* v = xattr(e, k); return v ? atof(v) : 0.0; }
static int xi(const xel* e, const char* k) { const char* v = xattr(e, k); return v ? atoi(v) : 0; }
static v3 xv3(const xel* e) { return mk((float)xd(e, "x"), (float)xd(e, "y"), (float)xd(e, "z")); }
static c3 xc3(const xel* e) { return mkc((float)xd(e, "r"), (float)xd(e, "g"), (float)xd(e, "b")); }
static const xel* xnth(const xel* e, int i) { return (e && i < e->nchild) ? e->child[i] : NULL; }

/* ---- KD tree: KDtreeAccel.cpp:12-307 ------------------------------------- */
typedef struct { float pos; int type; int index; } event_t;  /* End=0 Planar=1 Start=2 */

static int ev_cmp(const event_t* a, const event_t* b) { /* KDtreeAccel.cpp:3-10 */
    if (cmpf(a->pos - b->pos) != 0) return cmpf(a->pos - b->pos);
    return a->type - b->type;
}
/* qsort() of glibc 2.35 (the reference's platform) is a top-down merge sort
 * (msort.c: n1 = n/2, take from the left run while cmp <= 0).  The comparator
 * is EPS-tolerant and not transitive, so the exact merge order is part of the
 * tree; restated here rather than delegated to whatever libc is present. */
static void ev_msort(event_t* b, size_t n, event_t* tmp) {
    if (n <= 1) return;
    size_t n1 = n / 2, n2 = n - n1;
    event_t *b1 = b, *b2 = b + n1;
    ev_msort(b1, n1, tmp);
    ev_msort(b2, n2, tmp);
    event_t* t = tmp;
    while (n1 > 0 && n2 > 0) {
        if (ev_cmp(b1, b2) <= 0) { *t++ = *b1++; n1--; }
        else { *t++ = *b2++; n2--; }
    }
    if (n1 > 0) memcpy(t, b1, n1 * sizeof(event_t));
    memcpy(b, tmp, (n - n2) * sizeof(event_t));
}

typedef struct {
    int nobj;
    int* obj;          /* primitive indices */
    aabb box;
    int nev[3];
    event_t* ev[3];
} bnode;

static float SA(v3 v) { return 2 * (v.x * v.y + v.x * v.z + v.y * v.z); } /* :59-62 */
static float SAH(const bnode* t, int axis, float plane, int NL, int NR) { /* :64-80 */
    v3 v = vsub(t->box.r, t->box.l), vl = v, vr = v;
    if (axis == 0) { vl.x = plane - t->box.l.x; vr.x = t->box.r.x - plane; }
    if (axis == 1) { vl.y = plane - t->box.l.y; vr.y = t->box.r.y - plane; }
    if (axis == 2) { vl.z = plane - t->box.l.z; vr.z = t->box.r.z - plane; }
    float lambda = 1.0f;
    if (NL == 0 || NR == 0) lambda = 0.8f;
    return (lambda / SA(v)) * (SA(vl) * (float)NL + SA(vr) * (float)NR);
}
static int find_split(const bnode* t, float* split) { /* :82-116 */
    float cost = R_INF;
    int best = -1;
    for (int axis = 0; axis < 3; axis++) {
        int nl = 0, nr = t->nobj, i = 0;
        while (i < t->nev[axis]) {
            int pe = 0, ps = 0;
            float now = t->ev[axis][i].pos;
            while (i < t->nev[axis] && t->ev[axis][i].pos == now) {
                if (t->ev[axis][i].type == 0) pe++;
                if (t->ev[axis][i].type == 2) ps++;
                i++;
            }
            nr -= pe;
            float c = SAH(t, axis, now, nl, nr);
            if (cmpf(c - cost) < 0) { cost = c; *split = now; best = axis; }
            nl += ps;
        }
    }
    return best;
}

static int new_node(cr_scene* s) {
    GROW(s->nodes, s->nnodes, s->cap_nodes, node_t);
    memset(&s->nodes[s->nnodes], 0, sizeof(node_t));
    s->nodes[s->nnodes].axis = -1;
    return s->nnodes++;
}
static void make_leaf(cr_scene* s, int id, const bnode* t) {
    node_t* n = &s->nodes[id];
    n->axis = -1;
    n->first = (int)s->nrefs;
    n->count = t->nobj;
    for (int i = 0; i < t->nobj; i++) {
        if (s->nrefs >= s->cap_refs) { s->cap_refs = s->cap_refs ? 2 * s->cap_refs : 1024;
            s->refs = (int*)realloc(s->refs, (size_t)s->cap_refs * sizeof(int)); }
        s->refs[s->nrefs++] = t->obj[i];
    }
}
static void free_bnode(bnode* t) {
    free(t->obj);
    for (int i = 0; i < 3; i++) free(t->ev[i]);
}

/* buildTree (KDtreeAccel.cpp:118-307).  The reference keeps every node's event
 * arrays alive (its deletes are commented out, :299-304); here a node's arrays
 * are freed once both children have theirs. */
static void build(cr_scene* s, int id, bnode* t, int dep) {
    if (dep > s->dep_max || t->nobj <= 1) { make_leaf(s, id, t); free_bnode(t); return; }
    float split = 0.f;
    int axis = find_split(t, &split);
    if (axis < 0) { make_leaf(s, id, t); free_bnode(t); return; }  /* reference: UB (axis -1) */
    char* div = (char*)malloc((size_t)t->nobj);
    int nl = 0, nr = 0, nb = 0;
    for (int i = 0; i < t->nobj; i++) {
        const aabb* b = &s->prims[t->obj[i]].box;
        float st = vget(b->l, axis), ed = vget(b->r, axis);
        if (cmpf(ed - split) <= 0) { div[i] = 0; nl++; }
        else if (cmpf(split - st) <= 0) { div[i] = 1; nr++; }
        else { div[i] = 2; nb++; }
    }
    bnode L, R;
    memset(&L, 0, sizeof L);
    memset(&R, 0, sizeof R);
    L.nobj = nl + nb; R.nobj = nb + nr;
    L.obj = (int*)malloc(sizeof(int) * (size_t)(L.nobj ? L.nobj : 1));
    R.obj = (int*)malloc(sizeof(int) * (size_t)(R.nobj ? R.nobj : 1));
    int* toL = (int*)malloc(sizeof(int) * (size_t)t->nobj);
    int* toR = (int*)malloc(sizeof(int) * (size_t)t->nobj);
    int pl = 0, pr = 0;
    for (int i = 0; i < t->nobj; i++) {
        if (div[i] == 0) { toL[i] = pl; L.obj[pl++] = t->obj[i]; }
        else if (div[i] == 1) { toR[i] = pr; R.obj[pr++] = t->obj[i]; }
        else { toL[i] = pl; L.obj[pl++] = t->obj[i]; toR[i] = pr; R.obj[pr++] = t->obj[i]; }
    }
    for (int a = 0; a < 3; a++) {
        L.ev[a] = (event_t*)malloc(sizeof(event_t) * (size_t)(2 * L.nobj + 1));
        R.ev[a] = (event_t*)malloc(sizeof(event_t) * (size_t)(2 * R.nobj + 1));
        for (int j = 0; j < t->nev[a]; j++) {
            event_t e = t->ev[a][j];
            int d = div[e.index];
            if (d == 0) { event_t x = e; x.index = toL[e.index]; L.ev[a][L.nev[a]++] = x; }
            else if (d == 1) { event_t x = e; x.index = toR[e.index]; R.ev[a][R.nev[a]++] = x; }
            else if (a != axis) {
                event_t x = e; x.index = toL[e.index]; L.ev[a][L.nev[a]++] = x;
                x.index = toR[e.index]; R.ev[a][R.nev[a]++] = x;
            } else if (e.type == 0) {        /* End: clipped on the left (:240-252) */
                event_t x = e; x.pos = split; x.index = toL[e.index]; L.ev[a][L.nev[a]++] = x;
                x = e; x.index = toR[e.index]; R.ev[a][R.nev[a]++] = x;
            } else if (e.type == 2) {        /* Start: clipped on the right (:253-265) */
                event_t x = e; x.index = toL[e.index]; L.ev[a][L.nev[a]++] = x;
                x = e; x.pos = split; x.index = toR[e.index]; R.ev[a][R.nev[a]++] = x;
            }
        }
    }
    if (L.nobj > 0) {
        L.box.l = mk(L.ev[0][0].pos, L.ev[1][0].pos, L.ev[2][0].pos);
        L.box.r = mk(L.ev[0][L.nev[0] - 1].pos, L.ev[1][L.nev[1] - 1].pos, L.ev[2][L.nev[2] - 1].pos);
    }
    if (R.nobj > 0) {
        R.box.l = mk(R.ev[0][0].pos, R.ev[1][0].pos, R.ev[2][0].pos);
        R.box.r = mk(R.ev[0][R.nev[0] - 1].pos, R.ev[1][R.nev[1] - 1].pos, R.ev[2][R.nev[2] - 1].pos);
    }
    free(div); free(toL); free(toR);
    s->nodes[id].count = t->nobj;
    free_bnode(t);
    s->nodes[id].axis = axis;
    s->nodes[id].split = split;
    int li = new_node(s);
    build(s, li, &L, dep + 1);
    int ri = new_node(s);
    build(s, ri, &R, dep + 1);
    s->nodes[id].left = li;
    s->nodes[id].right = ri;
}

static void kd_build(cr_scene* s) { /* KDtreeAccel.cpp:12-57 */
    int n = s->nprims;
    s->dep_max = (int)(1.2 * log((double)n) + 2.0);
    bnode root;
    memset(&root, 0, sizeof root);
    root.nobj = n;
    root.obj = (int*)malloc(sizeof(int) * (size_t)n);
    for (int i = 0; i < n; i++) root.obj[i] = i;
    event_t* tmp = (event_t*)malloc(sizeof(event_t) * (size_t)(2 * n));
    for (int a = 0; a < 3; a++) {
        root.ev[a] = (event_t*)malloc(sizeof(event_t) * (size_t)(2 * n));
        for (int j = 0; j < n; j++) {
            event_t st = {vget(s->prims[j].box.l, a), 2, j};
            event_t ed = {vget(s->prims[j].box.r, a), 0, j};
            root.ev[a][root.nev[a]++] = st;
            root.ev[a][root.nev[a]++] = ed;
        }
        ev_msort(root.ev[a], (size_t)root.nev[a], tmp);
    }
    free(tmp);
    root.box.l = mk(root.ev[0][0].pos, root.ev[1][0].pos, root.ev[2][0].pos);
    root.box.r = mk(root.ev[0][root.nev[0] - 1].pos, root.ev[1][root.nev[1] - 1].pos,
                    root.ev[2][root.nev[2] - 1].pos);
    s->root_box = root.box;
    int r = new_node(s);
    build(s, r, &root, 1);
}

/* ---- Scene::loadScene(char*) + Scene::init ------------------------------- */
cr_scene* cr_scene_load(const char* path) {
    init_consts();
    FILE* f = fopen(path, "rb");
    if (!f) { set_err("cannot open scene", path); return NULL; }
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    char* txt = (char*)malloc((size_t)sz + 1);
    size_t got = fread(txt, 1, (size_t)sz, f);
    txt[got] = 0;
    fclose(f);
    const char* p = txt;
    xel* root = xparse(&p);
    free(txt);
    if (!root) { set_err("no root element", path); return NULL; }
    cr_scene* s = (cr_scene*)calloc(1, sizeof(cr_scene));
    for (int ci = 0; ci < root->nchild; ci++) {
        const xel* it = root->child[ci];
        if (strcmp(it->name, "camera") == 0) {         /* scene.cpp:276-304 */
            v3 pos = xv3(xnth(it, 0)), fwd = xv3(xnth(it, 1)), up = xv3(xnth(it, 2));
            const xel* res = xnth(it, 3);
            float xr = (float)xd(res, "height"), yr = (float)xd(res, "width");
            float fov = (float)xd(xnth(it, 4), "horizontalFOV");
            cam_setup(&s->cam, pos, fwd, up, xr, yr, fov);
        } else if (strcmp(it->name, "material") == 0) { /* scene.cpp:305-332 */
            mat_t m;
            m.diffuse = xc3(xnth(it, 0));
            m.phong = xc3(xnth(it, 1));
            m.specular = xc3(xnth(it, 2));
            m.phong_exp = (float)xd(xnth(it, 3), "phongExp");
            m.index = (float)xd(xnth(it, 4), "refracIndex");
            GROW(s->mats, s->nmats, s->cap_mats, mat_t);
            s->mats[s->nmats++] = m;
        } else if (strcmp(it->name, "object") == 0) {   /* scene.cpp:333-374 */
            const char* fp = xattr(xnth(it, 0), "path");
            if (!fp) { set_err("object without path", path); xfree(root); cr_scene_free(s); return NULL; }
            obj_ctx c = {s, xi(xnth(it, 1), "matid")};
            if (load_obj(fp, obj_face, &c) < 0) { set_err("bad obj index", fp); xfree(root); cr_scene_free(s); return NULL; }
        } else if (strcmp(it->name, "sphere") == 0) {   /* scene.cpp:375-396 */
            v3 c = xv3(xnth(it, 0));
            float r = (float)xd(xnth(it, 1), "radius");
            add_prim(s, mk_sph(c, r, xi(xnth(it, 2), "matid")));
        } else if (strcmp(it->name, "area_light") == 0) { /* scene.cpp:397-432 */
            const char* fp = xattr(xnth(it, 0), "path");
            if (!fp) { set_err("area_light without path", path); xfree(root); cr_scene_free(s); return NULL; }
            light_ctx c = {s, xc3(xnth(it, 1))};
            if (load_obj(fp, light_face, &c) < 0) { set_err("bad obj index", fp); xfree(root); cr_scene_free(s); return NULL; }
        }
        /* homo_media: volumes, out of scope (no effect on the surface path) */
    }
    xfree(root);
    if (s->nprims > 0) {                               /* scene.cpp:475-488 */
        kd_build(s);
        v3 diag = vsub(s->root_box.r, s->root_box.l);
        float d2 = vsqr(diag);
        s->ssph.center = vscale(vadd(s->root_box.l, s->root_box.r), 0.5f);
        s->ssph.radius = sqrtf(d2) * 0.5f;
        s->ssph.inv_r2 = 1.f / d2;
    }
    return s;
}

void cr_scene_free(cr_scene* s) {
    if (!s) return;
    free(s->prims); free(s->lights); free(s->mats); free(s->nodes); free(s->refs);
    free(s);
}
int cr_scene_nobjs(const cr_scene* s) { return s->nprims; }
int cr_scene_nlights(const cr_scene* s) { return s->nlights; }

static void hv(FILE* f, float x) { fprintf(f, " %a", (double)x); }
static void hv3(FILE* f, v3 v) { hv(f, v.x); hv(f, v.y); hv(f, v.z); }
static void hc3(FILE* f, c3 c) { hv(f, c.r); hv(f, c.g); hv(f, c.b); }
static void dump_node(const cr_scene* s, FILE* f, int id) {
    const node_t* n = &s->nodes[id];
    if (n->axis == -1) {
        fprintf(f, "L %d", n->count);
        for (int i = 0; i < n->count; i++) fprintf(f, " %d", s->refs[n->first + i]);
        fprintf(f, "\n");
        return;
    }
    fprintf(f, "I %d", n->axis);
    hv(f, n->split);
    fprintf(f, " %d\n", n->count);
    dump_node(s, f, n->left);
    dump_node(s, f, n->right);
}
int cr_scene_dump(const cr_scene* s, const char* out) {
    FILE* f = fopen(out, "w");
    if (!f) return -1;
    fprintf(f, "nobjs %d\n", s->nprims);
    for (int i = 0; i < s->nprims; i++) {
        const prim_t* p = &s->prims[i];
        if (p->type == PRIM_TRI) { fprintf(f, "tri %d", p->matId); hv3(f, p->p0); hv3(f, p->p1); hv3(f, p->p2); }
        else { fprintf(f, "sph %d", p->matId); hv3(f, p->c); hv(f, p->rad); }
        fprintf(f, "\n");
    }
    fprintf(f, "nlights %d\n", s->nlights);
    for (int i = 0; i < s->nlights; i++) {
        const light_t* l = &s->lights[i];
        fprintf(f, "light"); hv3(f, l->p0); hv3(f, l->d1); hv3(f, l->d2);
        hv3(f, l->fr.x); hv3(f, l->fr.y); hv3(f, l->fr.z); hc3(f, l->le); hv(f, l->inv_area);
        fprintf(f, "\n");
    }
    fprintf(f, "nmat %d\n", s->nmats);
    for (int i = 0; i < s->nmats; i++) {
        const mat_t* m = &s->mats[i];
        fprintf(f, "mat"); hc3(f, m->diffuse); hc3(f, m->phong); hv(f, m->phong_exp);
        hc3(f, m->specular); hv(f, m->index); fprintf(f, "\n");
    }
    const camera_t* c = &s->cam;
    fprintf(f, "camera"); hv3(f, c->pos); hv3(f, c->fwd); hv3(f, c->up);
    hv(f, c->xres); hv(f, c->yres); hv(f, c->plane_dist); fprintf(f, "\n");
    fprintf(f, "w2r"); for (int i = 0; i < 16; i++) hv(f, c->w2r.m[i / 4][i % 4]); fprintf(f, "\n");
    fprintf(f, "r2w"); for (int i = 0; i < 16; i++) hv(f, c->r2w.m[i / 4][i % 4]); fprintf(f, "\n");
    fprintf(f, "sphere"); hv3(f, s->ssph.center); hv(f, s->ssph.radius); hv(f, s->ssph.inv_r2); fprintf(f, "\n");
    fprintf(f, "totarea"); hv(f, s->tot_area); fprintf(f, "\n");
    if (s->nprims > 0) {
        fprintf(f, "kd %d", s->dep_max); hv3(f, s->root_box.l); hv3(f, s->root_box.r); fprintf(f, "\n");
        dump_node(s, f, 0);
    }
    fclose(f);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* KDtreeAccel::traverse (KDtreeAccel.cpp:309-388) + Scene wrappers           */
/* ------------------------------------------------------------------------- */
typedef struct { int node; float tmin, tmax; } todo_t;

/* Debugging aid (tests / scripts only): every traversal query of the calls
 * that follow -- origin, direction, best t (-1 = miss), winner index as int
 * bits -- into buf[cap][8]; single-threaded callers only. */
static float* g_ray_log;
static int64_t g_ray_log_cap, g_ray_log_n;
void cr_set_ray_log(float* buf, int64_t cap) { g_ray_log = buf; g_ray_log_cap = cap; g_ray_log_n = 0; }
int64_t cr_ray_log_count(void) { return g_ray_log_n; }

static int traverse(const cr_scene* s, const ray_t* ray, cr_stats* st) {
    float tmin, tmax;
    if (!box_hit(&s->root_box, ray, &tmin, &tmax)) return -1;
    v3 inv = mk(1.f / ray->d.x, 1.f / ray->d.y, 1.f / ray->d.z);
    todo_t todo[64];
    int tp = 0, res = -1, cur = 0;
    float best = R_INF;
    int64_t ni = 0, nl = 0, nr = 0, ntt = 0, nst = 0;
    while (cur >= 0) {
        if (ray->tmax < tmin) break;
        const node_t* n = &s->nodes[cur];
        if (n->axis != -1) {
            ni++;
            int a = n->axis;
            float oa = vget(ray->o, a);
            float t = (n->split - oa) * vget(inv, a);
            int below = (oa < n->split) || (oa == n->split && vget(ray->d, a) <= 0);
            int nearc = below ? n->left : n->right, farc = below ? n->right : n->left;
            if (t > tmax || t <= 0) cur = nearc;
            else if (t < tmin) cur = farc;
            else {
                todo[tp].node = farc; todo[tp].tmin = t; todo[tp].tmax = tmax; tp++;
                cur = nearc;
                tmax = t;
            }
        } else {
            nl++;
            hit_t h;
            h.t = R_INF;
            for (int i = 0; i < n->count; i++) {
                const prim_t* g = &s->prims[s->refs[n->first + i]];
                nr++;
                if (g->type == PRIM_TRI) ntt++; else nst++;
                if (prim_hit(g, ray, &h)) {
                    if (cmpf(h.t - best) < 0) { best = h.t; res = s->refs[n->first + i]; }
                }
            }
            if (tp > 0) { tp--; cur = todo[tp].node; tmin = todo[tp].tmin; tmax = todo[tp].tmax; }
            else break;
        }
    }
    if (st) { st->inner_visits += ni; st->leaf_visits += nl; st->prim_refs += nr; st->tri_tests += ntt; st->sph_tests += nst; }
    if (g_ray_log && g_ray_log_n < g_ray_log_cap) { /* debugging: cr_set_ray_log */
        float* o = g_ray_log + 8 * g_ray_log_n++;
        o[0] = ray->o.x; o[1] = ray->o.y; o[2] = ray->o.z;
        o[3] = ray->d.x; o[4] = ray->d.y; o[5] = ray->d.z;
        o[6] = res >= 0 ? best : -1.f;
        memcpy(&o[7], &res, 4);
    }
    return res;
}

/* Scene::intersect (scene.cpp:21-43): traverse, then re-run hit on the winner */
static int intersect(const cr_scene* s, const ray_t* ray, hit_t* h, cr_stats* st) {
    if (st) st->closest_rays++;
    int g = traverse(s, ray, st);
    if (g >= 0) prim_hit(&s->prims[g], ray, h);
    return g;
}
/* Scene::occluded / shadowRayTest (scene.cpp:55-81) */
static int occluded(const cr_scene* s, v3 p1, v3 d, v3 p2, cr_stats* st) {
    ray_t ray = mkray(p1, d);
    if (st) st->shadow_rays++;
    int g = traverse(s, &ray, st);
    if (g < 0) return 0;
    hit_t h;
    prim_hit(&s->prims[g], &ray, &h);
    return veq(ray_at(&ray, h.t), p2) ? 0 : 1;
}

void cr_trace(const cr_scene* s, const float* r9, int64_t n, int32_t* oi, float* of,
              uint8_t* occ, cr_stats* st) {
    init_consts();
    for (int64_t k = 0; k < n; k++) {
        const float* r = r9 + 9 * k;
        ray_t ray = mkray(mk(r[0], r[1], r[2]), mk(r[3], r[4], r[5]));
        hit_t h;
        memset(&h, 0, sizeof h);
        int g = intersect(s, &ray, &h, st);
        oi[3 * k] = g;
        oi[3 * k + 1] = g >= 0 ? h.inside : 0;
        oi[3 * k + 2] = g >= 0 ? h.matId : 0;
        float* o = of + 7 * k;
        if (g >= 0) { o[0] = h.t; o[1] = h.p.x; o[2] = h.p.y; o[3] = h.p.z; o[4] = h.n.x; o[5] = h.n.y; o[6] = h.n.z; }
        else memset(o, 0, 7 * sizeof(float));
        if (occ) occ[k] = (uint8_t)occluded(s, mk(r[0], r[1], r[2]), mk(r[3], r[4], r[5]), mk(r[6], r[7], r[8]), st);
    }
}

/* ------------------------------------------------------------------------- */
/* BidirPathTracing (bidirPathTracing.cpp)                                    */
/* ------------------------------------------------------------------------- */
typedef struct {
    v3 origin, pos, dir;
    c3 thr;
    bsdf_t bsdf;
    float dVCM, dVC;
    int len, nspec, finite;
} bstate;

typedef struct {
    const cr_scene* s;
    int W, H, P, ctl, maxlen;
    float* film;
    cr_stats* st;
    bstate* lv; int64_t nlv, cap_lv;
    int* lidx;
} bdpt_ctx;

static inline int len_ok(const bdpt_ctx* c, int L) { return c->ctl <= 0 || L == c->ctl; }

static void film_add(float* film, int H, int W, int h, int w, c3 v) { /* film.cpp:4-9 */
    if (h < 0 || h >= H || w < 0 || w >= W) return;
    float* p = film + 3 * ((size_t)h * W + w);
    p[0] = p[0] + v.r;
    p[1] = p[1] + v.g;
    p[2] = p[2] + v.b;
}

static void gen_light(bdpt_ctx* c, rng_t* rng, bstate* ls) { /* :267-311 */
    const cr_scene* s = c->s;
    int nl = s->nlights;
    float lpp = 1.f / (float)nl;
    int id = (int)(rng_f(rng) * (float)nl);
    const light_t* l = &s->lights[id];
    float epdf, dpdf, cal;
    c3 rad;
    for (;;) {
        /* emit(sceneSphere, rng.randVector3(), rng.randVector3(), ...): GCC
         * evaluates the arguments right to left, so posRand3 is drawn first. */
        v3 pr = rng_v3(rng);
        v3 dr = rng_v3(rng);
        rad = light_emit(l, dr, pr, &ls->origin, &ls->dir, &epdf, &dpdf, &cal);
        if (epdf > 1e-7f) break;
    }
    ls->thr = rad;
    epdf *= lpp;
    dpdf *= lpp;
    ls->thr = cdivs(ls->thr, epdf);
    ls->len = 1;
    ls->finite = 1;
    ls->nspec = 0;
    ls->dVCM = dpdf / epdf;
    ls->dVC = 1.f / epdf;  /* AreaLight::isDelta() == 0 */
}

static int sample_scatter(bdpt_ctx* c, rng_t* rng, const bsdf_t* b, v3 hit, bstate* ps) { /* :370-416 */
    const mat_t* mats = c->s->mats;
    float dpdf, cosWo;
    int type;
    v3 r3 = rng_v3(rng);
    c3 f = bsdf_sample(b, mats, r3, &ps->dir, &dpdf, &cosWo, &type);
    if (cblack(f)) return 0;
    float rpdf = dpdf;
    if ((type & T_SPEC) == 0) rpdf = bsdf_pdf(b, mats, ps->dir, 1);
    float cp = b->cont;
    if (rng_f(rng) > cp) return 0;
    dpdf *= cp;
    rpdf *= cp;
    if (type & T_SPEC) {
        ps->nspec++;
        ps->dVCM = 0.f;
        ps->dVC *= cosWo;
    } else {
        ps->dVC = (1.f / dpdf) * (ps->dVCM + ps->dVC * rpdf);
        ps->dVCM = 1.f / dpdf;
    }
    ps->origin = hit;
    ps->thr = cscale(cmul(ps->thr, f), cosWo / dpdf);
    return 1;
}

#ifdef CR_DEBUG_PATH
static int g_dbg_on;
#endif
static c3 connect_camera(bdpt_ctx* c, const bstate* ls, v3 hit, const bsdf_t* b) { /* :313-368 */
    const cr_scene* s = c->s;
    const camera_t* cam = &s->cam;
    c3 res = C0;
    v3 dtc = vsub(cam->pos, hit);
    if (vdot(vneg(dtc), cam->fwd) <= 0) return res;
    float d2 = vsqr(dtc);
    float dist = sqrtf(d2);
    dtc = vdiv(dtc, dist);
    float cosTo, dp, rp;
    c3 f = bsdf_f(b, s->mats, dtc, &cosTo, &dp, &rp);
    if (cblack(f)) return res;
    rp *= b->cont;
    float cosAt = vdot(vneg(dtc), cam->fwd);
    float ipd = cam->plane_dist / cosAt;
    float i2sa = (ipd * ipd) / cosAt;
    float i2s = i2sa * fabsf(cosTo) / d2;
    float pdfA = i2s;
    float s2i = 1.f / i2s;
    res = cdivs(cmul(ls->thr, f), (float)c->P * s2i);
#ifdef CR_DEBUG_PATH
    if (g_dbg_on)
        printf("[dbg cpu] len %d hit %a %a %a thr %a %a %a f %a %a %a cos_to %a d2 %a i2s %a res %a %a %a rp %a dvcm %a dvc %a\n",
               ls->len, hit.x, hit.y, hit.z, ls->thr.r, ls->thr.g, ls->thr.b, f.r, f.g, f.b, cosTo, d2, i2s,
               res.r, res.g, res.b, rp, ls->dVCM, ls->dVC);
#endif
    if (cblack(res)) return res;
    if (occluded(s, hit, dtc, cam->pos, c->st)) return C0;
    float wl = (pdfA / (float)c->P) * (ls->dVCM + rp * ls->dVC);
    float w = 1.f / (wl + 1.f);
    return cscale(res, w);
}

static c3 light_radiance_mis(bdpt_ctx* c, const light_t* l, const bstate* cs, v3 rd) { /* :454-482 */
    float lpp = 1.f / (float)c->s->nlights;
    float dpa, ep;
    c3 r = light_radiance(l, rd, &dpa, &ep);
    if (cblack(r)) return C0;
    if (cs->len == 1) return r;
    dpa *= lpp;
    ep *= lpp;
    float wc = dpa * cs->dVCM + ep * cs->dVC;
    float w = 1.f / (1.f + wc);
    return cscale(r, w);
}

static c3 direct_illum(bdpt_ctx* c, rng_t* rng, const bstate* cs, v3 hit, const bsdf_t* b) { /* :484-608 */
    const cr_scene* s = c->s;
    c3 res = C0;
    float weight = 0.f;
    int nl = s->nlights;
    float lpp = 1.f / (float)nl;
    int id = (int)(rng_f(rng) * (float)nl);
    const light_t* l = &s->lights[id];
    v3 dtl;
    float dist, dpdf, epdf, cal, cosAtSurf;
    int type;
    v3 r3 = rng_v3(rng);
    c3 illu = light_illum(l, hit, r3, &dtl, &dist, &dpdf, &epdf, &cal);
    float bdp, brp, cosTo;
    if (!cblack(illu) && dpdf > 0) {
        c3 bf = bsdf_f(b, s->mats, dtl, &cosTo, &bdp, &brp);
        if (!cblack(bf)) {
            float cp = b->cont;
            bdp *= cp;  /* light is not delta */
            brp *= cp;
            c3 tmp = cdivs(cscale(cmul(illu, bf), cosTo), dpdf * lpp);
            if (!cblack(tmp) && !occluded(s, hit, dtl, vadd(hit, vscale(dtl, dist)), c->st)) {
                float wl = bdp / (dpdf * lpp);
                float wc = (epdf * cosTo / (dpdf * cal)) * (cs->dVCM + brp * cs->dVC);
                weight = 1.f / (wl + 1.f + wc);
                float w2 = dpdf / (dpdf + bdp);
                res = cadd(res, cscale(tmp, w2));
            }
        }
    }
    /* BSDF-sampled half (AreaLight is never delta) */
    v3 r3b = rng_v3(rng);
    c3 bf = bsdf_sample(b, s->mats, r3b, &dtl, &dpdf, &cosAtSurf, &type);
    if (!cblack(bf) && dpdf > 0) {
        float w = 1.f;
        float lpdf;
        if (!(type & T_SPEC)) {
            illu = light_radiance(l, dtl, &lpdf, &epdf);
            if (cmpf(lpdf) == 0) return res;       /* :563-564: outer weight skipped */
            w = dpdf / (dpdf + lpdf);
        }
        hit_t lh;
        ray_t ray = mkray(vadd(hit, vscale(dtl, R_EPS)), dtl);
        int g = intersect(s, &ray, &lh, c->st);
        if (g >= 0) {
            if (lh.matId < 0) { if (l != &s->lights[-lh.matId - 1]) illu = C0; }
            else illu = C0;
        } else {
            illu = C0;  /* background == NULL */
        }
        if (!cblack(illu)) {
            c3 tmp = cdivs(cscale(cmul(illu, bf), cosAtSurf), dpdf);
            res = cadd(res, cscale(tmp, w));
        }
    }
    return cscale(res, weight);
}

static c3 connect_vertices(bdpt_ctx* c, const bstate* ls, const bsdf_t* cb, v3 hit,
                           const bstate* cs) { /* :610-665 */
    const cr_scene* s = c->s;
    v3 dir = vsub(ls->pos, hit);
    float d2 = vsqr(dir);
    float dist = sqrtf(d2);
    dir = vdiv(dir, dist);
    c3 res = C0;
    float cosC, cdp, crp;
    c3 cf = bsdf_f(cb, s->mats, dir, &cosC, &cdp, &crp);
    if (cblack(cf)) return res;
    float ccp = cb->cont;
    cdp *= ccp;
    crp *= ccp;
    float cosL, ldp, lrp;
    c3 lf = bsdf_f(&ls->bsdf, s->mats, vneg(dir), &cosL, &ldp, &lrp);
    if (cblack(lf)) return res;
    float lcp = ls->bsdf.cont;
    ldp *= lcp;
    lrp *= lcp;
    float G = cosL * cosC / d2;
    if (cmpf(G) < 0) return res;
    float cdpa = cdp * fabsf(cosL) / (dist * dist);
    float ldpa = ldp * fabsf(cosC) / (dist * dist);
    res = cscale(cmul(cf, lf), G);
    if (cblack(res) || occluded(s, hit, dir, vadd(hit, vscale(dir, dist)), c->st)) return C0;
    float wl = cdpa * (ls->dVCM + lrp * ls->dVC);
    float wc = ldpa * (cs->dVCM + crp * cs->dVC);
    float w = 1.f / (wl + 1.f + wc);
    return cscale(res, w);
}

static void push_lv(bdpt_ctx* c, const bstate* v) {
    if (c->nlv >= c->cap_lv) { c->cap_lv = c->cap_lv ? 2 * c->cap_lv : 4096;
        c->lv = (bstate*)realloc(c->lv, (size_t)c->cap_lv * sizeof(bstate)); }
    c->lv[c->nlv++] = *v;
}

static void rng_for(rng_t* r, int mode, mt_state* mt, uint32_t seed, uint32_t iter, uint32_t sub, uint32_t path) {
    r->mode = mode;
    r->mt = mt;
    r->ctr = 0;
    r->key = mode == CR_RNG_COUNTER ? cr_stream_key(seed, iter, sub, path) : 0;
}

static void run_iteration(bdpt_ctx* c, mt_state* mt, int mode, uint32_t seed, uint32_t iter,
                          int64_t pb, int64_t pe) { /* :53-265 */
    const cr_scene* s = c->s;
    const camera_t* cam = &s->cam;
    int P = c->P;
    memset(c->lidx, 0, sizeof(int) * (size_t)P);
    c->nlv = 0;
    rng_t rng;
    /* light pass (:67-131) */
    for (int64_t pi = pb; pi < pe; pi++) {
        rng_for(&rng, mode, mt, seed, iter, 0, (uint32_t)pi);
        bstate ls;
        memset(&ls, 0, sizeof ls);
        gen_light(c, &rng, &ls);
#ifdef CR_DEBUG_PATH
        g_dbg_on = pi == CR_DEBUG_PATH && iter == CR_DEBUG_ITER;
#endif
        for (;; ls.len++) {
            ray_t ray = mkray(vadd(ls.origin, vscale(ls.dir, R_EPS)), ls.dir);
            hit_t h;
            if (intersect(s, &ray, &h, c->st) < 0) break;
            v3 hp = h.p;
            bsdf_t b;
            bsdf_init(&b, vneg(ray.d), &h, s->mats);
            if (b.matId == 0) break;
            ls.pos = hp;
            ls.bsdf = b;
            if (ls.len > 1 || ls.finite) ls.dVCM *= (h.t * h.t);
            ls.dVCM /= fabsf(b.wi.z);
            ls.dVC /= fabsf(b.wi.z);
            if (!b.delta) push_lv(c, &ls);
            if (!b.delta && len_ok(c, ls.len + 1)) {
                v3 ip = x_point(&cam->w2r, hp);
                if (cam_check(cam, ip.x, ip.y)) {
                    c3 r = connect_camera(c, &ls, hp, &b);
                    film_add(c->film, c->H, c->W, (int)ip.x, (int)ip.y, r);
                }
            }
            if (ls.len + 2 > c->maxlen) break;
            if (!sample_scatter(c, &rng, &b, hp, &ls)) break;
        }
        c->lidx[pi] = (int)c->nlv;
    }
    /* camera pass (:133-264) */
    for (int64_t pi = pb; pi < pe; pi++) {
        rng_for(&rng, mode, mt, seed, iter, 1, (uint32_t)pi);
        bstate cs;
        memset(&cs, 0, sizeof cs);
        /* generateCameraSample (:418-452) */
        int y = (int)(pi % c->W), x = (int)(pi / c->W);
        v3 jit = rng_v3(&rng);
        v3 smp = mk((float)x + jit.x, (float)y + jit.y, 0.f);
        v3 rp = x_point(&cam->r2w, mk(smp.x, smp.y, 0));
        ray_t cr = mkray(cam->pos, vsub(rp, cam->pos));
        float cosAt = vdot(cam->fwd, cr.d);
        float ipd = cam->plane_dist / cosAt;
        float i2sa = (ipd * ipd) / cosAt;
        cs.origin = cr.o;
        cs.dir = cr.d;
        cs.len = 1;
        cs.nspec = 0;
        cs.thr = mkc(1, 1, 1);
        cs.dVCM = (float)P / i2sa;
        cs.dVC = 0.f;
        c3 color = C0;
        for (;; cs.len++) {
            ray_t ray = mkray(vadd(cs.origin, vscale(cs.dir, R_EPS)), cs.dir);
            hit_t h;
            if (intersect(s, &ray, &h, c->st) < 0) break;
            v3 hp = h.p;
            bsdf_t b;
            bsdf_init(&b, vneg(ray.d), &h, s->mats);
            if (b.matId == 0) break;
            cs.dVCM *= (h.t * h.t);
            cs.dVCM /= fabsf(b.wi.z);
            cs.dVC /= fabsf(b.wi.z);
            if (h.matId < 0) {
                const light_t* l = &s->lights[-h.matId - 1];
                if (len_ok(c, cs.len))
                    color = cadd(color, cmul(cs.thr, light_radiance_mis(c, l, &cs, ray.d)));
                break;
            }
            if (cs.len >= c->maxlen) break;
            if (!b.delta && len_ok(c, cs.len + 1)) {
                float w = 1.f / ((float)cs.len + 1.f - (float)cs.nspec);
                color = cadd(color, cscale(cmul(cs.thr, direct_illum(c, &rng, &cs, hp, &b)), w));
            }
            if (!b.delta) {
                int st0 = pi == 0 ? 0 : c->lidx[pi - 1], ed = c->lidx[pi];
                for (int i = st0; i < ed; i++) {
                    const bstate* lsv = &c->lv[i];
                    if (lsv->len + 1 + cs.len > c->maxlen) break;
                    if (lsv->bsdf.delta) continue;
                    c3 tmp = connect_vertices(c, lsv, &b, hp, &cs);
                    float w = 1.f / ((float)lsv->len + 1.f + (float)cs.len - (float)lsv->nspec - (float)cs.nspec);
                    if (len_ok(c, lsv->len + 1 + cs.len))
                        color = cadd(color, cscale(cmul(cmul(cs.thr, lsv->thr), tmp), w));
                }
            }
            if (!sample_scatter(c, &rng, &b, hp, &cs)) break;
        }
        film_add(c->film, c->H, c->W, (int)smp.x, (int)smp.y, color);
    }
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

int cr_render_bdpt(const cr_scene* s, int W, int H, int iter_begin, int iterations, uint32_t seed,
                   int rng_mode, int control_length, int64_t path_begin, int64_t path_end,
                   float* film, cr_stats* st) {
    init_consts();
    if (!s || s->nprims == 0 || s->nlights == 0) { set_err("scene has no geometry or lights", NULL); return -1; }
    bdpt_ctx c;
    memset(&c, 0, sizeof c);
    c.s = s; c.W = W; c.H = H; c.P = W * H; c.ctl = control_length; c.maxlen = 10;
    c.film = film; c.st = st;
    c.lidx = (int*)calloc((size_t)c.P, sizeof(int));
    if (path_end > c.P) path_end = c.P;
    mt_state mt;
    mt_seed(&mt, seed);
    double t0 = now_s();
    for (int it = 0; it < iterations; it++)
        run_iteration(&c, &mt, rng_mode, seed, (uint32_t)(iter_begin + it), path_begin, path_end);
    if (st) st->seconds += now_s() - t0;
    free(c.lidx);
    free(c.lv);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* VertexCM (vertexcm.h, vertexcm.cpp) + the point KD tree (KDtree.h)         */
/* ------------------------------------------------------------------------- */
typedef struct {  /* SubPathState (vertexcm.h:25-37) / PathVertex (:12-23) */
    v3 origin, dir, pos;
    c3 thr;
    bsdf_t bsdf;
    float dVCM, dVC, dVM;
    int len;
} vstate;

typedef struct {  /* KdNode (KDtree.h:8-30): pre-order, left child = node + 1 */
    float split;
    int axis;      /* 0..2 inner, -1 leaf */
    int has_left;
    int right;     /* -1: none */
} vkd_node;

typedef struct {
    const cr_scene* s;
    int W, H, P, minlen, maxlen;
    float N;                           /* lightSubPathNum (:49-51) */
    float radius, vm_norm, mis_vm, mis_vc;
    float* film;
    cr_stats* st;
    vstate* lv; int64_t nlv, cap_lv;
    int* ends;                         /* pathEnds */
    vkd_node* nodes; int* node_vert; int64_t nnodes, next_node;
    int* idx;                          /* build scratch: buildNodes */
    int cur_axis;
} vcm_ctx;

/* CompareNode (KDtree.h:74-86): pos[axis], ties by address (= index in data). */
static inline int vkd_less(const vcm_ctx* c, int a, int b, int axis) {
    float pa = vget(c->lv[a].pos, axis), pb = vget(c->lv[b].pos, axis);
    return pa == pb ? a < b : pa < pb;
}

/* std::nth_element under a strict total order: the element of rank k lands at
 * k, smaller ones before it, larger after.  The tree depends only on these
 * sets (KDtree.h:117-138), not on their arrangement, so any selection
 * algorithm reproduces the reference's tree. */
static void vkd_select(vcm_ctx* c, int* a, int n, int k, int axis) {
    int lo = 0, hi = n - 1;
    while (hi > lo) {
        int mid = lo + (hi - lo) / 2;
        /* median of three to a[hi] */
        if (vkd_less(c, a[mid], a[lo], axis)) { int t = a[mid]; a[mid] = a[lo]; a[lo] = t; }
        if (vkd_less(c, a[hi], a[lo], axis)) { int t = a[hi]; a[hi] = a[lo]; a[lo] = t; }
        if (vkd_less(c, a[mid], a[hi], axis)) { int t = a[mid]; a[mid] = a[hi]; a[hi] = t; }
        int pv = a[hi], st = lo;
        for (int i = lo; i < hi; i++)
            if (vkd_less(c, a[i], pv, axis)) { int t = a[i]; a[i] = a[st]; a[st] = t; st++; }
        a[hi] = a[st]; a[st] = pv;
        if (st == k) return;
        if (k < st) hi = st - 1; else lo = st + 1;
    }
}

static void vkd_build(vcm_ctx* c, int64_t node, int st, int ed) { /* KdTree::buildTree (KDtree.h:88-139) */
    vkd_node* nd = &c->nodes[node];
    if (st + 1 == ed) {
        nd->axis = -1; nd->has_left = 0; nd->right = -1;
        c->node_vert[node] = c->idx[st];
        return;
    }
    v3 l = mk(R_INF, R_INF, R_INF), r = mk(-R_INF, -R_INF, -R_INF);
    for (int i = st; i < ed; i++) {
        v3 p = c->lv[c->idx[i]].pos;
        l.x = fmins(l.x, p.x); l.y = fmins(l.y, p.y); l.z = fmins(l.z, p.z);   /* std::min(l, p) */
        r.x = fmaxs(r.x, p.x); r.y = fmaxs(r.y, p.y); r.z = fmaxs(r.z, p.z);
    }
    v3 diag = vsub(r, l);
    float tmp = -R_INF;
    int axis = -1;
    for (int i = 0; i <= 2; i++)
        if (tmp < vget(diag, i)) { tmp = vget(diag, i); axis = i; }
    int sp = (st + ed) / 2;
    vkd_select(c, c->idx + st, ed - st, sp - st, axis);
    nd = &c->nodes[node];
    nd->split = vget(c->lv[c->idx[sp]].pos, axis);
    nd->axis = axis; nd->has_left = 0; nd->right = -1;
    c->node_vert[node] = c->idx[sp];
    if (st < sp) {
        c->nodes[node].has_left = 1;
        int64_t ch = c->next_node++;
        vkd_build(c, ch, st, sp);
    }
    if (sp + 1 < ed) {
        int64_t ch = c->next_node++;
        c->nodes[node].right = (int)ch;
        vkd_build(c, ch, sp + 1, ed);
    }
}

typedef struct {  /* RangeQuery (vertexcm.h:42-97) */
    const bsdf_t* cb;
    const vstate* cs;
    c3 contrib;
} vquery;

static void vquery_process(vcm_ctx* c, vquery* q, const vstate* lv) { /* vertexcm.h:59-96 */
    if (lv->len + q->cs->len > c->maxlen || lv->len + q->cs->len < c->minlen) return;
    v3 ldir = to_world(&lv->bsdf.fr, lv->bsdf.wi);  /* BSDF::wiWorld (bsdf.h:101-104) */
    float cosC, dp, rp;
    c3 f = bsdf_f(q->cb, c->s->mats, ldir, &cosC, &dp, &rp);
    if (cblack(f)) return;
    if (c->st) c->st->vm_merged++;
    dp *= q->cb->cont;
    rp *= lv->bsdf.cont;
    float wl = lv->dVCM * c->mis_vc + lv->dVM * dp;
    float wc = q->cs->dVCM * c->mis_vc + q->cs->dVM * rp;
    float w = 1.f / (wl + 1.f + wc);
    c3 tmp = cmul(f, lv->thr);
    q->contrib = cadd(q->contrib, cscale(tmp, w));
}

static void vkd_search(vcm_ctx* c, int64_t node, v3 pos, float radius, vquery* q) { /* KDtree.h:141-175 */
    const vkd_node* nd = &c->nodes[node];
    if (nd->axis >= 0) {
        float pa = vget(pos, nd->axis);
        float delta = fabsf(pa - nd->split);
        if (pa <= nd->split) {
            if (nd->has_left) vkd_search(c, node + 1, pos, radius, q);
            if (delta < radius && nd->right >= 0) vkd_search(c, nd->right, pos, radius, q);
        } else {
            if (nd->right >= 0) vkd_search(c, nd->right, pos, radius, q);
            if (delta < radius && nd->has_left) vkd_search(c, node + 1, pos, radius, q);
        }
    }
    const vstate* lv = &c->lv[c->node_vert[node]];
    v3 d = vsub(pos, lv->pos);
    float dis = sqrtf(vsqr(d));
    if (dis < radius) {
        if (c->st) c->st->vm_found++;
        vquery_process(c, q, lv);
    }
}

/* Known-answer hook: build the point tree over pts[n][3] and, per query, count
 * the vertices searchInRadius reports and sum their indices; the same two
 * numbers by brute force (|q - p| < radius, same float expression). */
typedef struct { int64_t n, isum; } vkd_acc;
static void vkd_collect(vcm_ctx* c, int64_t node, v3 pos, float radius, vkd_acc* a) {
    const vkd_node* nd = &c->nodes[node];
    if (nd->axis >= 0) {
        float pa = vget(pos, nd->axis), delta = fabsf(pa - nd->split);
        if (pa <= nd->split) {
            if (nd->has_left) vkd_collect(c, node + 1, pos, radius, a);
            if (delta < radius && nd->right >= 0) vkd_collect(c, nd->right, pos, radius, a);
        } else {
            if (nd->right >= 0) vkd_collect(c, nd->right, pos, radius, a);
            if (delta < radius && nd->has_left) vkd_collect(c, node + 1, pos, radius, a);
        }
    }
    int v = c->node_vert[node];
    if (sqrtf(vsqr(vsub(pos, c->lv[v].pos))) < radius) { a->n++; a->isum += v; }
}
void cr_kat_vkd(const float* pts, int n, const float* qs, int nq, float radius, int64_t* out4) {
    vcm_ctx c;
    memset(&c, 0, sizeof c);
    c.lv = (vstate*)calloc((size_t)n, sizeof(vstate));
    for (int i = 0; i < n; i++) c.lv[i].pos = mk(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]);
    c.nlv = n;
    c.nodes = (vkd_node*)calloc((size_t)n, sizeof(vkd_node));
    c.node_vert = (int*)calloc((size_t)n, sizeof(int));
    c.idx = (int*)calloc((size_t)n, sizeof(int));
    for (int i = 0; i < n; i++) c.idx[i] = i;
    c.next_node = 1;
    if (n > 0) vkd_build(&c, 0, 0, n);
    for (int k = 0; k < nq; k++) {
        v3 q = mk(qs[3 * k], qs[3 * k + 1], qs[3 * k + 2]);
        vkd_acc a = {0, 0}, b = {0, 0};
        if (n > 0) vkd_collect(&c, 0, q, radius, &a);
        for (int i = 0; i < n; i++)
            if (sqrtf(vsqr(vsub(q, c.lv[i].pos))) < radius) { b.n++; b.isum += i; }
        out4[4 * k] = a.n; out4[4 * k + 1] = a.isum; out4[4 * k + 2] = b.n; out4[4 * k + 3] = b.isum;
    }
    free(c.lv); free(c.nodes); free(c.node_vert); free(c.idx);
}

static void vcm_gen_light(vcm_ctx* c, rng_t* rng, vstate* ls) { /* :287-330 */
    const cr_scene* s = c->s;
    int nl = s->nlights;
    float lpp = 1.f / (float)nl;
    int id = (int)(rng_f(rng) * (float)nl);
    const light_t* l = &s->lights[id];
    float epdf, dpdf, cal;
    c3 rad;
    for (;;) {
        v3 pr = rng_v3(rng);  /* argument order as gen_light above */
        v3 dr = rng_v3(rng);
        rad = light_emit(l, dr, pr, &ls->origin, &ls->dir, &epdf, &dpdf, &cal);
        if (epdf > 1e-7f) break;
    }
    ls->thr = rad;
    epdf = fmaxs(epdf, 1e-7f);
    epdf *= lpp;
    dpdf *= lpp;
    ls->thr = cdivs(ls->thr, epdf);
    ls->len = 1;
    ls->dVCM = dpdf / epdf;
    ls->dVC = cal / epdf;     /* AreaLight: finite, not delta -> cosAtLight */
    ls->dVM = ls->dVC * c->mis_vc;
}

static int vcm_scatter(vcm_ctx* c, rng_t* rng, const bsdf_t* b, v3 hit, vstate* ps) { /* :386-444 */
    const mat_t* mats = c->s->mats;
    float dpdf, cosWo;
    int type;
    v3 r3 = rng_v3(rng);
    c3 f = bsdf_sample(b, mats, r3, &ps->dir, &dpdf, &cosWo, &type);
    if (cblack(f)) return 0;
    float rpdf = dpdf;
    if ((type & T_SPEC) == 0) rpdf = bsdf_pdf(b, mats, ps->dir, 1);
    float cp = b->cont;
    if (rng_f(rng) > cp) return 0;
    dpdf *= cp;
    rpdf *= cp;
    if (type & T_SPEC) {
        ps->dVCM = 0.f;
        ps->dVC *= cosWo;
        ps->dVM *= cosWo;
    } else {
        ps->dVC = (cosWo / dpdf) * (ps->dVC * rpdf + ps->dVCM + c->mis_vm);
        ps->dVM = (cosWo / dpdf) * (ps->dVM * rpdf + ps->dVCM * c->mis_vc + 1.f);
        ps->dVCM = 1.f / dpdf;
    }
    ps->origin = hit;
    ps->thr = cscale(cmul(ps->thr, f), cosWo / dpdf);
    return 1;
}

static c3 vcm_connect_camera(vcm_ctx* c, const vstate* ls, v3 hit, const bsdf_t* b) { /* :332-384 */
    const cr_scene* s = c->s;
    const camera_t* cam = &s->cam;
    c3 res = C0;
    v3 dtc = vsub(cam->pos, hit);
    if (cmpf(vdot(vneg(dtc), cam->fwd)) <= 0) return res;
    float d2 = vsqr(dtc);
    float dist = sqrtf(d2);
    dtc = vdiv(dtc, dist);
    float cosTo, dp, rp;
    c3 f = bsdf_f(b, s->mats, dtc, &cosTo, &dp, &rp);
    if (cblack(f)) return res;
    rp *= b->cont;
    float cosAt = vdot(vneg(dtc), cam->fwd);
    float ipd = cam->plane_dist / cosAt;
    float i2sa = (ipd * ipd) / cosAt;
    float i2s = i2sa * fabsf(cosTo) / d2;
    float pdfA = i2s;
    float wl = (pdfA / c->N) * (c->mis_vm + ls->dVCM + ls->dVC * rp);
    float w = 1.f / (wl + 1.f);
    float s2i = 1.f / i2s;
    res = cdivs(cscale(cmul(ls->thr, f), w), c->N * s2i);
    if (cblack(res)) return res;
    if (occluded(s, hit, dtc, cam->pos, c->st)) return C0;
    return res;
}

static c3 vcm_direct(vcm_ctx* c, rng_t* rng, const vstate* cs, v3 hit, const bsdf_t* b) { /* :516-573 */
    const cr_scene* s = c->s;
    c3 res = C0;
    int nl = s->nlights;
    float lpp = 1.f / (float)nl;
    int id = (int)(rng_f(rng) * (float)nl);
    const light_t* l = &s->lights[id];
    v3 dtl;
    float dist, dpdf, epdf, cal;
    v3 r3 = rng_v3(rng);
    c3 illu = light_illum(l, hit, r3, &dtl, &dist, &dpdf, &epdf, &cal);
    if (cblack(illu)) return res;
    float bdp, brp, cosTo;
    c3 f = bsdf_f(b, s->mats, dtl, &cosTo, &bdp, &brp);
    if (cblack(f)) return res;
    float cp = b->cont;
    bdp *= cp;  /* AreaLight is not delta */
    brp *= cp;
    float wl = bdp / (lpp * dpdf);
    float wc = (epdf * cosTo / (dpdf * cal)) * (c->mis_vm + cs->dVCM + cs->dVC * brp);
    float w = 1.f / (wl + 1.f + wc);
    res = cscale(cmul(illu, f), w * cosTo / (lpp * dpdf));
    if (cblack(res) || occluded(s, hit, dtl, vadd(hit, vscale(dtl, dist)), c->st)) return C0;
    return res;
}

static c3 vcm_connect(vcm_ctx* c, const vstate* ls, const bsdf_t* cb, v3 hit, const vstate* cs) { /* :575-636 */
    const cr_scene* s = c->s;
    v3 dir = vsub(ls->pos, hit);
    float d2 = vsqr(dir);
    float dist = sqrtf(d2);
    dir = vdiv(dir, dist);
    c3 res = C0;
    float cosC, cdp, crp;
    c3 cf = bsdf_f(cb, s->mats, dir, &cosC, &cdp, &crp);
    if (cblack(cf)) return res;
    float ccp = cb->cont;
    cdp *= ccp;
    crp *= ccp;
    float cosL, ldp, lrp;
    c3 lf = bsdf_f(&ls->bsdf, s->mats, vneg(dir), &cosL, &ldp, &lrp);
    if (cblack(lf)) return res;
    float lcp = ls->bsdf.cont;
    ldp *= lcp;
    lrp *= lcp;
    float G = cosL * cosC / d2;
    if (cmpf(G) < 0) return res;
    float cdpa = cdp * fabsf(cosL) / (dist * dist);  /* pdfWtoA (math.cpp:13-16) */
    float ldpa = ldp * fabsf(cosC) / (dist * dist);
    float wl = cdpa * (c->mis_vm + ls->dVCM + ls->dVC * lrp);
    float wc = ldpa * (c->mis_vm + cs->dVCM + cs->dVC * crp);
    float w = 1.f / (wl + 1.f + wc);
    res = cscale(cscale(cmul(cf, lf), w), G);
    if (cblack(res) || occluded(s, hit, dir, vadd(hit, vscale(dir, dist)), c->st)) return C0;
    return res;
}

static void vcm_push(vcm_ctx* c, const vstate* v) {
    if (c->nlv >= c->cap_lv) { c->cap_lv = c->cap_lv ? 2 * c->cap_lv : 4096;
        c->lv = (vstate*)realloc(c->lv, (size_t)c->cap_lv * sizeof(vstate)); }
    c->lv[c->nlv++] = *v;
}

/* VertexCM::runIteration (:47-285) for iteration index `it` (radius schedule)
 * with the RNG of global iteration `key_iter` (counter mode). */
static void vcm_iteration(vcm_ctx* c, mt_state* mt, int mode, uint32_t seed, int it, uint32_t key_iter,
                          float base_radius, float alpha, int64_t pb, int64_t pe) {
    const cr_scene* s = c->s;
    const camera_t* cam = &s->cam;
    float radius = base_radius;
    radius /= powf((float)(it + 1), 0.5f * (1.f - alpha));
    radius = fmaxs(radius, R_EPS);
    float r2 = radius * radius;
    c->radius = radius;
    c->vm_norm = 1.f / (r2 * R_PI * c->N);
    float eta = (R_PI * r2) * c->N;
    c->mis_vm = eta;
    c->mis_vc = 1.f / eta;
    memset(c->ends, 0, sizeof(int) * (size_t)c->P);
    c->nlv = 0;
    rng_t rng;
    bsdf_t stale;
    memset(&stale, 0, sizeof stale);
    /* light pass (:74-140) */
    for (int64_t pi = pb; pi < pe; pi++) {
        rng_for(&rng, mode, mt, seed, key_iter, 0, (uint32_t)pi);
        vstate ls;
        memset(&ls, 0, sizeof ls);
        vcm_gen_light(c, &rng, &ls);
        for (;; ls.len++) {
            ray_t ray = mkray(vadd(ls.origin, vscale(ls.dir, R_EPS)), ls.dir);
            hit_t h;
            if (intersect(s, &ray, &h, c->st) < 0) break;
            v3 hp = h.p;
            bsdf_t b;
            bsdf_init(&b, vneg(ray.d), &h, s->mats);
            if (b.matId == 0) break;
            if (b.matId < 0) {
                /* An emitter hit: BSDF::init skips calcComponentProb (bsdf.h:78-83), so
                 * componentProb / continueProb / fresnelReflect keep whatever the
                 * stack slot of `BSDF bsdf` (:90) held -- the previous BSDF built in
                 * this loop, in path order (pinned against refdrv, which matches it
                 * bit for bit).  isDelta is then computed from those, and a
                 * non-delta emitter vertex is stored and merged (vertexcm.h:77-78
                 * reads its continueProb).  On a path's first vertex that is the
                 * last BSDF of an EARLIER light path: pinned on the tent-luminaire
                 * fixtures (~500 such vertices per iteration).  Iteration start: a
                 * zeroed slot.  The reference reads uninitialized memory here
                 * (undefined behaviour): one refdrv build differs from this model by
                 * 1 ulp in 232 film values of tent64 x3 iterations (seed 7, radius
                 * factor 0.1), while the same objects relinked with an extra call
                 * before render() -- or called per iteration -- match it bit for bit. */
                b.pd = stale.pd; b.pg = stale.pg; b.pr = stale.pr; b.pt = stale.pt;
                b.cont = stale.cont; b.fres = stale.fres;
                b.delta = (cmpf(b.pd) == 0 && cmpf(b.pg) == 0);
                if (ls.len == 1 && c->st) c->st->vm_emitter_first++;
            }
            stale = b;
            /* `pathLength > 1 || isFiniteLight == 1` (:94-95): isFiniteLight is a signed
             * 1-bit field (vertexcm.h:31), so storing true reads back as -1 and only
             * pathLength > 1 scales -- unlike BDPT, whose flag is a plain int */
            if (ls.len > 1) ls.dVCM *= (h.t * h.t);
            ls.dVCM /= fabsf(b.wi.z);
            ls.dVC /= fabsf(b.wi.z);
            ls.dVM /= fabsf(b.wi.z);
            ls.pos = hp;
            ls.bsdf = b;
            if (!b.delta) vcm_push(c, &ls);
            if (!b.delta && ls.len + 1 >= c->minlen) {
                v3 ip = x_point(&cam->w2r, hp);
                if (cam_check(cam, ip.x, ip.y)) {
                    c3 r = vcm_connect_camera(c, &ls, hp, &b);
                    film_add(c->film, c->H, c->W, (int)ip.x, (int)ip.y, r);
                }
            }
            if (ls.len + 2 > c->maxlen) break;
            if (!vcm_scatter(c, &rng, &b, hp, &ls)) break;
        }
        c->ends[pi] = (int)c->nlv;
    }
    /* vertex kd-tree (:152) */
    c->nnodes = c->nlv;
    c->next_node = 1;
    if (c->nlv > 0) {
        c->nodes = (vkd_node*)realloc(c->nodes, (size_t)c->nlv * sizeof(vkd_node));
        c->node_vert = (int*)realloc(c->node_vert, (size_t)c->nlv * sizeof(int));
        c->idx = (int*)realloc(c->idx, (size_t)c->nlv * sizeof(int));
        for (int64_t i = 0; i < c->nlv; i++) c->idx[i] = (int)i;
        vkd_build(c, 0, 0, (int)c->nlv);
    }
    /* camera pass (:157-283) */
    for (int64_t pi = pb; pi < pe; pi++) {
        rng_for(&rng, mode, mt, seed, key_iter, 1, (uint32_t)pi);
        vstate cs;
        memset(&cs, 0, sizeof cs);
        int y = (int)(pi % c->W), x = (int)(pi / c->W);  /* generateCameraSample (:446-479) */
        v3 jit = rng_v3(&rng);
        v3 smp = mk((float)x + jit.x, (float)y + jit.y, 0.f);
        v3 rp = x_point(&cam->r2w, mk(smp.x, smp.y, 0));
        ray_t cr = mkray(cam->pos, vsub(rp, cam->pos));
        float cosAt = vdot(cam->fwd, cr.d);
        float ipd = cam->plane_dist / cosAt;
        float i2sa = (ipd * ipd) / cosAt;
        cs.origin = cr.o;
        cs.dir = cr.d;
        cs.thr = mkc(1, 1, 1);
        cs.len = 1;
        cs.dVCM = c->N / i2sa;
        cs.dVC = 0.f;
        cs.dVM = 0.f;
        c3 color = C0;
        for (;; cs.len++) {
            ray_t ray = mkray(vadd(cs.origin, vscale(cs.dir, R_EPS)), cs.dir);
            hit_t h;
            if (intersect(s, &ray, &h, c->st) < 0) break;
            v3 hp = h.p;
            bsdf_t b;
            bsdf_init(&b, vneg(ray.d), &h, s->mats);
            if (b.matId == 0) break;
            cs.dVCM *= (h.t * h.t);
            cs.dVCM /= fabsf(b.wi.z);
            cs.dVC /= fabsf(b.wi.z);
            cs.dVM /= fabsf(b.wi.z);
            if (h.matId < 0) {  /* getLightRadiance (:481-514) == BDPT's */
                const light_t* l = &s->lights[-h.matId - 1];
                if (cs.len >= c->minlen) {
                    float lpp = 1.f / (float)s->nlights;
                    float dpa, ep;
                    c3 r = light_radiance(l, ray.d, &dpa, &ep);
                    if (!cblack(r)) {
                        if (cs.len != 1) {
                            dpa *= lpp;
                            ep *= lpp;
                            float wc = dpa * cs.dVCM + ep * cs.dVC;
                            r = cscale(r, 1.f / (1.f + wc));
                        }
                        color = cadd(color, cmul(cs.thr, r));
                    }
                }
                break;
            }
            if (cs.len >= c->maxlen) break;
            if (!b.delta && cs.len + 1 >= c->minlen)
                color = cadd(color, cmul(cs.thr, vcm_direct(c, &rng, &cs, hp, &b)));
            if (!b.delta) {
                int st0 = pi == 0 ? 0 : c->ends[pi - 1], ed = c->ends[pi];
                for (int i = st0; i < ed; i++) {
                    const vstate* lsv = &c->lv[i];
                    if (lsv->len + 1 + cs.len < c->minlen) continue;
                    if (lsv->len + 1 + cs.len > c->maxlen) break;
                    c3 tmp = vcm_connect(c, lsv, &b, hp, &cs);
                    color = cadd(color, cmul(cmul(cs.thr, lsv->thr), tmp));
                }
            }
            if (!b.delta && c->nlv > 0) {  /* vertex merging (:265-276) */
                vquery q = {&b, &cs, C0};
                if (c->st) c->st->vm_queries++;
                vkd_search(c, 0, hp, radius, &q);
                color = cadd(color, cscale(cmul(cs.thr, q.contrib), c->vm_norm));
            }
            if (!vcm_scatter(c, &rng, &b, hp, &cs)) break;
        }
        film_add(c->film, c->H, c->W, (int)smp.x, (int)smp.y, color);
    }
}

int cr_render_vcm(const cr_scene* s, int W, int H, int iter_begin, int iterations, uint32_t seed,
                  int rng_mode, int min_path_length, int max_path_length, float radius_factor,
                  float radius_alpha, int64_t path_begin, int64_t path_end, float* film, cr_stats* st) {
    init_consts();
    if (!s || s->nprims == 0 || s->nlights == 0) { set_err("scene has no geometry or lights", NULL); return -1; }
    vcm_ctx c;
    memset(&c, 0, sizeof c);
    c.s = s; c.W = W; c.H = H; c.P = W * H;
    c.minlen = min_path_length;
    c.maxlen = max_path_length;
    c.N = (float)(H * W);
    c.film = film; c.st = st;
    c.ends = (int*)calloc((size_t)c.P, sizeof(int));
    if (path_end > c.P) path_end = c.P;
    float base_radius = radius_factor * s->ssph.radius;  /* VertexCM::init (:13) */
    mt_state mt;
    mt_seed(&mt, seed);
    double t0 = now_s();
    for (int it = 0; it < iterations; it++)
        vcm_iteration(&c, &mt, rng_mode, seed, iter_begin + it, (uint32_t)(iter_begin + it), base_radius,
                      radius_alpha, path_begin, path_end);
    if (st) st->seconds += now_s() - t0;
    free(c.ends); free(c.lv); free(c.nodes); free(c.node_vert); free(c.idx);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* PathIntegrator (pathIntegrator.cpp:29-148) + SurfaceIntegrator::render      */
/* ------------------------------------------------------------------------- */
static c3 pt_trace(const cr_scene* s, rng_t* rng, ray_t r, int max_depth, cr_stats* st) {
    c3 pw = mkc(1.f, 1.f, 1.f), res = C0;
    int plen = 1, last_spec = 1;
    float last_pdf = 1.f;
    float lpp = 1.f / (float)s->nlights;
    hit_t h;
    for (;; plen++) {
        if (intersect(s, &r, &h, st) < 0) break;
        v3 hp = h.p;
        bsdf_t b;
        bsdf_init(&b, vneg(r.d), &h, s->mats);
        if (b.matId == 0) break;
        if (b.matId < 0) {
            const light_t* l = &s->lights[-b.matId - 1];
            float dpa;
            c3 contrib = light_radiance(l, r.d, &dpa, NULL);
            if (cblack(contrib)) break;
            float mw = 1.f;
            if (plen > 1 && !last_spec) {
                float dp = dpa * (h.t * h.t) / fabsf(b.wi.z);
                mw = last_pdf / (last_pdf + dp * lpp);
            }
            res = cadd(res, cscale(cmul(pw, contrib), mw));
            break;
        }
        if (plen > max_depth) break;
        if (cmpf(b.cont) == 0) break;
        if (!b.delta) {
            int id = (int)(rng_f(rng) * (float)s->nlights);
            const light_t* l = &s->lights[id];
            v3 dtl;
            float dist, dpdf;
            v3 r3 = rng_v3(rng);
            c3 illu = light_illum(l, hp, r3, &dtl, &dist, &dpdf, NULL, NULL);
            if (!cblack(illu) &&
                !occluded(s, vadd(hp, vscale(dtl, R_EPS)), dtl, vadd(hp, vscale(dtl, dist - R_EPS)), st)) {
                float bp, cw;
                c3 bf = bsdf_f(&b, s->mats, dtl, &cw, &bp, NULL);
                if (!cblack(bf)) {
                    float w = 1.f;
                    float cp = b.cont;
                    bp *= cp;
                    w = (dpdf * lpp) / ((dpdf * lpp) + bp);
                    c3 contrib = cscale(cmul(illu, bf), w * cw / (lpp * dpdf));
                    res = cadd(res, cmul(contrib, pw));
                }
            }
        }
        float pdf, cw;
        int type;
        v3 r3 = rng_v3(rng);
        c3 bf = bsdf_sample(&b, s->mats, r3, &r.d, &pdf, &cw, &type);
        if (cblack(bf)) break;
        float cp = b.cont;
        last_spec = (type & T_SPEC) != 0;
        last_pdf = pdf * cp;
        if (cmpf(cp - 1.f) < 0) {
            if (cmpf(rng_f(rng) - cp) > 0) break;
            pdf *= cp;
        }
        pw = cscale(cmul(pw, bf), cw / pdf);
        r.o = vadd(hp, vscale(r.d, R_EPS));  /* r.dir stays un-normalised (:144-145) */
        r.tmin = 0.f;
        r.tmax = R_INF;
    }
    return res;
}

/* Samples [k_begin, k_begin + k_count) of the spp-sample stratification grid,
 * summed into film (no 1/spp scale): one rank's share of a sample-sharded PT
 * render (winmad_rt.dist.pt_sample_range), surfaceIntegrator.cpp:14-46 */
int cr_render_pt_samples(const cr_scene* s, int W, int H, int spp, int k_begin, int k_count, int max_depth,
                         uint32_t seed, int rng_mode, int64_t pix_begin, int64_t pix_end, float* film,
                         cr_stats* st) {
    init_consts();
    if (!s || s->nprims == 0 || s->nlights == 0) { set_err("scene has no geometry or lights", NULL); return -1; }
    if (k_begin < 0 || k_count < 0 || k_begin + k_count > spp) { set_err("bad sample range", NULL); return -1; }
    if (rng_mode != CR_RNG_COUNTER && (k_begin != 0 || k_count != spp)) {
        set_err("sample ranges need the counter RNG", NULL);
        return -1;
    }
    const camera_t* cam = &s->cam;
    mt_state mt;
    mt_seed(&mt, seed);
    rng_t rng;
    if (pix_end > (int64_t)W * H) pix_end = (int64_t)W * H;
    double t0 = now_s();
    for (int64_t pix = pix_begin; pix < pix_end; pix++) {
        int i = (int)(pix / W), j = (int)(pix % W);
        for (int k = k_begin; k < k_begin + k_count; k++) {
            rng_for(&rng, rng_mode, &mt, seed, (uint32_t)k, 2, (uint32_t)pix);
            v3 v0 = mk((float)j - 0.5f, (float)i - 0.5f, 0);
            v3 v1 = mk((float)j + 0.5f, (float)i - 0.5f, 0);
            v3 v2 = mk((float)j - 0.5f, (float)i + 0.5f, 0);
            v3 pr = sample_rect_strat(rng_v3(&rng), v0, v1, v2, k, spp);
            v3 wp = x_point(&cam->r2w, mk(pr.x, pr.y, 0));
            ray_t ray = mkray(cam->pos, vsub(wp, cam->pos));
            c3 v = pt_trace(s, &rng, ray, max_depth, st);
            film_add(film, H, W, i, j, v);
        }
    }
    if (st) st->seconds += now_s() - t0;
    return 0;
}

int cr_render_pt(const cr_scene* s, int W, int H, int spp, int max_depth, uint32_t seed, int rng_mode,
                 int64_t pix_begin, int64_t pix_end, float* film, cr_stats* st) {
    int rc = cr_render_pt_samples(s, W, H, spp, 0, spp, max_depth, seed, rng_mode, pix_begin, pix_end, film, st);
    if (rc) return rc;
    if (pix_end > (int64_t)W * H) pix_end = (int64_t)W * H;
    float inv = 1.f / (float)spp;  /* film->scale(1.f / samplesPerPixel) */
    for (int64_t pix = pix_begin; pix < pix_end; pix++)
        for (int ch = 0; ch < 3; ch++) film[3 * pix + ch] = film[3 * pix + ch] * inv;
    return 0;
}

/* PathIntegrator::raytracing for caller rays (o, d as given), counter RNG
 * stream (seed, sample, 2, k) from its first draw: the check of wr_path_radiance */
int cr_pt_radiance(const cr_scene* s, const float* rays6, int64_t n, int max_depth, uint32_t seed,
                   uint32_t sample, float* out3, cr_stats* st) {
    init_consts();
    if (!s || s->nprims == 0 || s->nlights == 0) { set_err("scene has no geometry or lights", NULL); return -1; }
    rng_t rng;
    for (int64_t k = 0; k < n; k++) {
        rng_for(&rng, CR_RNG_COUNTER, NULL, seed, sample, 2, (uint32_t)k);
        ray_t r = {mk(rays6[6 * k], rays6[6 * k + 1], rays6[6 * k + 2]),
                   mk(rays6[6 * k + 3], rays6[6 * k + 4], rays6[6 * k + 5]), 0.f, R_INF};
        c3 v = pt_trace(s, &rng, r, max_depth, st);
        out3[3 * k] = v.r; out3[3 * k + 1] = v.g; out3[3 * k + 2] = v.b;
    }
    return 0;
}

/* ------------------------------------------------------------------------- */
/* Known-answer hooks                                                         */
/* ------------------------------------------------------------------------- */
void cr_kat_sampler(const float* u, float power, float* o) {
    init_consts();
    float pdf = -1.f;
    v3 a = sample_cos_hemi(mk(u[0], u[1], u[2]), &pdf);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = pdf;
    v3 b = sample_pow_cos_hemi(mk(u[0], u[1], u[2]), power, &pdf);
    o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = pdf;
    o[8] = pow_cos_hemi_pdf(mk(0, 0, 1), b, power);
}
void cr_kat_triangle(const float* u, const float* p, float* o) {
    v3 t = sample_triangle(mk(u[0], u[1], u[2]), mk(p[0], p[1], p[2]), mk(p[3], p[4], p[5]), mk(p[6], p[7], p[8]));
    o[0] = t.x; o[1] = t.y; o[2] = t.z;
}
void cr_kat_frame(const float* z, float* o) {
    frame_t f = frame_from_z(mk(z[0], z[1], z[2]));
    o[0] = f.x.x; o[1] = f.x.y; o[2] = f.x.z; o[3] = f.y.x; o[4] = f.y.y; o[5] = f.y.z;
    o[6] = f.z.x; o[7] = f.z.y; o[8] = f.z.z;
}
float cr_kat_fresnel(float ci, float idx) { return fresnel(ci, idx); }
void cr_kat_strat(const float* u, int k, int tot, float* o) {
    v3 r = sample_rect_strat(mk(u[0], u[1], u[2]), mk(3.f, 4.f, 0.f), mk(4.f, 4.f, 0.f), mk(3.f, 5.f, 0.f), k, tot);
    o[0] = r.x; o[1] = r.y; o[2] = r.z;
}
int cr_kat_bsdf(const cr_scene* s, int matId, const float* n, const float* wi, const float* wo,
                const float* r3, float* o) {
    init_consts();
    hit_t h;
    memset(&h, 0, sizeof h);
    h.n = mk(n[0], n[1], n[2]);
    h.matId = matId;
    h.t = 1.f;
    bsdf_t b;
    bsdf_init(&b, mk(wi[0], wi[1], wi[2]), &h, s->mats);
    if (b.matId == 0) return 0;
    o[0] = (float)b.delta; o[1] = b.wi.z; o[2] = b.cont; o[3] = b.fres;
    o[4] = b.pd; o[5] = b.pg; o[6] = b.pr; o[7] = b.pt;
    float cw = -7.f, dp = -7.f, rp = -7.f;
    c3 f = bsdf_f(&b, s->mats, mk(wo[0], wo[1], wo[2]), &cw, &dp, &rp);
    o[8] = f.r; o[9] = f.g; o[10] = f.b; o[11] = cw; o[12] = dp; o[13] = rp;
    o[14] = bsdf_pdf(&b, s->mats, mk(wo[0], wo[1], wo[2]), 0);
    o[15] = bsdf_pdf(&b, s->mats, mk(wo[0], wo[1], wo[2]), 1);
    v3 ow = mk(-7.f, -7.f, -7.f);
    float sp = -7.f, sc = -7.f;
    int ty = -7;
    c3 sv = bsdf_sample(&b, s->mats, mk(r3[0], r3[1], r3[2]), &ow, &sp, &sc, &ty);
    o[16] = (float)ty; o[17] = sv.r; o[18] = sv.g; o[19] = sv.b;
    o[20] = ow.x; o[21] = ow.y; o[22] = ow.z; o[23] = sp; o[24] = sc;
    return 1;
}
void cr_kat_light(const cr_scene* s, int li, const float* pos, const float* r3, const float* dr,
                  const float* pr, const float* rd, float* o) {
    init_consts();
    const light_t* l = &s->lights[li];
    v3 dtl;
    float dist = -7.f, dp = -7.f, ep = -7.f, cal = -7.f;
    c3 il = light_illum(l, mk(pos[0], pos[1], pos[2]), mk(r3[0], r3[1], r3[2]), &dtl, &dist, &dp, &ep, &cal);
    o[0] = il.r; o[1] = il.g; o[2] = il.b; o[3] = dtl.x; o[4] = dtl.y; o[5] = dtl.z;
    o[6] = dist; o[7] = dp; o[8] = ep; o[9] = cal;
    v3 p, d;
    float emp = -7.f, dpa = -7.f, cal2 = -7.f;
    c3 em = light_emit(l, mk(dr[0], dr[1], dr[2]), mk(pr[0], pr[1], pr[2]), &p, &d, &emp, &dpa, &cal2);
    o[10] = em.r; o[11] = em.g; o[12] = em.b; o[13] = p.x; o[14] = p.y; o[15] = p.z;
    o[16] = d.x; o[17] = d.y; o[18] = d.z; o[19] = emp; o[20] = dpa; o[21] = cal2;
    float gpa = -7.f, gep = -7.f;
    c3 gr = light_radiance(l, mk(rd[0], rd[1], rd[2]), &gpa, &gep);
    o[22] = gr.r; o[23] = gr.g; o[24] = gr.b; o[25] = gpa; o[26] = gep;
}
void cr_kat_camera(const cr_scene* s, float x, float y, const float* w, float* o) {
    init_consts();
    const camera_t* c = &s->cam;
    v3 p = x_point(&c->r2w, mk(x, y, 0));
    ray_t r = mkray(c->pos, vsub(p, c->pos));
    v3 ras = x_point(&c->w2r, mk(w[0], w[1], w[2]));
    o[0] = r.o.x; o[1] = r.o.y; o[2] = r.o.z; o[3] = r.d.x; o[4] = r.d.y; o[5] = r.d.z;
    o[6] = ras.x; o[7] = ras.y; o[8] = ras.z; o[9] = (float)cam_check(c, ras.x, ras.y);
}
