/* TEST INFRASTRUCTURE ONLY -- C port of the CPU oracle (oracle/cotix_oracle).
 *
 * A transliteration of the Python restatement, itself citing the reference
 * (cotix/_colliders.py, _contacts.py, _collisions.py, _collision_resolution.py,
 * _physics_solvers.py, _lunar_lander.py, examples/test_viz.py).  Like the
 * Python oracle it runs the reference's algorithm faithfully: the full
 * N1 x N2 candidate cross product in the reference's scan order, one
 * bernoulli per non-NaN candidate, "last write wins".  Used as (a) the timed
 * CPU baseline of bench.py (OpenMP over envs) and (b) a fast checker for the
 * GPU tests at large batch sizes.  Never linked into the product.
 *
 * Numerics: IEEE f32, no contraction (-ffp-contract=off), same op order as
 * the Python oracle; deterministic sin/cos/atan2 (cephes) as in the oracle.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct { float x, y; } V2;
static inline V2 v2(float x, float y) { V2 r = {x, y}; return r; }
static inline V2 vadd(V2 a, V2 b) { return v2(a.x + b.x, a.y + b.y); }
static inline V2 vsub(V2 a, V2 b) { return v2(a.x - b.x, a.y - b.y); }
static inline V2 vneg(V2 a) { return v2(-a.x, -a.y); }
static inline V2 vscale(V2 a, float s) { return v2(a.x * s, a.y * s); }
static inline V2 vdivs(V2 a, float s) { return v2(a.x / s, a.y / s); }
static inline float dot(V2 a, V2 b) { return a.x * b.x + a.y * b.y; }
static inline float cross(V2 a, V2 b) { return a.x * b.y - a.y * b.x; }
static inline float sumsq(V2 a) { return a.x * a.x + a.y * a.y; }
static inline float norm(V2 a) { return sqrtf(sumsq(a)); }
static inline int isn(float x) { return x != x; }
static inline int vnan(V2 a) { return isn(a.x) || isn(a.y); }
static inline V2 fnormal(V2 a) { return v2(-a.y, a.x); }
static inline float fmax_(float a, float b) { return isn(a) ? a : (isn(b) ? b : (a >= b ? a : b)); }
static inline float fmin_(float a, float b) { return isn(a) ? a : (isn(b) ? b : (a <= b ? a : b)); }
static inline float clip_(float x, float lo, float hi) { return fmin_(hi, fmax_(lo, x)); }
static inline float qnan(void) { return __builtin_nanf(""); }
static inline float bitsf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

static int argmin_(const float* v, int n) {
  for (int k = 0; k < n; ++k) if (isn(v[k])) return k;
  int b = 0;
  for (int k = 1; k < n; ++k) if (v[k] < v[b]) b = k;
  return b;
}
static int argmax_(const float* v, int n) {
  for (int k = 0; k < n; ++k) if (isn(v[k])) return k;
  int b = 0;
  for (int k = 1; k < n; ++k) if (v[k] > v[b]) b = k;
  return b;
}

/* ---------------- deterministic transcendentals ---------------- */
static float sin_poly(float r) { float z = r * r; return (((-1.9515295891e-4f * z + 8.3321608736e-3f) * z + -1.6666654611e-1f) * z) * r + r; }
static float cos_poly(float r) {
  float z = r * r;
  return ((((2.443315711809948e-5f * z + -1.388731625493765e-3f) * z + 4.166664568298827e-2f) * z) * z - 0.5f * z) + 1.0f;
}
static void sincos32(float x, float* so, float* co) {
  if (isn(x) || isinf(x)) { *so = qnan(); *co = qnan(); return; }
  float t = x * 0.636619772367581343f;
  float k = (t + 12582912.0f) - 12582912.0f;
  float r = ((x - k * 1.5703125f) - k * 4.837512969970703125e-4f) - k * 7.54978995489188216e-8f;
  float s = sin_poly(r), c = cos_poly(r);
  int q = ((int)k) & 3;
  if (q == 0) { *so = s; *co = c; } else if (q == 1) { *so = c; *co = -s; }
  else if (q == 2) { *so = -s; *co = -c; } else { *so = -c; *co = s; }
}
static float atan01(float t) {
  float y0 = 0.0f;
  if (t > 0.4142135623730950f) { y0 = 0.785398163397448309616f; t = (t - 1.0f) / (t + 1.0f); }
  float z = t * t;
  return y0 + (((((8.05374449538e-2f * z + -1.38776856032e-1f) * z + 1.99777106478e-1f) * z + -3.33329491539e-1f) * z) * t + t);
}
static float atan2_32(float y, float x) {
  const float PI = 3.14159265358979323846f, PIO2 = 1.57079632679489661923f;
  if (isn(x) || isn(y)) return qnan();
  if (y == 0.0f) {
    if (x > 0.0f || (x == 0.0f && !signbit(x))) return y;
    return signbit(y) ? -PI : PI;
  }
  if (x == 0.0f) return y < 0.0f ? -PIO2 : PIO2;
  float ax = fabsf(x), ay = fabsf(y);
  float r = (ay <= ax) ? atan01(ay / ax) : (PIO2 - atan01(ax / ay));
  if (x < 0.0f) r = PI - r;
  return y < 0.0f ? -r : r;
}
static int sort_lt(float a, float b) { if (isn(a)) return 0; if (isn(b)) return 1; return a < b; }
static void order_clockwise(V2* v, int n) {
  float sx = 0.0f, sy = 0.0f;
  for (int k = 0; k < n; ++k) { sx = sx + v[k].x; sy = sy + v[k].y; }
  float mx = sx / (float)n, my = sy / (float)n;
  float ang[16];
  for (int k = 0; k < n; ++k) ang[k] = atan2_32(v[k].y - my, v[k].x - mx);
  for (int k = 1; k < n; ++k) {  /* stable insertion sort */
    float a = ang[k]; V2 p = v[k]; int j = k - 1;
    while (j >= 0 && sort_lt(a, ang[j])) { ang[j + 1] = ang[j]; v[j + 1] = v[j]; --j; }
    ang[j + 1] = a; v[j + 1] = p;
  }
}

/* ---------------- threefry / jax.random (legacy and partitionable layouts) ---------------- */
typedef struct { uint32_t a, b; } K2;
static inline uint32_t rotl(uint32_t v, int r) { return (v << r) | (v >> (32 - r)); }
static K2 threefry(K2 k, uint32_t x0, uint32_t x1) {
  static const int R[2][4] = {{13, 15, 26, 6}, {17, 29, 16, 24}};
  uint32_t ks[3] = {k.a, k.b, k.a ^ k.b ^ 0x1BD11BDAu};
  x0 += ks[0]; x1 += ks[1];
  for (int g = 0; g < 5; ++g) {
    for (int i = 0; i < 4; ++i) { x0 += x1; x1 = rotl(x1, R[g & 1][i]); x1 ^= x0; }
    x0 += ks[(g + 1) % 3]; x1 += ks[(g + 2) % 3] + (uint32_t)(g + 1);
  }
  K2 r = {x0, x1}; return r;
}
/* split(key, num) -> out[num] (counters iota(2*num)) */
static void split_n(K2 k, uint32_t num, K2* out) {
  for (uint32_t b = 0; b < num; ++b) {
    K2 y = threefry(k, b, num + b);
    /* flat = y0[0..num) || y1[0..num); key q = (flat[2q], flat[2q+1]) */
    uint32_t m0 = b, m1 = num + b;
    ((uint32_t*)out)[m0] = y.a;
    ((uint32_t*)out)[m1] = y.b;
  }
}
/* the partitionable layout (jax_threefry_partitionable=True): split(k, n)[i] =
 * threefry(k, (0, i)); a 32-bit random_bits word m = y0 ^ y1 of threefry(k, (0, m)) */
static void split_nl(K2 k, uint32_t num, K2* out, int part) {
  if (!part) { split_n(k, num, out); return; }
  for (uint32_t i = 0; i < num; ++i) out[i] = threefry(k, 0u, i);
}
static K2 split0l(K2 k, int part) { K2 o[2]; split_nl(k, 2, o, part); return o[0]; }
static float unit_float(uint32_t bits) { uint32_t u = (bits >> 9) | 0x3F800000u; float f; memcpy(&f, &u, 4); return f - 1.0f; }
static uint32_t bits1l(K2 k, int part) { K2 r = threefry(k, 0u, 0u); return part ? (r.a ^ r.b) : r.a; }
static void cumsum_assoc(const float* x, int n, float* out) {
  if (n < 2) { if (n == 1) out[0] = x[0]; return; }
  int m = n / 2;
  float red[16], odd[16], even[17];
  for (int k = 0; k < m; ++k) red[k] = x[2 * k] + x[2 * k + 1];
  cumsum_assoc(red, m, odd);
  int ne = (n % 2 == 0) ? m - 1 : m;
  even[0] = x[0];
  for (int k = 0; k < ne; ++k) even[k + 1] = odd[k] + x[2 * k + 2];
  for (int k = 0; k < n; ++k) out[k] = (k % 2 == 0) ? even[k / 2] : odd[k / 2];
}

/* ---------------- shapes ---------------- */
enum { S_CIRCLE = 0, S_AABB = 1, S_POLY = 2 };
typedef struct { int kind, n; float r; V2 c, lo, up; V2 v[8]; } Shape;
static V2 support(const Shape* s, V2 d) {
  if (s->kind == S_CIRCLE) { float n = norm(d); V2 nd = v2(d.x / n, d.y / n); return v2(nd.x * s->r + s->c.x, nd.y * s->r + s->c.y); }
  if (s->kind == S_AABB) return v2(d.x >= 0.0f ? s->up.x : s->lo.x, d.y >= 0.0f ? s->up.y : s->lo.y);
  if (vnan(d)) return v2(qnan(), qnan());
  float dots[8];
  for (int k = 0; k < s->n; ++k) dots[k] = dot(s->v[k], d);
  return s->v[argmax_(dots, s->n)];
}
static V2 mdiff(const Shape* a, const Shape* b, V2 d) { return vsub(support(a, d), support(b, vneg(d))); }
static int circle_contains(const Shape* s, V2 p) { float r = s->r + 1e-6f; return sumsq(vsub(p, s->c)) <= r * r; }
static int aabb_contains(const Shape* s, V2 p) {
  return p.x >= s->lo.x - 1e-6f && p.y >= s->lo.y - 1e-6f && p.x <= s->up.x + 1e-6f && p.y <= s->up.y + 1e-6f;
}
static float signf_(float x) { return isn(x) ? x : (x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : x)); }
static int poly_contains(const Shape* s, V2 p) {
  float s0 = 0.0f; int ok = 1;
  for (int k = 0; k < s->n; ++k) {
    V2 e0 = s->v[k], e1 = s->v[k == 0 ? s->n - 1 : k - 1];
    float sg = signf_(dot(vsub(p, e0), fnormal(vsub(e0, e1))));
    if (k == 0) s0 = sg; else ok = ok && (sg == s0);
  }
  return ok && !isn(s0);
}
static int contains(const Shape* s, V2 p) {
  return s->kind == S_CIRCLE ? circle_contains(s, p) : (s->kind == S_AABB ? aabb_contains(s, p) : poly_contains(s, p));
}

typedef struct { V2 pen, cp; } Contact;
static Contact nan_contact(void) { Contact c = {{0.0f, 0.0f}, {qnan(), qnan()}}; return c; }

static Contact aabb_vs_aabb(const Shape* a, const Shape* b) {
  if (a->up.y <= b->lo.y || a->up.x <= b->lo.x || a->lo.y >= b->up.y || a->lo.x >= b->up.x) return nan_contact();
  float me = -1e-8f;
  float dep[4] = {fmax_(a->up.y - b->lo.y, me), fmax_(b->up.y - a->lo.y, me), fmax_(a->up.x - b->lo.x, me), fmax_(b->up.x - a->lo.x, me)};
  const float dx[4] = {0, 0, -1, 1}, dy[4] = {-1, 1, 0, 0};
  int k = argmin_(dep, 4);
  float md = fmax_(0.0f, dep[k]);
  Contact c;
  c.pen = v2(md * dx[k], md * dy[k]);
  c.cp = vdivs(vadd(v2(fmin_(a->up.x, b->up.x), fmin_(a->up.y, b->up.y)), v2(fmax_(a->lo.x, b->lo.x), fmax_(a->lo.y, b->lo.y))), 2.0f);
  return c;
}
static Contact circle_vs_circle(const Shape* a, const Shape* b) {
  V2 delta = vsub(a->c, b->c);
  float dist = norm(delta);
  V2 dir = dist == 0.0f ? v2(1.0f, 0.0f) : vdivs(delta, dist);
  V2 pen = vscale(dir, fmin_(dist - (a->r + b->r), 0.0f));
  V2 cp = vdivs(vadd(vadd(b->c, vscale(dir, b->r - a->r)), a->c), 2.0f);
  if (!(dot(vsub(a->c, cp), vsub(b->c, cp)) <= 0.0f)) cp = circle_contains(a, b->c) ? b->c : a->c;
  if (dist <= a->r + b->r) { Contact c = {vneg(pen), cp}; return c; }
  return nan_contact();
}
static Contact circle_vs_aabb(const Shape* a, const Shape* b, uint32_t* err) {
  V2 bc = v2((b->lo.x + b->up.x) / 2.0f, (b->lo.y + b->up.y) / 2.0f);
  V2 disp = vsub(a->c, bc), l = vsub(b->lo, bc), h = vsub(b->up, bc);
  V2 ccp = vadd(bc, v2(clip_(disp.x, l.x, h.x), clip_(disp.y, l.y, h.y)));
  if (!aabb_contains(b, ccp)) { *err |= 1u; ccp = v2(qnan(), qnan()); }
  V2 vs[4] = {b->lo, v2(b->lo.x, b->up.y), b->up, v2(b->up.x, b->lo.y)};
  int perfect = 0;
  for (int k = 0; k < 4; ++k) perfect = perfect || (norm(vsub(vs[k], ccp)) < 1e-6f);
  if (!circle_contains(a, ccp)) return nan_contact();
  Contact c;
  if (perfect) {
    V2 d = vsub(ccp, a->c), dn = vdivs(d, norm(d));
    c.pen = vneg(vsub(vadd(a->c, vscale(dn, a->r)), ccp));
    c.cp = ccp;
    return c;
  }
  float r = a->r;
  float sh[4] = {(a->c.y + r) - b->lo.y, b->up.y - (a->c.y - r), (a->c.x + r) - b->lo.x, b->up.x - (a->c.x - r)};
  const float dx[4] = {0, 0, 1, -1}, dy[4] = {1, -1, 0, 0};
  int k = argmin_(sh, 4);
  float ns = -sh[k];
  c.pen = v2(ns * dx[k], ns * dy[k]);
  c.cp = ccp;
  return c;
}

/* GJK / EPA */
static int in_tri0(V2 v1, V2 v2_, V2 v3) {
  V2 p = v2(0.0f, 0.0f);
#define SGN(p1, p2, p3) (((p1).x - (p3).x) * ((p2).y - (p3).y) - ((p2).x - (p3).x) * ((p1).y - (p3).y))
  float d1 = SGN(p, v1, v2_), d2 = SGN(p, v2_, v3), d3 = SGN(p, v3, v1);
#undef SGN
  int neg = d1 < 0 || d2 < 0 || d3 < 0, pos = d1 > 0 || d2 > 0 || d3 > 0;
  return !(neg && pos);
}
/* narrow-phase parameters (cotix_params): GJK steps, EPA iteration cap of the
 * polygon contacts, circle x polygon's EPA iterations */
typedef struct { V2 d0; int gjk_steps, epa_cap, epa_cp; } NP;
static int gjk(const Shape* a, const Shape* b, V2 d0, V2* s, int max_steps) {
  V2 s0 = mdiff(a, b, d0), s1 = mdiff(a, b, vneg(s0));
  V2 dir = fnormal(vsub(s1, s0));
  if (dot(dir, vneg(s1)) > 0.0f) { V2 t = s0; s0 = s1; s1 = t; } else dir = vneg(dir);
  V2 s2 = mdiff(a, b, dir);
  for (int step = 0; step < max_steps; ++step) {
    int c1 = dot(s2, dir) <= 0.0f;
    int c2 = dot(fnormal(vsub(s2, s0)), vneg(s2)) < 0.0f;
    int c3 = dot(fnormal(vsub(s1, s2)), vneg(s2)) < 0.0f;
    if (c1 || (c2 && c3)) break;
    V2 c = s2, acn = fnormal(vsub(c, s0)), cbn = fnormal(vsub(s1, c));
    if (dot(acn, vneg(c)) >= 0.0f) { s1 = c; dir = acn; } else { s0 = c; dir = cbn; }
    s2 = mdiff(a, b, dir);
  }
  if (!in_tri0(s0, s1, s2)) { s0 = s1 = s2 = v2(0.0f, 0.0f); }
  float area = cross(vsub(s1, s0), vsub(s2, s0));
  int allzero = s0.x == 0 && s0.y == 0 && s1.x == 0 && s1.y == 0 && s2.x == 0 && s2.y == 0;
  s[0] = s0; s[1] = s1; s[2] = s2;
  return !(allzero || vnan(s0) || vnan(s1) || vnan(s2) || area == 0.0f);
}
static V2 closest0(V2 a, V2 b) {
  V2 p = v2(0.0f, 0.0f);
  float len = sumsq(vsub(a, b));
  if (len == 0.0f) return vsub(p, a);
  float t = clip_(dot(vsub(p, b), vsub(a, b)) / len, 0.0f, 1.0f);
  return vsub(p, vadd(b, vscale(vsub(a, b), t)));
}
static float edist(V2 a, V2 b) {
  if (a.x == 0 && a.y == 0 && b.x == 0 && b.y == 0) { float i = INFINITY; return i * i + i * i; }
  V2 p = v2(0.0f, 0.0f);
  float len = sumsq(vsub(a, b));
  float t = clip_(dot(vsub(p, b), vsub(a, b)) / len, 0.0f, 1.0f);
  V2 disp = vsub(p, vadd(b, vscale(vsub(a, b), t)));
  if (len == 0.0f) disp = vneg(a);
  return sumsq(disp);
}
static V2 epa(const Shape* a, const Shape* b, const V2* s, int iters) {
  V2 e0[140], e1[140];
  float dist[140];
  int ne = iters + 3;
  for (int k = 0; k < ne; ++k) { e0[k] = v2(0, 0); e1[k] = v2(0, 0); }
  e0[0] = s[0]; e1[0] = s[1]; e0[1] = s[1]; e1[1] = s[2]; e0[2] = s[2]; e1[2] = s[0];
  for (int k = 0; k < ne; ++k) dist[k] = edist(e0[k], e1[k]);
  int bei = argmin_(dist, ne);
  V2 b0 = e0[bei], b1 = e1[bei], np_ = s[2], p0 = e0[0], p1 = e1[0];
  for (int i = 0; i < iters; ++i) {
    int c1 = sumsq(vsub(b0, b1)) > 1e-9f, c2 = cross(b0, b1) >= 0.0f;
    V2 n = fnormal(vsub(p0, p1));
    n = vdivs(n, norm(n));
    float d = dot(np_, n), ed = norm(closest0(p0, p1));
    int c4 = (d - ed > 1e-6f) || (d <= 0.0f);
    if (!(c4 && !vnan(b0) && !vnan(b1) && c1 && c2)) break;
    n = fnormal(vsub(b0, b1));
    n = vdivs(n, norm(n));
    np_ = mdiff(a, b, n);
    e1[bei] = np_; dist[bei] = edist(b0, np_);
    e0[i + 3] = np_; e1[i + 3] = b1; dist[i + 3] = edist(np_, b1);
    p0 = b0; p1 = b1;
    bei = argmin_(dist, ne);
    b0 = e0[bei]; b1 = e1[bei];
  }
  return closest0(b0, b1);
}
static V2 edge_x(V2 pa0, V2 pa1, V2 qb0, V2 qb1) {
  V2 p = pa0, r = vsub(pa1, pa0), q = qb0, s = vsub(qb1, qb0);
#define C2(u, v) ((u).x * (v).y - (v).x * (u).y)
  float c = C2(r, s);
  float t = C2(vsub(q, p), s) / c, u = C2(vsub(q, p), r) / c;
#undef C2
  if (c != 0.0f && t >= 0.0f && t <= 1.0f && u >= 0.0f && u <= 1.0f) return vadd(p, vscale(r, t));
  return v2(qnan(), qnan());
}
typedef struct { int n; V2 v[8], ea[8], eb[8]; } Edges;
static void edges_of(const Shape* s, Edges* e) {
  if (s->kind == S_AABB) {
    e->n = 4;
    e->v[0] = s->up; e->v[1] = v2(s->up.x, s->lo.y); e->v[2] = s->lo; e->v[3] = v2(s->lo.x, s->up.y);
    for (int k = 0; k < 4; ++k) { e->ea[k] = e->v[k]; e->eb[k] = e->v[(k + 1) & 3]; }
  } else {
    e->n = s->n;
    for (int k = 0; k < s->n; ++k) { e->v[k] = s->v[k]; e->ea[k] = s->v[k]; e->eb[k] = s->v[k == 0 ? s->n - 1 : k - 1]; }
  }
}
static V2 contact_from_edges(const Shape* A, const Edges* ea, const Shape* B, const Edges* eb) {
  float n = 0.0f;
  V2 acc = v2(0.0f, 0.0f);
  for (int k = 0; k < ea->n; ++k) if (contains(B, ea->v[k])) { acc = vadd(acc, ea->v[k]); n = n + 1.0f; }
  for (int k = 0; k < eb->n; ++k) if (contains(A, eb->v[k])) { acc = vadd(acc, eb->v[k]); n = n + 1.0f; }
  for (int jb = 0; jb < eb->n; ++jb)
    for (int ia = 0; ia < ea->n; ++ia) {
      V2 x = edge_x(ea->ea[ia], ea->eb[ia], eb->ea[jb], eb->eb[jb]);
      if (!vnan(x)) { acc = vadd(acc, x); n = n + 1.0f; }
    }
  return n > 0.0f ? vdivs(acc, n) : v2(qnan(), qnan());
}
static Contact convex_vs_polygon(const Shape* A, const Shape* B, const NP* np) {
  V2 s[3];
  if (!gjk(A, B, np->d0, s, np->gjk_steps)) return nan_contact();
  int iters = A->kind == S_AABB ? 4 + B->n + 1 : A->n + B->n + 1;
  if (iters > np->epa_cap) iters = np->epa_cap;
  Contact c;
  c.pen = epa(A, B, s, iters);
  Edges ea, eb;
  edges_of(A, &ea); edges_of(B, &eb);
  c.cp = contact_from_edges(A, &ea, B, &eb);
  return c;
}
static Contact circle_vs_polygon(const Shape* C, const Shape* P, const NP* np) {
  V2 s[3];
  if (!gjk(C, P, np->d0, s, np->gjk_steps)) return nan_contact();
  Contact c;
  c.pen = epa(C, P, s, np->epa_cp);
  float dists[8]; V2 disps[8];
  for (int k = 0; k < P->n; ++k) {
    V2 a = P->v[k], b = P->v[k == 0 ? P->n - 1 : k - 1];
    if (a.x == 0 && a.y == 0 && b.x == 0 && b.y == 0) disps[k] = v2(INFINITY, INFINITY);
    else {
      float len = sumsq(vsub(a, b));
      float t = clip_(dot(vsub(C->c, b), vsub(a, b)) / len, 0.0f, 1.0f);
      disps[k] = vsub(C->c, vadd(b, vscale(vsub(a, b), t)));
    }
    dists[k] = sumsq(disps[k]);
  }
  int k = argmin_(dists, P->n);
  c.cp = vadd(C->c, disps[k]);
  if (dists[k] > C->r * C->r) c.cp = C->c;
  return c;
}
static Contact run_contact(int fn, const Shape* a, const Shape* b, const NP* np, uint32_t* err) {
  switch (fn) {
    case 0: return aabb_vs_aabb(a, b);
    case 1: return circle_vs_circle(a, b);
    case 2: return circle_vs_aabb(a, b, err);
    case 3: case 4: return convex_vs_polygon(a, b, np);
    default: return circle_vs_polygon(a, b, np);
  }
}

/* registry (cotix/_colliders.py:21-35); type ids as include/cotix_amd.h */
static int registry_fn(int ta, int tb) {
  if (ta == 1 && tb == 1) return 0;
  if (ta == 0 && tb == 0) return 1;
  if (ta == 0 && tb == 1) return 2;
  if (ta == 2 && tb == 2) return 3;
  if (ta == 1 && (tb == 2 || tb == 4 || tb == 6)) return 4;
  if (ta == 0 && (tb == 2 || tb == 4 || tb == 6)) return 5;
  if (ta == 4 && (tb == 4 || tb == 6)) return 3;
  if (ta == 6 && tb == 6) return 3;
  return -1;
}

/* ---------------- dynamics ---------------- */
typedef struct { float px, py, vx, vy, a, w; } Dyn;
typedef struct { float m, I, e, f; } Par;
static V2 vel_at(const Dyn* b, V2 p) { V2 r = vsub(p, v2(b->px, b->py)); return v2(b->vx + (-r.y) * b->w, b->vy + r.x * b->w); }
static void apply_impulse(Dyn* b, const Par* m, V2 imp, V2 pt) {
  V2 arm = vsub(pt, v2(b->px, b->py));
  float tq = cross(arm, imp);
  b->vx = b->vx + imp.x / m->m;
  b->vy = b->vy + imp.y / m->m;
  b->w = b->w + tq / m->I;
}
static void resolve(Dyn* b1, const Par* m1, Dyn* b2, const Par* m2, V2 pen, V2 cp, float bk, float bdt) {
  if (vnan(cp)) return;
  V2 relv = vsub(vel_at(b2, cp), vel_at(b1, cp));
  float pn = norm(pen);
  V2 n = v2(pen.x / pn, pen.y / pn);
  float vn = dot(relv, n);
  float e = fmin_(m1->e, m2->e);
  V2 r1 = vsub(cp, v2(b1->px, b1->py)), r2 = vsub(cp, v2(b2->px, b2->py));
  float ang = (r1.x * r1.x + r1.y * r1.y) / m1->I + (r2.x * r2.x + r2.y * r2.y) / m2->I;
  float nim = (-(1.0f + e)) * vn - (bk * norm(pen)) / bdt;
  float ni = nim / ((1.0f / m1->m + 1.0f / m2->m) + ang);
  V2 imp = vscale(n, ni);
  float mu = (m1->f + m2->f) / 2.0f;
  V2 vd = v2(relv.x + vn * n.x, relv.y + vn * n.y);
  float vdn = norm(vd);
  V2 vdu = v2(vd.x / vdn, vd.y / vdn);
  float idr = clip_((-vdn) / ((1.0f / m1->m + 1.0f / m2->m) + ang), 0.0f, ni * mu);
  imp = vadd(imp, vscale(vdu, idr));
  if (dot(pen, relv) < 0.0f) return;
  apply_impulse(b1, m1, vneg(imp), cp);
  apply_impulse(b2, m2, imp, cp);
}
static V2 rotate(V2 v, float a) { float s, c; sincos32(a, &s, &c); return v2(c * v.x + (-s) * v.y, s * v.x + c * v.y); }
static void lunar(Dyn* L, Dyn* R, Dyn* Lg, const Par* pl, const Par* pr, const Par* pg) {
  const float f05 = 0.05f;
  V2 lp = v2(L->px, L->py);
  V2 llj1 = vadd(rotate(v2(24.0f * f05, -8.0f * f05), L->a), lp), llj2 = vadd(rotate(v2(24.0f * f05, 0.0f * f05), L->a), lp);
  V2 lj1 = v2(Lg->px, Lg->py), lj2 = vadd(v2(Lg->px, Lg->py), rotate(v2(0.0f, 0.4f), Lg->a));
  V2 lrj1 = vadd(rotate(v2(-24.0f * f05, -8.0f * f05), L->a), lp), lrj2 = vadd(rotate(v2(-24.0f * f05, 0.0f * f05), L->a), lp);
  V2 rj1 = v2(R->px, R->py), rj2 = vadd(v2(R->px, R->py), rotate(v2(0.0f, 0.4f), R->a));
  Dyn* B1[4] = {L, L, L, L};
  Dyn* B2[4] = {Lg, Lg, R, R};
  const Par* M2[4] = {pg, pg, pr, pr};
  V2 C1[4] = {llj1, llj2, lrj1, lrj2}, C2[4] = {lj1, lj2, rj1, rj2};
  for (int q = 0; q < 4; ++q) {
    V2 dp = vsub(C1[q], C2[q]);
    V2 dv = vsub(vel_at(B1[q], C1[q]), vel_at(B2[q], C2[q]));
    float k = norm(dv) + 0.1f;
    V2 imp = v2(dp.x * 1.0f + (dv.x * k) * f05, dp.y * 1.0f + (dv.y * k) * f05);
    apply_impulse(B1[q], pl, vneg(imp), C1[q]);
    apply_impulse(B2[q], M2[q], imp, C2[q]);
  }
  R->w = R->w * 0.95f;
  Lg->w = Lg->w * 0.95f;
}

/* ---------------- scene + faithful collider ---------------- */
#define MAXB 16
#define MAXP 32
#define MAXN 512
/* cotix_params (include/cotix_amd.h), same field order */
typedef struct { int layout; float baum, baum_dt, p; int gjk_steps, epa_cap, epa_cp, epa_body; } OParams;
typedef struct {
  int nb, np, nt;
  OParams prm;
  Par par[MAXB];
  int pbody[MAXP], ptype[MAXP], pn[MAXP], pgoff[MAXP];
  int tk[13][2], fn[13], n1[13], n2[13];
  int penv, gparts; /* per-env body parameters: [nb][4] words after the parts' geometry (gparts floats) */
  int l1b[13][MAXN], l1p[13][MAXN], l2b[13][MAXN], l2p[13][MAXN];
} OScene;

static int kind_of(int t) { return t == 0 ? S_CIRCLE : (t == 1 ? S_AABB : S_POLY); }

int oracle_scene_size(void) { return (int)sizeof(OScene); }

int oracle_scene_init(void* mem, int nb, const float* params, int np, const int* pbody, const int* ptype, const int* pnv) {
  OScene* s = (OScene*)mem;
  memset(s, 0, sizeof(*s));
  if (nb > MAXB || np > MAXP) return -1;
  OParams d = {0, 0.3f, 0.01f, 0.5f, 32, 48, 128, 48};  /* the reference's literals */
  s->prm = d;
  s->nb = nb; s->np = np;
  for (int b = 0; b < nb; ++b) { s->par[b].m = params[4 * b]; s->par[b].I = params[4 * b + 1]; s->par[b].e = params[4 * b + 2]; s->par[b].f = params[4 * b + 3]; }
  int goff = 0;
  for (int p = 0; p < np; ++p) {
    s->pbody[p] = pbody[p]; s->ptype[p] = ptype[p];
    int n = ptype[p] == 2 ? pnv[p] : (ptype[p] >= 3 ? ptype[p] : 0);
    s->pn[p] = n; s->pgoff[p] = goff;
    goff += ptype[p] <= 1 ? 4 : 2 * n;
  }
  /* enumeration, cotix/_colliders.py:86-113 */
  for (int i = 0; i < nb; ++i)
    for (int j = 0; j < nb; ++j) {
      if (i <= j) continue;
      for (int pa = 0; pa < np; ++pa) {
        if (pbody[pa] != i) continue;
        for (int pb = 0; pb < np; ++pb) {
          if (pbody[pb] != j) continue;
          int t1 = ptype[pa], t2 = ptype[pb], k1, k2;
          if (registry_fn(t1, t2) >= 0) { k1 = t1; k2 = t2; }
          else if (registry_fn(t2, t1) >= 0) { k1 = t2; k2 = t1; }
          else return -2;
          int k = -1;
          for (int q = 0; q < s->nt; ++q) if (s->tk[q][0] == k1 && s->tk[q][1] == k2) k = q;
          if (k < 0) { k = s->nt++; s->tk[k][0] = k1; s->tk[k][1] = k2; s->fn[k] = registry_fn(k1, k2); }
          if (s->n1[k] >= MAXN) return -3;
          s->l1b[k][s->n1[k]] = i; s->l1p[k][s->n1[k]++] = pa;
          s->l2b[k][s->n2[k]] = j; s->l2p[k][s->n2[k]++] = pb;
        }
      }
    }
  return 0;
}

/* a non-default parameter block (scene created by oracle_scene_init first) */
/* every env's own mass, inertia, elasticity, friction per body, read from its
 * geometry row after the parts' words (include/cotix_amd.h
 * COTIX_SCENE_PER_ENV_BODY_PARAMS); returns the geometry floats per env */
int oracle_scene_set_per_env_params(void* mem, int on) {
  OScene* s = (OScene*)mem;
  int goff = 0;
  for (int p = 0; p < s->np; ++p) goff += s->ptype[p] <= 1 ? 4 : 2 * s->pn[p];
  s->penv = on ? 1 : 0;
  s->gparts = goff;
  return goff + (on ? 4 * s->nb : 0);
}

int oracle_scene_set_params(void* mem, const void* params) {
  OScene* s = (OScene*)mem;
  memcpy(&s->prm, params, sizeof(OParams));
  return 0;
}
static V2 d0_of(int part) {
  return part ? v2(bitsf(0xbf607449u), bitsf(0x3ef638cdu)) : v2(bitsf(0xbd56c50bu), bitsf(0x3f7fa5d9u));
}
static NP np_of(const OParams* p) { NP n = {d0_of(p->layout), p->gjk_steps, p->epa_cap, p->epa_cp}; return n; }

static void world_shape(const OScene* s, int p, const Dyn* d, const float* lg, Shape* out) {
  const Dyn* b = &d[s->pbody[p]];
  int t = s->ptype[p];
  out->kind = kind_of(t);
  out->n = s->pn[p];
  if (t == 0) { out->r = lg[0]; out->c = v2(lg[1] + b->px, lg[2] + b->py); }
  else if (t == 1) { out->lo = v2(lg[0] + b->px, lg[1] + b->py); out->up = v2(lg[2] + b->px, lg[3] + b->py); }
  else {
    float s_, c;
    sincos32(b->a, &s_, &c);
    for (int k = 0; k < out->n; ++k) {
      float x = lg[2 * k], y = lg[2 * k + 1];
      float t0 = (c * x + (-s_) * y) + b->px * 1.0f, t1 = (s_ * x + c * y) + b->py * 1.0f;
      float t2 = (0.0f * x + 0.0f * y) + 1.0f * 1.0f;
      out->v[k] = v2(t0 / t2, t1 / t2);
    }
    order_clockwise(out->v, out->n);
  }
}

/* RandomizedCollider.resolve, faithful (forward scan over the full cross product) */
typedef struct { Contact* cur; K2* keys2; K2* keys1; } Work;
/* tr_ch [nb] / tr_cells [nb*nb] (nullable): the chosen partner per body and
 * the winning candidate per cell (ind1 | ind2 << 9 | type << 18, -1 empty) */
static void collider(const OScene* s, const Par* par, Dyn* d, const float* geom, K2 rkey, uint32_t* err, Work* wk,
                     int* tr_ch, int* tr_cells) {
  int nb = s->nb;
  const int part = s->prm.layout;
  const NP np = np_of(&s->prm);
  int win[MAXB][MAXB];
  for (int i = 0; i < nb; ++i) for (int j = 0; j < nb; ++j) win[i][j] = -1;
  Shape world[MAXP];
  for (int p = 0; p < s->np; ++p) world_shape(s, p, d, geom + s->pgoff[p], &world[p]);
  V2 pen[MAXB][MAXB], cp[MAXB][MAXB];
  for (int i = 0; i < nb; ++i) for (int j = 0; j < nb; ++j) { pen[i][j] = v2(0, 0); cp[i][j] = v2(qnan(), qnan()); }
  K2 skey = split0l(rkey, part);
  Contact* cur = wk->cur;
  K2* keys2 = wk->keys2;
  K2* keys1 = wk->keys1;
  for (int k = 0; k < s->nt; ++k) {
    int N1 = s->n1[k], N2 = s->n2[k];
    for (int i1 = 0; i1 < N1; ++i1)
      for (int i2 = 0; i2 < N2; ++i2) {
        const Shape* a = &world[s->l1p[k][i1]];
        const Shape* b = &world[s->l2p[k][i2]];
        if (registry_fn(s->ptype[s->l1p[k][i1]], s->ptype[s->l2p[k][i2]]) < 0) { const Shape* t = a; a = b; b = t; }
        Contact c = run_contact(s->fn[k], a, b, &np, err);
        cur[i1 * N2 + i2] = s->l1b[k][i1] < s->l2b[k][i2] ? nan_contact() : c;
      }
    skey = split0l(skey, part);
    split_nl(skey, (uint32_t)N2, keys2, part);
    for (int i2 = 0; i2 < N2; ++i2) {
      split_nl(keys2[i2], (uint32_t)N1, keys1, part);
      for (int i1 = 0; i1 < N1; ++i1) {
        Contact c = cur[i1 * N2 + i2];
        if (vnan(c.cp)) continue;
        if (unit_float(bits1l(split0l(keys1[i1], part), part)) < s->prm.p) {  /* bernoulli(p): uniform < p */
          int bi = s->l1b[k][i1], bj = s->l2b[k][i2];
          pen[bi][bj] = c.pen; cp[bi][bj] = c.cp;
          win[bi][bj] = i1 | (i2 << 9) | (k << 18);
        }
      }
    }
  }
  K2 ck[MAXB];
  split_nl(skey, (uint32_t)nb, ck, part);
  int ch[MAXB];
  for (int i = 0; i < nb; ++i) {
    int cnt = 0;
    for (int j = 0; j < nb; ++j) cnt += !vnan(cp[i][j]);
    if (cnt == 0) { ch[i] = i; continue; }
    float p[MAXB], c[MAXB];
    for (int j = 0; j < nb; ++j) p[j] = (vnan(cp[i][j]) ? 0.0f : 1.0f) / (float)cnt;
    cumsum_assoc(p, nb, c);
    float u = unit_float(bits1l(ck[i], part));
    float r = c[nb - 1] * (1.0f - u);
    ch[i] = nb;
    for (int j = 0; j < nb; ++j) if (!(c[j] < r)) { ch[i] = j; break; }
  }
  if (tr_ch) for (int i = 0; i < nb; ++i) tr_ch[i] = ch[i];
  if (tr_cells) for (int i = 0; i < nb; ++i) for (int j = 0; j < nb; ++j) tr_cells[i * nb + j] = win[i][j];
  for (int i = 0; i < nb; ++i) {
    int j = ch[i];
    if (j == i || j >= nb) continue;
    resolve(&d[i], &par[i], &d[j], &par[j], pen[i][j], cp[i][j], s->prm.baum, s->prm.baum_dt);
  }
}

/* The driver (examples/test_viz.py), n_steps per env, OpenMP over envs.
 * dyn [nb][6][B]; keys u32 [B][2]; err u32 [B] (OR-ed); geom [G] or [B][gstride];
 * stages as include/cotix_amd.h; dyn_reset nullable (autoreset like the bench). */
static int drive(const void* scene, float* dyn, uint32_t* keys, uint32_t* err, const float* geom, int gstride, int B,
                 int n_steps, float dt, int stages, const float* dyn_reset, uint32_t* resets, const float* action,
                 int action_body, const float* ret_w, float* ret, int32_t* tr_chosen, int32_t* tr_cells,
                 int nthreads) {
  const OScene* s = (const OScene*)scene;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 16)
#endif
  for (int g = 0; g < B; ++g) {
    int nb = s->nb;
    Dyn d[MAXB];
    for (int b = 0; b < nb; ++b) {
      float* q = dyn + (size_t)b * 6 * B + g;
      d[b].px = q[0]; d[b].py = q[(size_t)B]; d[b].vx = q[2 * (size_t)B]; d[b].vy = q[3 * (size_t)B];
      d[b].a = q[4 * (size_t)B]; d[b].w = q[5 * (size_t)B];
    }
    K2 key = {keys[2 * (size_t)g], keys[2 * (size_t)g + 1]};
    int m1 = 1, m2 = 1;
    for (int k = 0; k < s->nt; ++k) { if (s->n1[k] > m1) m1 = s->n1[k]; if (s->n2[k] > m2) m2 = s->n2[k]; }
    Work wk;
    wk.cur = (Contact*)malloc(sizeof(Contact) * (size_t)m1 * m2);
    wk.keys2 = (K2*)malloc(sizeof(K2) * (size_t)(m2 + 1));
    wk.keys1 = (K2*)malloc(sizeof(K2) * (size_t)(m1 + 1));
    uint32_t e = err[g];
    const float* gg = geom + (gstride ? (size_t)g * gstride : 0);
    Par par[MAXB];
    for (int b = 0; b < nb; ++b) {
      par[b] = s->par[b];
      if (s->penv) {  /* the env's own parameters (oracle_scene_set_per_env_params) */
        const float* q = gg + s->gparts + 4 * b;
        par[b].m = q[0]; par[b].I = q[1]; par[b].e = q[2]; par[b].f = q[3];
      }
    }
    for (int t = 0; t < n_steps; ++t) {
      if (stages & 1)
        for (int b = 0; b < nb; ++b) { d[b].px = d[b].px + d[b].vx * dt; d[b].py = d[b].py + d[b].vy * dt; d[b].a = d[b].a + d[b].w * dt; }
      if (stages & 2) { d[0].vx = d[0].vx + 0.0f; d[0].vy = d[0].vy + -0.002f; }
      if (action) {  /* config 5: velocity += action after Euler */
        const float* ac = action + ((size_t)t * B + g) * 2;
        d[action_body].vx = d[action_body].vx + ac[0];
        d[action_body].vy = d[action_body].vy + ac[1];
      }
      if (stages & 4) {
        int tch[MAXB], tcl[MAXB * MAXB];
        collider(s, par, d, gg, key, &e, &wk, tch, tcl);
        if (tr_chosen)
          for (int i = 0; i < nb; ++i) tr_chosen[((size_t)t * nb + i) * B + g] = tch[i];
        if (tr_cells)
          for (int q = 0; q < nb * nb; ++q) tr_cells[((size_t)t * nb * nb + q) * B + g] = tcl[q];
      } else {
        if (tr_chosen) for (int i = 0; i < nb; ++i) tr_chosen[((size_t)t * nb + i) * B + g] = -1;
        if (tr_cells) for (int q = 0; q < nb * nb; ++q) tr_cells[((size_t)t * nb * nb + q) * B + g] = -1;
      }
      if (stages & 8) lunar(&d[0], &d[1], &d[2], &par[0], &par[1], &par[2]);
      if (stages & 16) key = split0l(key, s->prm.layout);
      if (dyn_reset && e) {
        for (int b = 0; b < nb; ++b) {
          const float* q = dyn_reset + (size_t)b * 6 * B + g;
          d[b].px = q[0]; d[b].py = q[(size_t)B]; d[b].vx = q[2 * (size_t)B]; d[b].vy = q[3 * (size_t)B];
          d[b].a = q[4 * (size_t)B]; d[b].w = q[5 * (size_t)B];
        }
        e = 0;
        if (resets) resets[g] += 1;
      }
      if (ret) {  /* return: sum over steps of sum_k w_k * state_k (w_k != 0) */
        float acc = ret[g];
        for (int k = 0; k < nb * 6; ++k) {
          if (ret_w[k] == 0.0f) continue;
          const Dyn* q = &d[k / 6];
          const float x[6] = {q->px, q->py, q->vx, q->vy, q->a, q->w};
          acc = acc + ret_w[k] * x[k % 6];
        }
        ret[g] = acc;
      }
    }
    for (int b = 0; b < nb; ++b) {
      float* q = dyn + (size_t)b * 6 * B + g;
      q[0] = d[b].px; q[(size_t)B] = d[b].py; q[2 * (size_t)B] = d[b].vx; q[3 * (size_t)B] = d[b].vy;
      q[4 * (size_t)B] = d[b].a; q[5 * (size_t)B] = d[b].w;
    }
    keys[2 * (size_t)g] = key.a; keys[2 * (size_t)g + 1] = key.b;
    err[g] = e;
    free(wk.cur); free(wk.keys2); free(wk.keys1);
  }
  return 0;
}

int oracle_step(const void* scene, float* dyn, uint32_t* keys, uint32_t* err, const float* geom, int gstride, int B,
                int n_steps, float dt, int stages, const float* dyn_reset, uint32_t* resets, int nthreads) {
  return drive(scene, dyn, keys, err, geom, gstride, B, n_steps, dt, stages, dyn_reset, resets, NULL, 0, NULL, NULL,
               NULL, NULL, nthreads);
}

/* the step with actions (nullable, [n_steps][B][2]), restarts and the collider
 * trace (chosen [n_steps][nb][B], cells [n_steps][nb][nb][B], both nullable) */
int oracle_step_ex(const void* scene, float* dyn, uint32_t* keys, uint32_t* err, const float* geom, int gstride, int B,
                   int n_steps, float dt, int stages, const float* action, int action_body, const float* dyn_reset,
                   uint32_t* resets, int32_t* chosen, int32_t* cells, int nthreads) {
  return drive(scene, dyn, keys, err, geom, gstride, B, n_steps, dt, stages, dyn_reset, resets, action, action_body,
               NULL, NULL, chosen, cells, nthreads);
}

/* forward of the differentiable rollout: action [n_steps][B][2], ret [B] += */
int oracle_rollout(const void* scene, float* dyn, uint32_t* keys, uint32_t* err, const float* geom, int gstride,
                   int B, int n_steps, float dt, int stages, const float* action, int action_body, const float* ret_w,
                   float* ret, int nthreads) {
  return drive(scene, dyn, keys, err, geom, gstride, B, n_steps, dt, stages, NULL, NULL, action, action_body, ret_w,
               ret, NULL, NULL, nthreads);
}

/* the contact operators; params nullable (the defaults) */
int oracle_contacts_ex(int fn, int n, const float* a, const float* b, float* out, uint32_t* err, const void* params) {
  OParams dp = {0, 0.3f, 0.01f, 0.5f, 32, 48, 128, 48};
  const NP np = np_of(params ? (const OParams*)params : &dp);
  for (int i = 0; i < n; ++i) {
    Shape A, Bs;
    const float* p[2] = {a + 18 * (size_t)i, b + 18 * (size_t)i};
    Shape* S[2] = {&A, &Bs};
    for (int q = 0; q < 2; ++q) {
      S[q]->kind = (int)p[q][0]; S[q]->n = (int)p[q][1];
      if (S[q]->kind == S_CIRCLE) { S[q]->r = p[q][2]; S[q]->c = v2(p[q][3], p[q][4]); }
      else if (S[q]->kind == S_AABB) { S[q]->lo = v2(p[q][2], p[q][3]); S[q]->up = v2(p[q][4], p[q][5]); }
      else for (int k = 0; k < S[q]->n; ++k) S[q]->v[k] = v2(p[q][2 + 2 * k], p[q][3 + 2 * k]);
    }
    uint32_t e = 0;
    Contact c = run_contact(fn, &A, &Bs, &np, &e);
    out[4 * i] = c.pen.x; out[4 * i + 1] = c.pen.y; out[4 * i + 2] = c.cp.x; out[4 * i + 3] = c.cp.y;
    if (err) err[i] = e;
  }
  return 0;
}
int oracle_contacts(int fn, int n, const float* a, const float* b, float* out, uint32_t* err) {
  return oracle_contacts_ex(fn, n, a, b, out, err, NULL);
}

/* check_for_collision_convex / compute_penetration_vector_convex as operators
 * (cotix/_collisions.py:277-329): hit [n], simplex [n][3][2] (NaN * simplex
 * without a collision); EPA from a given simplex with `iters` iterations */
static void load_shape(const float* p, Shape* S) {
  S->kind = (int)p[0]; S->n = (int)p[1];
  if (S->kind == S_CIRCLE) { S->r = p[2]; S->c = v2(p[3], p[4]); }
  else if (S->kind == S_AABB) { S->lo = v2(p[2], p[3]); S->up = v2(p[4], p[5]); }
  else for (int k = 0; k < S->n; ++k) S->v[k] = v2(p[2 + 2 * k], p[3 + 2 * k]);
}
int oracle_gjk(int n, const float* a, const float* b, int32_t* hit, float* simplex, const void* params) {
  OParams dp = {0, 0.3f, 0.01f, 0.5f, 32, 48, 128, 48};
  const NP np = np_of(params ? (const OParams*)params : &dp);
  for (int i = 0; i < n; ++i) {
    Shape A, Bs;
    load_shape(a + 18 * (size_t)i, &A);
    load_shape(b + 18 * (size_t)i, &Bs);
    V2 s[3];
    int h = gjk(&A, &Bs, np.d0, s, np.gjk_steps);
    hit[i] = h;
    for (int k = 0; k < 3; ++k) {
      simplex[6 * i + 2 * k] = h ? s[k].x : s[k].x * qnan();
      simplex[6 * i + 2 * k + 1] = h ? s[k].y : s[k].y * qnan();
    }
  }
  return 0;
}
int oracle_epa(int n, const float* a, const float* b, const float* simplex, int iters, float* pen) {
  if (iters < 3 || iters > 128) return -1;
  for (int i = 0; i < n; ++i) {
    Shape A, Bs;
    load_shape(a + 18 * (size_t)i, &A);
    load_shape(b + 18 * (size_t)i, &Bs);
    const float* q = simplex + 6 * i;
    V2 s[3] = {v2(q[0], q[1]), v2(q[2], q[3]), v2(q[4], q[5])};
    V2 p = epa(&A, &Bs, s, iters);
    pen[2 * i] = p.x; pen[2 * i + 1] = p.y;
  }
  return 0;
}
