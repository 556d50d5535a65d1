// Device-side building blocks of the cotix hot path for gfx950 (CDNA4).
//
// Every function here restates one reference function; the cited file:line
// is in /root/reference (DelftMercurians/Parallax, package `cotix`).  Numeric
// contract (shared with the oracle, DESIGN.md "Numerics"): IEEE f32, one
// rounding per operation, NO fma contraction (built with -ffp-contract=off),
// the reference expression's evaluation order, NaN-propagating min/max/clip,
// argmin/argmax = first NaN else first extremum, and deterministic f32
// sin/cos/atan2 kernels (cephes polynomials) so results are bit-identical
// to the CPU oracle.
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIP__) || defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define CX_DEV __device__ __forceinline__
#define CX_MF __device__ __forceinline__  // member functions
#define CX_HD __host__ __device__ inline   // host + device (layout arithmetic)
#else
// host build of the same code: used ONLY by the CPU emulation harness of the
// test suite (tests/emu/), to run the kernel logic under AddressSanitizer.
#define CX_DEV static inline
#define CX_MF inline
#define CX_HD static inline
static inline float __uint_as_float(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}
static inline uint32_t __float_as_uint(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}
#endif

namespace cx {

// ---------------------------------------------------------------------------
// float helpers
// ---------------------------------------------------------------------------
CX_DEV bool isn(float x) { return x != x; }
CX_DEV float qnan() { return __builtin_nanf(""); }
CX_DEV float finf() { return __builtin_inff(); }

// lax.max / lax.min: NaN-propagating (the first NaN operand), ties keep the
// first operand.  Two flat selects: a >= b is false when either is NaN, so
// m is already b when b is NaN, and only a NaN a needs its own test (the two
// compares are independent: their select hazards overlap).  The
// nested-ternary form compiles to divergent branches on gfx950.
CX_DEV float fmax_(float a, float b) {
  const float m = (a >= b) ? a : b;
  return isn(a) ? a : m;
}
CX_DEV float fmin_(float a, float b) {
  const float m = (a <= b) ? a : b;
  return isn(a) ? a : m;
}
// jnp.clip (jax 0.4.x): minimum(hi, maximum(lo, x))
CX_DEV float clip_(float x, float lo, float hi) { return fmin_(hi, fmax_(lo, x)); }

struct v2 {
  float x, y;
};
CX_DEV v2 mk(float x, float y) { return v2{x, y}; }
CX_DEV v2 add(v2 a, v2 b) { return v2{a.x + b.x, a.y + b.y}; }
CX_DEV v2 sub(v2 a, v2 b) { return v2{a.x - b.x, a.y - b.y}; }
CX_DEV v2 neg(v2 a) { return v2{-a.x, -a.y}; }
CX_DEV v2 scl(v2 a, float s) { return v2{a.x * s, a.y * s}; }
CX_DEV v2 divs(v2 a, float s) { return v2{a.x / s, a.y / s}; }
CX_DEV float dot(v2 a, v2 b) { return a.x * b.x + a.y * b.y; }
CX_DEV float crs(v2 a, v2 b) { return a.x * b.y - a.y * b.x; }  // jnp.cross (2-D)
CX_DEV float sumsq(v2 a) { return a.x * a.x + a.y * a.y; }
CX_DEV float nrm(v2 a) { return __builtin_sqrtf(sumsq(a)); }
CX_DEV bool vnan(v2 a) { return isn(a.x) || isn(a.y); }
CX_DEV v2 fnormal(v2 a) { return v2{-a.y, a.x}; }  // fast_normal, _geometry_utils.py:30-34

// ---------------------------------------------------------------------------
// deterministic f32 transcendentals (the build's fixed choice; see oracle)
// ---------------------------------------------------------------------------
CX_DEV float sin_poly(float r) {
  float z = r * r;
  return (((-1.9515295891e-4f * z + 8.3321608736e-3f) * z + -1.6666654611e-1f) * z) * r + r;
}
CX_DEV float cos_poly(float r) {
  float z = r * r;
  return ((((2.443315711809948e-5f * z + -1.388731625493765e-3f) * z + 4.166664568298827e-2f) * z) * z -
          0.5f * z) +
         1.0f;
}
// (the kernels below are written as flat selects: their branchy forms
// compile to divergent branches on gfx950; every value is computed by the
// same expression as the branchy form, so the results are identical)
CX_DEV void sincos32(float x, float* s_out, float* c_out) {
  const bool bad = isn(x) || __builtin_isinf(x);
  const float xs = bad ? 0.0f : x;
  float t = xs * 0.636619772367581343f;
  float k = (t + 12582912.0f) - 12582912.0f;
  float r = ((xs - k * 1.5703125f) - k * 4.837512969970703125e-4f) - k * 7.54978995489188216e-8f;
  float s = sin_poly(r), c = cos_poly(r);
  int q = ((int)k) & 3;
  // q = 0: (s, c), 1: (c, -s), 2: (-s, -c), 3: (-c, s)
  float so = (q & 1) ? c : s, co = (q & 1) ? -s : c;
  so = (q & 2) ? -so : so;
  co = (q & 2) ? -co : co;
  *s_out = bad ? qnan() : so;
  *c_out = bad ? qnan() : co;
}
CX_DEV float atan01(float t) {
  const bool big = t > 0.4142135623730950f;
  const float y0 = big ? 0.785398163397448309616f : 0.0f;
  t = big ? (t - 1.0f) / (t + 1.0f) : t;
  float z = t * t;
  float p = ((((8.05374449538e-2f * z + -1.38776856032e-1f) * z + 1.99777106478e-1f) * z + -3.33329491539e-1f) * z) * t + t;
  return y0 + p;
}
CX_DEV float atan2_32(float y, float x) {
  const float PI = 3.14159265358979323846f, PIO2 = 1.57079632679489661923f;
  const float ax = __builtin_fabsf(x), ay = __builtin_fabsf(y);
  const bool sw = !(ay <= ax);  // (ay <= ax) ? atan01(ay / ax) : PIO2 - atan01(ax / ay)
  float r = atan01((sw ? ax : ay) / (sw ? ay : ax));
  r = sw ? PIO2 - r : r;
  r = x < 0.0f ? PI - r : r;
  r = y < 0.0f ? -r : r;
  // special cases, lowest priority first: x == 0, then y == 0, then NaN
  r = x == 0.0f ? (y < 0.0f ? -PIO2 : PIO2) : r;
  const float y0r = (x > 0.0f || (x == 0.0f && !__builtin_signbit(x))) ? y : (__builtin_signbit(y) ? -PI : PI);
  r = y == 0.0f ? y0r : r;
  return (isn(x) || isn(y)) ? qnan() : r;
}
// lax.sort order key: -0 == +0, NaN after everything (all NaN equal).
CX_DEV bool sort_lt(float a, float b) {
  if (isn(a)) return false;
  if (isn(b)) return true;
  return a < b;
}

// ---------------------------------------------------------------------------
// threefry2x32-20 and the jax.random legacy layouts (jax/_src/prng.py)
// ---------------------------------------------------------------------------
struct key2 {
  uint32_t a, b;
};
CX_DEV uint32_t rotl(uint32_t v, uint32_t r) { return (v << r) | (v >> (32u - r)); }
#define CX_RND(r) \
  x0 += x1;       \
  x1 = rotl(x1, r); \
  x1 ^= x0;
CX_DEV key2 threefry(key2 k, uint32_t x0, uint32_t x1) {
  const uint32_t k0 = k.a, k1 = k.b, k2 = k.a ^ k.b ^ 0x1BD11BDAu;
  x0 += k0;
  x1 += k1;
  CX_RND(13) CX_RND(15) CX_RND(26) CX_RND(6)
  x0 += k1; x1 += k2 + 1u;
  CX_RND(17) CX_RND(29) CX_RND(16) CX_RND(24)
  x0 += k2; x1 += k0 + 2u;
  CX_RND(13) CX_RND(15) CX_RND(26) CX_RND(6)
  x0 += k0; x1 += k1 + 3u;
  CX_RND(17) CX_RND(29) CX_RND(16) CX_RND(24)
  x0 += k1; x1 += k2 + 4u;
  CX_RND(13) CX_RND(15) CX_RND(26) CX_RND(6)
  x0 += k2; x1 += k0 + 5u;
  return key2{x0, x1};
}
#undef CX_RND
// word m of the flat output of split(key, num) (counters iota(2*num)): the
// y0 of block (m, num+m) when m < num, else the y1 of block (m-num, m).
// Branch-free (one block per word even when lanes diverge on m < num).
CX_DEV uint32_t split_word(key2 k, uint32_t num, uint32_t m) {
  const bool lo = m < num;
  const key2 r = threefry(k, lo ? m : m - num, lo ? num + m : m);
  return lo ? r.a : r.b;
}
// split(key, num)[idx]: two blocks (for num == 1 both words come from block
// (0, 1), which the same formula yields).
CX_DEV key2 split_at(key2 k, uint32_t num, uint32_t idx) {
  return key2{split_word(k, num, 2u * idx), split_word(k, num, 2u * idx + 1u)};
}
// the single 32-bit word of random_bits(key, ()) (odd count -> zero pad).
CX_DEV uint32_t bits1(key2 k) { return threefry(k, 0u, 0u).a; }
CX_DEV float unit_float(uint32_t bits) { return __uint_as_float((bits >> 9) | 0x3F800000u) - 1.0f; }
// jax.random.uniform(key, (), lo, hi): max(lo, f*(hi-lo)+lo)
CX_DEV float uniform1(key2 k, float lo, float hi) { return fmax_(lo, unit_float(bits1(k)) * (hi - lo) + lo); }
// jax.random.bernoulli(key, 0.5, ()): top bit of the word is 0.
CX_DEV bool bernoulli_half(key2 k) { return (bits1(k) >> 31) == 0u; }

// The partitionable layout (jax_threefry_partitionable=True, the default from
// JAX 0.5; include/cotix_amd.h COTIX_PRNG_*): _threefry_split_foldlike gives
// split(key, n)[i] = threefry(key, (0, i)) -- the (hi, lo) words of
// iota_2x32_shape -- and _threefry_random_bits_partitionable gives word m of a
// 32-bit draw as y0 ^ y1 of threefry(key, (0, m)).  `part` is a scene
// constant (wave-uniform branch).
CX_DEV key2 split_at_l(key2 k, uint32_t num, uint32_t idx, bool part) {
  if (part) return threefry(k, 0u, idx);
  return split_at(k, num, idx);
}
// the single word of random_bits(key, ()) in either layout
CX_DEV uint32_t bits1_l(key2 k, bool part) {
  const key2 r = threefry(k, 0u, 0u);
  return part ? (r.a ^ r.b) : r.a;
}
// jax.random.bernoulli(key, p, ()) = uniform(key) < p (p as f32)
CX_DEV bool bernoulli_l(key2 k, float p, bool part) { return unit_float(bits1_l(k, part)) < p; }

// jnp.cumsum via lax.associative_scan (CPU lowering), n <= 16.
CX_DEV void cumsum_assoc(const float* in, int n, float* out) {
  float lv[5][16];
  int ln[5];
  int L = 0;
  for (int k = 0; k < n; ++k) lv[0][k] = in[k];
  ln[0] = n;
  while (ln[L] >= 2 && L < 4) {
    int m = ln[L] / 2;
    for (int k = 0; k < m; ++k) lv[L + 1][k] = lv[L][2 * k] + lv[L][2 * k + 1];
    ln[L + 1] = m;
    ++L;
  }
  // lv[L] is its own scan (length < 2); walk back down.
  float res[16];
  for (int k = 0; k < ln[L]; ++k) res[k] = lv[L][k];
  for (int l = L - 1; l >= 0; --l) {
    int nl = ln[l], no = ln[l + 1];
    float odd[16], even[16], outl[16];
    for (int k = 0; k < no; ++k) odd[k] = res[k];
    int ne_tail = (nl % 2 == 0) ? no - 1 : no;
    even[0] = lv[l][0];
    for (int k = 0; k < ne_tail; ++k) even[k + 1] = odd[k] + lv[l][2 * k + 2];
    for (int k = 0; k < nl; ++k) outl[k] = (k % 2 == 0) ? even[k / 2] : odd[k / 2];
    for (int k = 0; k < nl; ++k) res[k] = outl[k];
  }
  for (int k = 0; k < n; ++k) out[k] = res[k];
}

// ---------------------------------------------------------------------------
// shapes (cotix/_convex_shapes.py); world-frame geometry in 16 floats
// ---------------------------------------------------------------------------
enum : int { KIND_CIRCLE = 0, KIND_AABB = 1, KIND_POLY = 2 };
constexpr int MAXV = 8;
// A shape's geometry words (circle: r,cx,cy; aabb: lo.x,lo.y,up.x,up.y; poly:
// xy*n) live in registers.  Every polygon loop below is unrolled to MAXV with
// a k < n guard and every per-lane vertex pick is a select chain, so the
// array is only ever indexed with compile-time constants (no scratch), and a
// contact fetches its two shapes once (GJK/EPA iterations are pure ALU).
struct Shape {
  int kind, n;
  float w[2 * MAXV];
  CX_MF float d(int k) const { return w[k]; }
};
CX_DEV uint32_t f2u(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}
// c ? a : b on the bit patterns (a select between two elements of a private
// array can be rewritten by LLVM into a select of their ADDRESSES and a load
// from a scratch copy; the masked OR keeps both operands in registers)
CX_DEV float bsel(bool c, float a, float b) {
  const uint32_t m = 0u - (uint32_t)c;
  return __uint_as_float((f2u(a) & m) | (f2u(b) & ~m));
}
// vertex k, k varying per lane (0 <= k < MAXV): masked OR of the bit
// patterns (a plain select chain gets rewritten by LLVM into an indexed
// load from a scratch copy of the array); constant-folds for constant k
CX_DEV v2 vert(const Shape& s, int k) {
  uint32_t x = 0u, y = 0u;
#pragma unroll
  for (int q = 0; q < MAXV; ++q) {
    const uint32_t m = 0u - (uint32_t)(q == k);
    x |= f2u(s.w[2 * q]) & m;
    y |= f2u(s.w[2 * q + 1]) & m;
  }
  return v2{__uint_as_float(x), __uint_as_float(y)};
}
// argmin over v[0..n), n <= N at run time: first NaN, else first minimum
template <int N>
CX_DEV int argmin_first_n(const float* v, int n) {
  int nan = -1, b = 0;
  float bv = v[0];
#pragma unroll
  for (int k = 0; k < N; ++k)
    if (k < n) {
      if (nan < 0 && isn(v[k])) nan = k;
      if (k > 0 && v[k] < bv) {
        bv = v[k];
        b = k;
      }
    }
  return nan >= 0 ? nan : b;
}

CX_DEV int argmax_first(const float* v, int n) {
  for (int k = 0; k < n; ++k)
    if (isn(v[k])) return k;
  int b = 0;
  for (int k = 1; k < n; ++k)
    if (v[k] > v[b]) b = k;
  return b;
}
CX_DEV int argmin_first(const float* v, int n) {
  for (int k = 0; k < n; ++k)
    if (isn(v[k])) return k;
  int b = 0;
  for (int k = 1; k < n; ++k)
    if (v[k] < v[b]) b = k;
  return b;
}

// get_support: Circle :22-26, AABB :62-66, Polygon :149-155
CX_DEV v2 support(const Shape& s, v2 d) {
  if (s.kind == KIND_CIRCLE) {
    float n = nrm(d);
    v2 nd = v2{d.x / n, d.y / n};
    return v2{nd.x * s.d(0) + s.d(1), nd.y * s.d(0) + s.d(2)};
  }
  if (s.kind == KIND_AABB) {
    return v2{d.x >= 0.0f ? s.d(2) : s.d(0), d.y >= 0.0f ? s.d(3) : s.d(1)};
  }
  if (vnan(d)) return v2{qnan(), qnan()};
  // argmax(v . d): first NaN, else first maximum.  Branch-free select chain
  // (a guarded/branchy form of this loop was miscompiled by hipcc 7.2 at -O2+).
  float bv = s.w[0] * d.x + s.w[1] * d.y;
  float bx = s.w[0], by = s.w[1];
  auto step = [&](int k) {
    const float x = s.w[2 * k], y = s.w[2 * k + 1];
    const float t = x * d.x + y * d.y;
    // bitwise, not short-circuit: && / || compile to exec-mask branches here
    const bool take = (k < s.n) & !isn(bv) & (isn(t) | (t > bv));
    bv = take ? t : bv;
    bx = take ? x : bx;
    by = take ? y : by;
  };
  // vertices 1..3 always (n >= 3); 4..5 and 6..7 only when some lane of the
  // wave has that many (the select chain itself stays branch-free)
  step(1);
  step(2);
  step(3);
  if (s.n > 4) {
    step(4);
    step(5);
  }
  if (s.n > 6) {
    step(6);
    step(7);
  }
  static_assert(MAXV == 8, "support() unrolls for MAXV == 8");
  return v2{bx, by};
}
// a part inside its body's frame, as UniversalShape.wrap_local_support sees it
// (cotix/_universal_shape.py:32-45): the inverse_direction result is
// discarded there (:38), so the local support is taken in the GLOBAL direction
// and then mapped forward (rotation + translation).  Body-level GJK/EPA only.
struct WrappedShape {
  Shape s;
  float c, sn, px, py;  // cos, sin of the body angle; body position
};
CX_DEV v2 support(const WrappedShape& w, v2 d) {
  const v2 l = support(w.s, d);
  const float t0 = (w.c * l.x + (-w.sn) * l.y) + w.px * 1.0f;
  const float t1 = (w.sn * l.x + w.c * l.y) + w.py * 1.0f;
  const float t2 = (0.0f * l.x + 0.0f * l.y) + 1.0f * 1.0f;
  return v2{t0 / t2, t1 / t2};
}
// a shape known to be a polygon (the step kernel's polygon x polygon items):
// the support without the kind dispatch -- the same select chain, NaN
// direction as a final select
struct PolyRef {
  const Shape& s;
};
CX_DEV v2 support(const PolyRef& p, v2 d) {
  const Shape& s = p.s;
  float bv = s.w[0] * d.x + s.w[1] * d.y;
  float bx = s.w[0], by = s.w[1];
  auto step = [&](int k) {
    const float x = s.w[2 * k], y = s.w[2 * k + 1];
    const float t = x * d.x + y * d.y;
    const bool take = (k < s.n) & !isn(bv) & (isn(t) | (t > bv));
    bv = take ? t : bv;
    bx = take ? x : bx;
    by = take ? y : by;
  };
  step(1);
  step(2);
  step(3);
  if (s.n > 4) {
    step(4);
    step(5);
  }
  if (s.n > 6) {
    step(6);
    step(7);
  }
  const bool dn = vnan(d);
  return v2{dn ? qnan() : bx, dn ? qnan() : by};
}
template <class SA, class SB>
CX_DEV v2 minkowski(const SA& a, const SB& b, v2 d) { return sub(support(a, d), support(b, neg(d))); }

CX_DEV bool circle_contains(const Shape& c, v2 p) {  // :28-29
  float r = c.d(0) + 1e-6f;
  return sumsq(sub(p, v2{c.d(1), c.d(2)})) <= r * r;
}
CX_DEV bool aabb_contains(const Shape& a, v2 p) {  // :105-106
  return (p.x >= a.d(0) - 1e-6f) && (p.y >= a.d(1) - 1e-6f) && (p.x <= a.d(2) + 1e-6f) && (p.y <= a.d(3) + 1e-6f);
}
CX_DEV float fsign(float x) {  // jnp.sign: NaN and +-0 map to themselves (flat selects)
  float r = x > 0.0f ? 1.0f : x;
  return x < 0.0f ? -1.0f : r;
}
CX_DEV bool poly_contains(const Shape& s, v2 p) {  // :168-175, edge k = (v_k, v_{k-1})
  float s0 = 0.0f;
  bool ok = true;
  const v2 last = vert(s, s.n - 1);
#pragma unroll
  for (int k = 0; k < MAXV; ++k)
    if (k < s.n) {
      const v2 e0 = v2{s.w[2 * k], s.w[2 * k + 1]};
      const v2 e1 = k == 0 ? last : v2{s.w[2 * k - 2], s.w[2 * k - 1]};
      float sg = fsign(dot(sub(p, e0), fnormal(sub(e0, e1))));
      if (k == 0) s0 = sg;
      else ok = ok && (sg == s0);
    }
  return ok && !isn(s0);
}
// order_clockwise (cotix/_geometry_utils.py:60-67): sequential mean, atan2,
// stable sort by angle.  The stable order is computed as ranks -- vertex k
// goes to #{j : ang_j < ang_k} + #{j < k : ang_j ~ ang_k} under sort_lt (a
// strict weak order: NaN last, -0 ~ +0), the same permutation insertion sort
// produces -- with every loop unrolled to MAXV (register-only, no scratch).
struct Poly {
  float x[MAXV], y[MAXV];
};
CX_DEV Poly order_clockwise(const Poly& q, int n) {
  float sx = 0.0f, sy = 0.0f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k)
    if (k < n) {
      sx = sx + q.x[k];
      sy = sy + q.y[k];
    }
  const float fn = (float)n;
  const float mx = sx / fn, my = sy / fn;
  // sort keys: atan2 lies in [-pi, pi] or is NaN, so NaN -> 4 (after every
  // angle, all NaN equal) makes sort_lt(a, b) == key(a) < key(b) (-0 == +0
  // under <): one compare per pair
  float key[MAXV];
#pragma unroll
  for (int k = 0; k < MAXV; ++k) key[k] = 0.0f;
  auto angle = [&](int k) {
    const float a = k < n ? atan2_32(q.y[k] - my, q.x[k] - mx) : 0.0f;
    key[k] = isn(a) ? 4.0f : a;
  };
  // vertices 4..5 / 6..7 only when some lane of the wave has that many
  angle(0);
  angle(1);
  angle(2);
  angle(3);
  if (n > 4) {
    angle(4);
    angle(5);
  }
  if (n > 6) {
    angle(6);
    angle(7);
  }
  static_assert(MAXV == 8, "order_clockwise unrolls for MAXV == 8");
  // stable rank: j before k if key_j < key_k, or j < k and not key_k < key_j
  int rank[MAXV];
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    int r = 0;
#pragma unroll
    for (int j = 0; j < MAXV; ++j)
      if (j != k && j < n) r += (j < k ? !(key[k] < key[j]) : (key[j] < key[k])) ? 1 : 0;
    rank[k] = r;
  }
  Poly out;
#pragma unroll
  for (int p = 0; p < MAXV; ++p) {
    float x = q.x[p], y = q.y[p];
#pragma unroll
    for (int k = 0; k < MAXV; ++k)
      if (k < n && rank[k] == p) {
        x = q.x[k];
        y = q.y[k];
      }
    out.x[p] = x;
    out.y[p] = y;
  }
  return out;
}
CX_DEV void order_clockwise(float* xy, int n) {  // interleaved form (operator kernel, tests)
  Poly q;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    q.x[k] = k < n ? xy[2 * k] : 0.0f;
    q.y[k] = k < n ? xy[2 * k + 1] : 0.0f;
  }
  const Poly r = order_clockwise(q, n);
  for (int k = 0; k < n; ++k) {
    xy[2 * k] = r.x[k];
    xy[2 * k + 1] = r.y[k];
  }
}

// ---------------------------------------------------------------------------
// contacts (cotix/_contacts.py); ContactInfo = (pen, cp), NaN cp = none
// ---------------------------------------------------------------------------
struct Contact {
  v2 pen, cp;
};
CX_DEV Contact nan_contact() { return Contact{v2{0.0f, 0.0f}, v2{qnan(), qnan()}}; }

// argmin over 4 values (first NaN, else first minimum) as flat selects
CX_DEV int argmin4(const float* v) {
  int k = 0;
  float bv = v[0];
#pragma unroll
  for (int q = 1; q < 4; ++q) {
    const bool lt = v[q] < bv;
    bv = lt ? v[q] : bv;
    k = lt ? q : k;
  }
  int nk = isn(v[3]) ? 3 : -1;
  nk = isn(v[2]) ? 2 : nk;
  nk = isn(v[1]) ? 1 : nk;
  nk = isn(v[0]) ? 0 : nk;
  return nk >= 0 ? nk : k;
}
CX_DEV float pick4(int k, float a0, float a1, float a2, float a3) {
  const float lo = k == 0 ? a0 : a1, hi = k == 2 ? a2 : a3;
  return k < 2 ? lo : hi;
}

CX_DEV Contact aabb_vs_aabb(const Shape& a, const Shape& b) {  // :61-96
  const float alx = a.d(0), aly = a.d(1), aux = a.d(2), auy = a.d(3);
  const float blx = b.d(0), bly = b.d(1), bux = b.d(2), buy = b.d(3);
  bool below = auy <= bly, above = aly >= buy, left = aux <= blx, right = alx >= bux;
  if (below || left || above || right) return nan_contact();
  const float me = -1e-8f;
  float dep[4] = {fmax_(auy - bly, me), fmax_(buy - aly, me), fmax_(aux - blx, me), fmax_(bux - alx, me)};
  const float dx[4] = {0.0f, 0.0f, -1.0f, 1.0f}, dy[4] = {-1.0f, 1.0f, 0.0f, 0.0f};
  (void)dx;
  (void)dy;
  const int k = argmin4(dep);
  float md = fmax_(0.0f, pick4(k, dep[0], dep[1], dep[2], dep[3]));
  Contact c;
  c.pen = v2{md * pick4(k, 0.0f, 0.0f, -1.0f, 1.0f), md * pick4(k, -1.0f, 1.0f, 0.0f, 0.0f)};
  v2 mu = v2{fmin_(aux, bux), fmin_(auy, buy)}, ml = v2{fmax_(alx, blx), fmax_(aly, bly)};
  c.cp = divs(add(mu, ml), 2.0f);
  return c;
}

CX_DEV Contact circle_vs_circle(const Shape& a, const Shape& b) {  // :30-58
  v2 ap = v2{a.d(1), a.d(2)}, bp = v2{b.d(1), b.d(2)};
  float ar = a.d(0), br = b.d(0);
  v2 delta = sub(ap, bp);
  float dist = nrm(delta);
  v2 dir = (dist == 0.0f) ? v2{1.0f, 0.0f} : divs(delta, dist);
  v2 pen = scl(dir, fmin_(dist - (ar + br), 0.0f));
  v2 cp = divs(add(add(bp, scl(dir, br - ar)), ap), 2.0f);
  if (!(dot(sub(ap, cp), sub(bp, cp)) <= 0.0f)) cp = circle_contains(a, bp) ? bp : ap;
  if (dist <= ar + br) return Contact{neg(pen), cp};
  return nan_contact();
}

// circle_vs_aabb :99-154.  *err |= 1 when eqx.error_if trips (ccp not in the
// AABB); the guarded ccp then becomes NaN (EQX_ON_ERROR=nan semantics).
CX_DEV Contact circle_vs_aabb(const Shape& a, const Shape& b, uint32_t* err) {
  v2 ap = v2{a.d(1), a.d(2)};
  float r = a.d(0);
  v2 lo = v2{b.d(0), b.d(1)}, up = v2{b.d(2), b.d(3)};
  v2 bc = v2{(lo.x + up.x) / 2.0f, (lo.y + up.y) / 2.0f};
  v2 disp = sub(ap, bc);
  v2 l = sub(lo, bc), h = sub(up, bc);
  v2 ccp = add(bc, v2{clip_(disp.x, l.x, h.x), clip_(disp.y, l.y, h.y)});
  if (!aabb_contains(b, ccp)) {
    *err |= 1u;
    ccp = v2{qnan(), qnan()};
  }
  v2 vs[4] = {lo, v2{lo.x, up.y}, up, v2{up.x, lo.y}};
  // |vs[k] - ccp| < 1e-6 (:118): with correctly rounded sqrt, sqrt(s) < 1e-6f
  // exactly when s < 0x2b8cbccb (the least s with sqrt(s) >= 1e-6f)
  const float T = __uint_as_float(0x2b8cbccbu);
  bool perfect = false;
#pragma unroll
  for (int k = 0; k < 4; ++k) perfect = perfect | (sumsq(sub(vs[k], ccp)) < T);
  if (!circle_contains(a, ccp)) return nan_contact();
  if (perfect) {
    v2 d = sub(ccp, ap);
    v2 dn = divs(d, nrm(d));
    return Contact{neg(sub(add(ap, scl(dn, r)), ccp)), ccp};
  }
  float sh[4] = {(ap.y + r) - lo.y, up.y - (ap.y - r), (ap.x + r) - lo.x, up.x - (ap.x - r)};
  const float dx[4] = {0.0f, 0.0f, 1.0f, -1.0f}, dy[4] = {1.0f, -1.0f, 0.0f, 0.0f};
  (void)dx;
  (void)dy;
  const int k = argmin4(sh);
  float ns = -pick4(k, sh[0], sh[1], sh[2], sh[3]);
  return Contact{v2{ns * pick4(k, 0.0f, 0.0f, 1.0f, -1.0f), ns * pick4(k, 1.0f, -1.0f, 0.0f, 0.0f)}, ccp};
}

// ---------------------------------------------------------------------------
// narrow-phase parameters (cotix_params): the GJK start direction
// random_direction(PRNGKey(1)) of the scene's PRNG layout
// (cotix/_collisions.py:287-298), GJK steps (:101), the EPA iteration cap of
// the polygon contacts (cotix/_contacts.py:271,295), circle x polygon's EPA
// iterations (:162-163) and the body-level penetration_depth's
// (cotix/_universal_shape.py:120)
// ---------------------------------------------------------------------------
struct NarrowParams {
  v2 d0;
  int gjk_steps, epa_cap, epa_cp, epa_body;
};
// random_direction(PRNGKey(1)) = normal(PRNGKey(1), (2,)) / norm: legacy
// (0xbd56c50b, 0x3f7fa5d9), partitionable (0xbf607449, 0x3ef638cd)
// (oracle/cotix_oracle/prng.py gjk_initial_direction, XLA's f32 ErfInv)
CX_HD v2 gjk_d0(bool part) {
  return part ? v2{__builtin_bit_cast(float, 0xbf607449u), __builtin_bit_cast(float, 0x3ef638cdu)}
              : v2{__builtin_bit_cast(float, 0xbd56c50bu), __builtin_bit_cast(float, 0x3f7fa5d9u)};
}
CX_HD NarrowParams narrow_default() { return NarrowParams{gjk_d0(false), 32, 48, 128, 48}; }

// random_direction(key) for any key (cotix/_geometry_utils.py:37-46): x / |x|,
// x = normal(key, (2,)) = sqrt(2) * erf_inv(uniform(key, (2,), nextafter(-1,
// 0), 1)) with XLA's f32 ErfInv (Giles) whose log1p is correctly rounded
// (the f64 log1p rounded once; oracle/cotix_oracle/prng.py random_direction,
// erf_inv32_cr).  PRNGKey(1) is the constant gjk_d0, as the oracle: key=None
// and key=PRNGKey(1) agree as in the reference.  Operator path only (cotix_gjk_ex).
CX_DEV float log1p_cr(float a) {
#if defined(__HIP__)
  return (float)__ocml_log1p_f64((double)a);
#else
  return (float)__builtin_log1p((double)a);
#endif
}
CX_DEV float erf_inv32_cr(float x) {
  const float w0 = -log1p_cr(-(x * x));
  const bool lt = w0 < 5.0f;
  const float w = lt ? w0 - 2.5f : __builtin_sqrtf(w0) - 3.0f;
  float p;
  if (lt) {
    p = 2.81022636e-08f;
    p = 3.43273939e-07f + p * w; p = -3.5233877e-06f + p * w; p = -4.39150654e-06f + p * w;
    p = 0.00021858087f + p * w; p = -0.00125372503f + p * w; p = -0.00417768164f + p * w;
    p = 0.246640727f + p * w; p = 1.50140941f + p * w;
  } else {
    p = -0.000200214257f;
    p = 0.000100950558f + p * w; p = 0.00134934322f + p * w; p = -0.00367342844f + p * w;
    p = 0.00573950773f + p * w; p = -0.0076224613f + p * w; p = 0.00943887047f + p * w;
    p = 1.00167406f + p * w; p = 2.83297682f + p * w;
  }
  return p * x;
}
CX_DEV v2 random_direction(key2 k, bool part) {
  if (k.a == 0u && k.b == 1u) return gjk_d0(part);
  uint32_t bits[2];
  if (part) {  // word m = y0 ^ y1 of threefry(key, (0, m))
    const key2 r0 = threefry(k, 0u, 0u), r1 = threefry(k, 0u, 1u);
    bits[0] = r0.a ^ r0.b;
    bits[1] = r1.a ^ r1.b;
  } else {  // the two words of threefry(key, iota(2)) = block (0, 1)
    const key2 r = threefry(k, 0u, 1u);
    bits[0] = r.a;
    bits[1] = r.b;
  }
  const float lo = __builtin_bit_cast(float, 0xbf7fffffu), hi = 1.0f;  // nextafter(-1, 0), 1
  float x[2];
  for (int m = 0; m < 2; ++m) {
    const float u = fmax_(lo, unit_float(bits[m]) * (hi - lo) + lo);
    x[m] = __builtin_bit_cast(float, 0x3fb504f3u) * erf_inv32_cr(u);  // f32(sqrt(2))
  }
  const float n = __builtin_sqrtf(x[0] * x[0] + x[1] * x[1]);
  return v2{x[0] / n, x[1] / n};
}
// check_for_collision_convex's start direction (cotix/_collisions.py:285-298):
// rnd if initial_direction has a NaN, else rnd * 0.1 + initial_direction * 0.9
CX_DEV v2 gjk_start(v2 rnd, v2 init) {
  if (init.x != init.x || init.y != init.y) return rnd;
  return v2{rnd.x * 0.1f + init.x * 0.9f, rnd.y * 0.1f + init.y * 0.9f};
}

// ---------------------------------------------------------------------------
// GJK (cotix/_collisions.py:20-112, 277-310)
// ---------------------------------------------------------------------------
CX_DEV bool point_in_triangle0(v2 v1, v2 v2_, v2 v3) {  // _geometry_utils.py:12-27, pt = 0
  v2 pt = v2{0.0f, 0.0f};
  auto sgn = [](v2 p1, v2 p2, v2 p3) { return (p1.x - p3.x) * (p2.y - p3.y) - (p2.x - p3.x) * (p1.y - p3.y); };
  float d1 = sgn(pt, v1, v2_), d2 = sgn(pt, v2_, v3), d3 = sgn(pt, v3, v1);
  bool has_neg = (d1 < 0.0f) || (d2 < 0.0f) || (d3 < 0.0f);
  bool has_pos = (d1 > 0.0f) || (d2 > 0.0f) || (d3 > 0.0f);
  return !(has_neg && has_pos);
}

template <class SA, class SB>
CX_DEV bool gjk(const SA& a, const SB& b, v2 d0, v2* simplex, int max_steps = 32) {
  v2 s0 = minkowski(a, b, d0);
  v2 s1 = minkowski(a, b, neg(s0));
  v2 dir = fnormal(sub(s1, s0));
  {  // orientation fix (:44-53) as selects
    const bool sw = dot(dir, neg(s1)) > 0.0f;
    const v2 t0 = s0;
    s0 = sw ? s1 : s0;
    s1 = sw ? t0 : s1;
    dir = sw ? dir : neg(dir);
  }
  v2 s2 = minkowski(a, b, dir);
  for (int step = 0; step < max_steps; ++step) {  // while_loop(max_steps=32), :101
    bool c1 = dot(s2, dir) <= 0.0f;
    bool c2 = dot(fnormal(sub(s2, s0)), neg(s2)) < 0.0f;
    bool c3 = dot(fnormal(sub(s1, s2)), neg(s2)) < 0.0f;
    if (c1 || (c2 && c3)) break;
    v2 c = s2;
    v2 acn = fnormal(sub(c, s0)), cbn = fnormal(sub(s1, c));
    const bool ac = dot(acn, neg(c)) >= 0.0f;
    s1 = ac ? c : s1;
    s0 = ac ? s0 : c;
    dir = ac ? acn : cbn;
    s2 = minkowski(a, b, dir);
  }
  v2 z = v2{0.0f, 0.0f};
  if (!point_in_triangle0(s0, s1, s2)) {
    s0 = z;
    s1 = z;
    s2 = z;
  }
  // check_for_collision_convex :300-310
  float area = crs(sub(s1, s0), sub(s2, s0));
  bool allzero = s0.x == 0.0f && s0.y == 0.0f && s1.x == 0.0f && s1.y == 0.0f && s2.x == 0.0f && s2.y == 0.0f;
  bool anynan = vnan(s0) || vnan(s1) || vnan(s2);
  simplex[0] = s0;
  simplex[1] = s1;
  simplex[2] = s2;
  return !(allzero || anynan || area == 0.0f);
}

// ---------------------------------------------------------------------------
// EPA (cotix/_collisions.py:115-273), edge buffer of NE = iters + 3 edges.
// Distances are cached per edge (only the two rewritten edges change per
// iteration); the reference recomputes all of them -- same values.
// ---------------------------------------------------------------------------
// (both written as flat selects: every path is evaluated and the reference's
// one is selected -- same values, no divergent branches in the GJK/EPA loops)
CX_DEV v2 closest_on_edge_to_origin(v2 a, v2 b) {  // :156-166, point = 0
  v2 p = v2{0.0f, 0.0f};
  float len = sumsq(sub(a, b));
  float t = dot(sub(p, b), sub(a, b)) / len;
  t = clip_(t, 0.0f, 1.0f);
  v2 proj = add(b, scl(sub(a, b), t));
  const v2 r = sub(p, proj), r0 = sub(p, a);
  return len == 0.0f ? r0 : r;
}
CX_DEV float edge_dist(v2 a, v2 b) {  // distance_to_origin :137-154,168-169
  const bool zero = a.x == 0.0f && a.y == 0.0f && b.x == 0.0f && b.y == 0.0f;
  const float i = finf();
  v2 p = v2{0.0f, 0.0f};
  float len = sumsq(sub(a, b));
  float t = dot(sub(p, b), sub(a, b)) / len;
  t = clip_(t, 0.0f, 1.0f);
  v2 proj = add(b, scl(sub(a, b), t));
  v2 disp = sub(p, proj);
  disp = len == 0.0f ? neg(a) : disp;
  return zero ? i * i + i * i : sumsq(disp);
}

// EPA edge storage: registers (operator kernels, host; dynamic indices as
// select chains) or a per-lane LDS column of the step kernel's wave scratch
// (dynamic indices native, keeps ~4*NE floats out of the VGPR budget).
template <int NE>
struct EdgeRegs {
  v2 e0[NE], e1[NE];
  CX_MF v2 g0(int k) const {
    v2 r = e0[0];
#pragma unroll
    for (int q = 1; q < NE; ++q)
      if (q == k) r = e0[q];
    return r;
  }
  CX_MF v2 g1(int k) const {
    v2 r = e1[0];
#pragma unroll
    for (int q = 1; q < NE; ++q)
      if (q == k) r = e1[q];
    return r;
  }
  CX_MF void s0(int k, v2 v) {
#pragma unroll
    for (int q = 0; q < NE; ++q)
      if (q == k) e0[q] = v;
  }
  CX_MF void s1(int k, v2 v) {
#pragma unroll
    for (int q = 0; q < NE; ++q)
      if (q == k) e1[q] = v;
  }
};
struct EdgeCol {  // edge k, component c at p[(4k + c) * st]
  float* p;
  int st;
  CX_MF v2 g0(int k) const { return v2{p[(4 * k) * st], p[(4 * k + 1) * st]}; }
  CX_MF v2 g1(int k) const { return v2{p[(4 * k + 2) * st], p[(4 * k + 3) * st]}; }
  CX_MF void s0(int k, v2 v) {
    p[(4 * k) * st] = v.x;
    p[(4 * k + 1) * st] = v.y;
  }
  CX_MF void s1(int k, v2 v) {
    p[(4 * k + 2) * st] = v.x;
    p[(4 * k + 3) * st] = v.y;
  }
};

// epa_edge: EPA's final closest polytope edge (two Minkowski points) -- the
// penetration is its closest point to the origin (epa below); the backward
// (cotix_grad.h convex_contact_vjp) differentiates through the edge's points
template <int NE, class ES, class SA, class SB>
CX_DEV void epa_edge(const SA& a, const SB& b, const v2* simplex, int iters, ES& es, v2* e0, v2* e1) {
  float dist[NE];
  const v2 z = v2{0.0f, 0.0f};
#pragma unroll
  for (int k = 0; k < NE; ++k) {
    es.s0(k, z);
    es.s1(k, z);
  }
  es.s0(0, simplex[0]); es.s1(0, simplex[1]);
  es.s0(1, simplex[1]); es.s1(1, simplex[2]);
  es.s0(2, simplex[2]); es.s1(2, simplex[0]);
  const int ne = iters + 3;
  const v2 sim[3] = {simplex[0], simplex[1], simplex[2]};
#pragma unroll
  for (int k = 0; k < NE; ++k) dist[k] = (k < 3) ? edge_dist(sim[k], sim[(k + 1) % 3]) : ((k < ne) ? edge_dist(z, z) : finf());
  float bd = 0.0f;    // dist of the edge argmin_d picked
  auto argmin_d = [&]() {  // first NaN, else first minimum, over the ne live edges (selects)
    int nanidx = NE, b = 0;
    float bv = dist[0];
#pragma unroll
    for (int k = 1; k < NE; ++k) {
      const bool lt = k < ne && dist[k] < bv;
      bv = lt ? dist[k] : bv;
      b = lt ? k : b;
    }
#pragma unroll
    for (int k = NE - 1; k >= 0; --k) nanidx = (k < ne && isn(dist[k])) ? k : nanidx;
    bd = nanidx < NE ? qnan() : bv;
    return nanidx < NE ? nanidx : b;
  };
  int bei = argmin_d();
  v2 best0 = es.g0(bei), best1 = es.g1(bei);
  v2 newp = simplex[2];
  // the previous best edge (iteration 0: the simplex's edge 0) as the loop
  // condition reads it (:177-212): its unit normal and the norm of its
  // closest point to the origin.  Both are carried over from where that edge
  // was the best instead of recomputed -- the same expressions on the same
  // operands: the normal is the one the split direction used, and
  // nrm(closest_on_edge_to_origin(e)) == sqrt(edge_dist(e)) (the same sumsq;
  // a len-0 edge's -a and 0 - a square alike) except for the all-zero edge,
  // whose edge_dist is inf and whose closest point is the origin (norm 0).
  v2 pn = fnormal(sub(simplex[0], simplex[1]));
  pn = divs(pn, nrm(pn));
  float pd = dist[0];
  bool pz = simplex[0].x == 0.0f && simplex[0].y == 0.0f && simplex[1].x == 0.0f && simplex[1].y == 0.0f;
  for (int i = 0; i < iters; ++i) {
    bool c1 = sumsq(sub(best0, best1)) > 1e-9f;
    bool c2 = crs(best0, best1) >= 0.0f;
    float d = dot(newp, pn);
    float ed = pz ? 0.0f : __builtin_sqrtf(pd);
    bool c4 = (d - ed > 1e-6f) || (d <= 0.0f);
    if (!(c4 && !vnan(best0) && !vnan(best1) && c1 && c2)) break;
    v2 n = fnormal(sub(best0, best1));
    n = divs(n, nrm(n));
    newp = minkowski(a, b, n);
    const int slot = i + 3;
    const float dA = edge_dist(best0, newp), dB = edge_dist(newp, best1);
    es.s1(bei, newp);
    es.s0(slot, newp);
    es.s1(slot, best1);
#pragma unroll
    for (int k = 0; k < NE; ++k) {
      if (k == bei) dist[k] = dA;
      if (k == slot) dist[k] = dB;
    }
    pn = n;
    pd = bd;
    pz = best0.x == 0.0f && best0.y == 0.0f && best1.x == 0.0f && best1.y == 0.0f;
    bei = argmin_d();
    best0 = es.g0(bei);
    best1 = es.g1(bei);
  }
  *e0 = best0;
  *e1 = best1;
}
template <int NE, class ES, class SA, class SB>
CX_DEV v2 epa(const SA& a, const SB& b, const v2* simplex, int iters, ES& es) {
  v2 e0, e1;
  epa_edge<NE, ES>(a, b, simplex, iters, es, &e0, &e1);
  return closest_on_edge_to_origin(e0, e1);
}
template <int NE, class SA, class SB>
CX_DEV v2 epa(const SA& a, const SB& b, const v2* simplex, int iters) {
  EdgeRegs<NE> es;
  return epa<NE, EdgeRegs<NE>>(a, b, simplex, iters, es);
}

// generic-iteration EPA (circle_vs_polygon uses 128 iterations): buffer in
// private memory.  Not on either scenario's path.
template <class SA, class SB>
CX_DEV v2 epa_big(const SA& a, const SB& b, const v2* simplex, int iters) {
  constexpr int NE = 131;  // iters <= 128 (cotix_params bounds)
  v2 e0[NE], e1[NE];
  float dist[NE];
  const int ne = iters + 3;
  for (int k = 0; k < ne; ++k) { e0[k] = v2{0.0f, 0.0f}; e1[k] = v2{0.0f, 0.0f}; }
  e0[0] = simplex[0]; e1[0] = simplex[1];
  e0[1] = simplex[1]; e1[1] = simplex[2];
  e0[2] = simplex[2]; e1[2] = simplex[0];
  for (int k = 0; k < ne; ++k) dist[k] = edge_dist(e0[k], e1[k]);
  int bei = argmin_first(dist, ne);
  v2 best0 = e0[bei], best1 = e1[bei], newp = simplex[2], prev0 = e0[0], prev1 = e1[0];
  for (int i = 0; i < iters; ++i) {
    bool c1 = sumsq(sub(best0, best1)) > 1e-9f;
    bool c2 = crs(best0, best1) >= 0.0f;
    v2 n = fnormal(sub(prev0, prev1));
    n = divs(n, nrm(n));
    float d = dot(newp, n);
    float ed = nrm(closest_on_edge_to_origin(prev0, prev1));
    bool c4 = (d - ed > 1e-6f) || (d <= 0.0f);
    if (!(c4 && !vnan(best0) && !vnan(best1) && c1 && c2)) break;
    n = fnormal(sub(best0, best1));
    n = divs(n, nrm(n));
    newp = minkowski(a, b, n);
    e1[bei] = newp;
    dist[bei] = edge_dist(best0, newp);
    e0[i + 3] = newp;
    e1[i + 3] = best1;
    dist[i + 3] = edge_dist(newp, best1);
    prev0 = best0;
    prev1 = best1;
    bei = argmin_first(dist, ne);
    best0 = e0[bei];
    best1 = e1[bei];
  }
  return closest_on_edge_to_origin(best0, best1);
}

// ---------------------------------------------------------------------------
// edge-based contact point (cotix/_contacts.py:205-267)
// ---------------------------------------------------------------------------
CX_DEV v2 edge_vs_edge(v2 pa0, v2 pa1, v2 qb0, v2 qb1) {  // :206-225
  v2 p = pa0, r = sub(pa1, pa0), q = qb0, s = sub(qb1, qb0);
  auto c2 = [](v2 u, v2 v) { return u.x * v.y - v.x * u.y; };
  float c = c2(r, s);
  float t = c2(sub(q, p), s) / c;
  float u = c2(sub(q, p), r) / c;
  if (c != 0.0f && t >= 0.0f && t <= 1.0f && u >= 0.0f && u <= 1.0f) return add(p, scl(r, t));
  return v2{qnan(), qnan()};
}
// A and B as convex n-gons: polygon vertices v_k with edges (v_k, v_{k-1});
// an AABB is the 4-gon [up, (up.x,lo.y), lo, (lo.x,up.y)] with its own edge
// list [(v0,v1),(v1,v2),(v2,v3),(v3,v0)] (cotix/_convex_shapes.py:82-103).
// Computed on the fly from the shape view (no private edge arrays).
CX_DEV int cvx_count(const Shape& s) { return s.kind == KIND_AABB ? 4 : s.n; }
// vertex k (compile-time k after unrolling); `last` = vertex count-1 of a polygon
CX_DEV v2 cvx_vert(const Shape& s, int k) {
  if (s.kind == KIND_AABB) {
    const float x = (k == 0 || k == 1) ? s.w[2] : s.w[0];
    const float y = (k == 0 || k == 3) ? s.w[3] : s.w[1];
    return v2{x, y};
  }
  return v2{s.w[2 * k], s.w[2 * k + 1]};
}
CX_DEV void cvx_edge(const Shape& s, int k, v2 last, v2* e0, v2* e1) {
  if (s.kind == KIND_AABB) {
    *e0 = cvx_vert(s, k);
    *e1 = cvx_vert(s, (k + 1) & 3);
  } else {
    *e0 = cvx_vert(s, k);
    *e1 = k == 0 ? last : cvx_vert(s, k - 1);
  }
}
CX_DEV bool shape_contains(const Shape& s, v2 p) {
  if (s.kind == KIND_AABB) return aabb_contains(s, p);
  if (s.kind == KIND_CIRCLE) return circle_contains(s, p);
  return poly_contains(s, p);
}
// accumulation order (Appendix A): vertices of A in B, vertices of B in A,
// then edge intersections B-edge-major, A-edge-minor
CX_DEV v2 contact_from_edges(const Shape& A, const Shape& B) {
  float n = 0.0f;
  v2 acc = v2{0.0f, 0.0f};
  const int na = cvx_count(A), nb = cvx_count(B);
  const v2 lastA = A.kind == KIND_AABB ? v2{0.0f, 0.0f} : vert(A, A.n - 1);
  const v2 lastB = B.kind == KIND_AABB ? v2{0.0f, 0.0f} : vert(B, B.n - 1);
#pragma unroll
  for (int k = 0; k < MAXV; ++k)
    if (k < na) {
      const v2 v = cvx_vert(A, k);
      if (shape_contains(B, v)) { acc = add(acc, v); n = n + 1.0f; }
    }
#pragma unroll
  for (int k = 0; k < MAXV; ++k)
    if (k < nb) {
      const v2 v = cvx_vert(B, k);
      if (shape_contains(A, v)) { acc = add(acc, v); n = n + 1.0f; }
    }
#pragma unroll
  for (int jb = 0; jb < MAXV; ++jb)
    if (jb < nb) {
      v2 b0, b1;
      cvx_edge(B, jb, lastB, &b0, &b1);
#pragma unroll
      for (int ia = 0; ia < MAXV; ++ia)
        if (ia < na) {
          v2 a0, a1;
          cvx_edge(A, ia, lastA, &a0, &a1);
          v2 x = edge_vs_edge(a0, a1, b0, b1);
          if (!vnan(x)) { acc = add(acc, x); n = n + 1.0f; }
        }
    }
  if (n > 0.0f) return divs(acc, n);
  return v2{qnan(), qnan()};
}

// polygon_vs_polygon :294-315 / aabb_vs_polygon :270-291 (A may be an AABB).
// EPA runs iters = |A| + |B| + 1 <= 2*MAXV + 1 steps: at most 20 edges, so
// the edge buffer is a compile-time register array (epa<14> / epa<20>).
// GJK, then EPA when the penetration is needed (need_pen = false: the step
// kernel, for a part paired with itself -- such a cell is only ever chosen as
// j == i, which resolution skips, so only the NaN-ness of the contact point
// is observable; pen is then 0).  Returns whether the shapes collide.
#if defined(COTIX_PHASE_PROF) && (defined(__HIP__) || defined(__HIPCC__))
static __device__ unsigned long long g_dev_sub[4];  // phase-timing build: GJK / EPA cycles (tools/phase_prof.py)
#define CX_DSUB_T0 const unsigned long long cx_dsub_t0 = clock64()
#define CX_DSUB_T1(k)                                                                                   \
  do {                                                                                                  \
    const int l_ = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));             \
    if (l_ == __builtin_amdgcn_readfirstlane(l_)) atomicAdd(&g_dev_sub[k], clock64() - cx_dsub_t0);  \
  } while (0)
#define CX_CLOCK() clock64()
#define CX_DSUB_ADD(k, t0)                                                                          \
  do {                                                                                              \
    const int l_ = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));         \
    if (l_ == __builtin_amdgcn_readfirstlane(l_)) atomicAdd(&g_dev_sub[k], clock64() - (t0));    \
  } while (0)
#else
#define CX_DSUB_T0 ((void)0)
#define CX_DSUB_T1(k) ((void)0)
#define CX_CLOCK() 0ull
#define CX_DSUB_ADD(k, t0) ((void)(t0))
#endif
// edge (nullable): EPA's final edge (e0, e1), when EPA ran (the rollout
// forward records it for the backward's VJP, cotix_grad.h)
template <class SA, class SB, class MakeStore>
CX_DEV bool gjk_epa_t(const SA& a, const SB& b, const Shape& A, const Shape& B, const NarrowParams& np, bool need_pen,
                      v2* pen, MakeStore make, v2* edge = nullptr) {
  static_assert(2 * MAXV + 1 + 3 <= 20, "EPA buffer bound");
  v2 simplex[3];
  *pen = v2{0.0f, 0.0f};
#if defined(COTIX_ASM_MARKERS) && (defined(__HIP__) || defined(__HIPCC__))
  asm volatile(";#GJK_BEGIN");
#endif
  CX_DSUB_T0;
  const bool hit = gjk(a, b, np.d0, simplex, np.gjk_steps);
  CX_DSUB_T1(0);
#if defined(COTIX_ASM_MARKERS) && (defined(__HIP__) || defined(__HIPCC__))
  asm volatile(";#GJK_END");
#endif
  if (!hit) return false;
  const int it0 = (A.kind == KIND_AABB) ? (4 + B.n + 1) : (A.n + B.n + 1);  // min(48, ...): :271, :295
  const int iters = it0 < np.epa_cap ? it0 : np.epa_cap;
  if (!need_pen) return true;
  [[maybe_unused]] const unsigned long long cx_epa_t0 = CX_CLOCK();
  struct EpaTimer {  // phase-timing build: EPA cycles into slot 1 at scope exit
    unsigned long long t0;
    CX_MF ~EpaTimer() { CX_DSUB_ADD(1, t0); }
  } cx_epa_timer{cx_epa_t0};
  v2 e0, e1;  // epa() = epa_edge + its closest point
  if (iters + 3 <= 14) {
    auto es = make.template get<14>();
    epa_edge<14, decltype(es)>(a, b, simplex, iters, es, &e0, &e1);
  } else {
    auto es = make.template get<20>();
    epa_edge<20, decltype(es)>(a, b, simplex, iters, es, &e0, &e1);
  }
  *pen = closest_on_edge_to_origin(e0, e1);
  if (edge != nullptr) {
    edge[0] = e0;
    edge[1] = e1;
  }
  return true;
}
// POLY: both shapes are polygons (supports without the kind dispatch)
template <bool POLY, class MakeStore>
CX_DEV bool gjk_epa(const Shape& A, const Shape& B, const NarrowParams& np, bool need_pen, v2* pen, MakeStore make,
                    v2* edge = nullptr) {
  if constexpr (POLY) return gjk_epa_t(PolyRef{A}, PolyRef{B}, A, B, np, need_pen, pen, make, edge);
  else return gjk_epa_t(A, B, A, B, np, need_pen, pen, make, edge);
}
struct MakeRegs {
  template <int NE>
  CX_MF EdgeRegs<NE> get() const { return EdgeRegs<NE>{}; }
};
struct MakeCol {
  float* p;
  int st;
  template <int NE>
  CX_MF EdgeCol get() const { return EdgeCol{p, st}; }
};
// GJK, then EPA when the penetration is needed; EPA edges in registers
CX_DEV bool convex_vs_polygon_pen(const Shape& A, const Shape& B, const NarrowParams& np, bool need_pen, v2* pen) {
  return gjk_epa<false>(A, B, np, need_pen, pen, MakeRegs{});
}
// the same with EPA edges in a per-lane memory column (the step kernel's LDS)
// (POLY: both shapes are polygons)
template <bool POLY>
CX_DEV bool convex_vs_polygon_pen_col(const Shape& A, const Shape& B, const NarrowParams& np, bool need_pen, v2* pen,
                                      float* col, int stride, v2* edge = nullptr) {
  return gjk_epa<POLY>(A, B, np, need_pen, pen, MakeCol{col, stride}, edge);
}
CX_DEV Contact convex_vs_polygon(const Shape& A, const Shape& B, const NarrowParams& np, bool need_pen = true) {
  Contact c;
  if (!convex_vs_polygon_pen(A, B, np, need_pen, &c.pen)) return nan_contact();
  c.cp = contact_from_edges(A, B);
  return c;
}

// contact_from_edges split into independent terms, for the wave-cooperative
// evaluation in the step kernel: term s (0 <= s < cfe_terms) is a vertex of
// A inside B (s < |A|), a vertex of B inside A, or the intersection of B-edge
// jb and A-edge ia (B-edge-major); NaN = no contribution.  Summing the terms
// in s order reproduces contact_from_edges exactly.
CX_DEV int cfe_terms(const Shape& A, const Shape& B) {
  const int na = cvx_count(A), nb = cvx_count(B);
  return na + nb + na * nb;
}
// vertex k (varying per lane) of an AABB from its 4 words, or of a polygon
// through the caller's fetch (the step kernel reads it from LDS)
template <class VF>
CX_DEV v2 cvx_vert_d(const Shape& s, int k, VF vf) {
  if (s.kind == KIND_AABB) {
    const float x = bsel(k == 0 || k == 1, s.w[2], s.w[0]);
    const float y = bsel(k == 0 || k == 3, s.w[3], s.w[1]);
    return v2{x, y};
  }
  return vf(k);
}
template <class VF>
CX_DEV void cvx_edge_d(const Shape& s, int k, VF vf, v2* e0, v2* e1) {
  *e0 = cvx_vert_d(s, k, vf);
  if (s.kind == KIND_AABB) *e1 = cvx_vert_d(s, (k + 1) & 3, vf);
  else *e1 = vf(k == 0 ? s.n - 1 : k - 1);
}
template <class VFA, class VFB>
CX_DEV v2 cfe_term_contain(const Shape& A, const Shape& B, int s, VFA va, VFB vb) {  // s < |A| + |B|
  const int na = cvx_count(A);
  const v2 nanv = v2{qnan(), qnan()};
  // a vertex of A tested in B, or of B in A: one containment test on the selected pair
  const bool fa = s < na;
  const v2 vA = cvx_vert_d(A, fa ? s : 0, va), vB = cvx_vert_d(B, fa ? 0 : s - na, vb);
  const v2 v = fa ? vA : vB;
  Shape S;
  S.kind = fa ? B.kind : A.kind;
  S.n = fa ? B.n : A.n;
#pragma unroll
  for (int q = 0; q < 2 * MAXV; ++q) S.w[q] = bsel(fa, B.w[q], A.w[q]);
  return shape_contains(S, v) ? v : nanv;
}
template <class VFA, class VFB>
CX_DEV v2 cfe_term_edge(const Shape& A, const Shape& B, int s, VFA va, VFB vb) {  // s >= |A| + |B|
  const int na = cvx_count(A), nb = cvx_count(B);
  const int q = s - na - nb, jb = q / na, ia = q - jb * na;
  v2 a0, a1, b0, b1;
  cvx_edge_d(A, ia, va, &a0, &a1);
  cvx_edge_d(B, jb, vb, &b0, &b1);
  return edge_vs_edge(a0, a1, b0, b1);
}
template <class VFA, class VFB>
CX_DEV v2 cfe_term(const Shape& A, const Shape& B, int s, VFA va, VFB vb) {
  return s < cvx_count(A) + cvx_count(B) ? cfe_term_contain(A, B, s, va, vb) : cfe_term_edge(A, B, s, va, vb);
}

// circle_vs_polygon :157-202
CX_DEV Contact circle_vs_polygon(const Shape& C, const Shape& P, const NarrowParams& np) {
  v2 simplex[3];
  if (!gjk(C, P, np.d0, simplex, np.gjk_steps)) return nan_contact();
  Contact c;
  c.pen = epa_big(C, P, simplex, np.epa_cp);
  v2 pos = v2{C.d(1), C.d(2)};
  float dists[MAXV];
  v2 disps[MAXV];
  const v2 last = vert(P, P.n - 1);
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    dists[k] = 0.0f;
    disps[k] = v2{0.0f, 0.0f};
    if (k < P.n) {
      v2 a = v2{P.w[2 * k], P.w[2 * k + 1]}, b = k == 0 ? last : v2{P.w[2 * k - 2], P.w[2 * k - 1]};
      if (a.x == 0.0f && a.y == 0.0f && b.x == 0.0f && b.y == 0.0f) {
        disps[k] = v2{finf(), finf()};
      } else {
        float len = sumsq(sub(a, b));
        float t = dot(sub(pos, b), sub(a, b)) / len;
        t = clip_(t, 0.0f, 1.0f);
        disps[k] = sub(pos, add(b, scl(sub(a, b), t)));
      }
      dists[k] = sumsq(disps[k]);
    }
  }
  const int k = argmin_first_n<MAXV>(dists, P.n);
  v2 dk = disps[0];
  float sk = dists[0];
#pragma unroll
  for (int q = 1; q < MAXV; ++q)
    if (q == k) { dk = disps[q]; sk = dists[q]; }
  c.cp = add(pos, dk);
  if (sk > C.d(0) * C.d(0)) c.cp = pos;
  return c;
}

// contact function ids (the _contact_funcs registry, cotix/_colliders.py:21-35)
enum : int {
  FN_AABB_AABB = 0,
  FN_CIRCLE_CIRCLE = 1,
  FN_CIRCLE_AABB = 2,
  FN_POLY_POLY = 3,
  FN_AABB_POLY = 4,
  FN_CIRCLE_POLY = 5,
};
CX_DEV Contact run_contact(int fn, const Shape& a, const Shape& b, const NarrowParams& np, uint32_t* err) {
  switch (fn) {
    case FN_AABB_AABB: return aabb_vs_aabb(a, b);
    case FN_CIRCLE_CIRCLE: return circle_vs_circle(a, b);
    case FN_CIRCLE_AABB: return circle_vs_aabb(a, b, err);
    case FN_POLY_POLY:
    case FN_AABB_POLY: return convex_vs_polygon(a, b, np);
    default: return circle_vs_polygon(a, b, np);
  }
}

// ---------------------------------------------------------------------------
// bodies / resolution (cotix/_collision_resolution.py, cotix/_bodies.py)
// ---------------------------------------------------------------------------
struct Dyn {
  float px, py, vx, vy, a, w;
};
struct Params {
  float mass, inertia, elast, fric;
};
CX_DEV v2 velocity_at(const Dyn& b, v2 p) {  // _bodies.py:50-55
  v2 r = sub(p, v2{b.px, b.py});
  return v2{b.vx + (-r.y) * b.w, b.vy + r.x * b.w};
}
CX_DEV void apply_impulse(Dyn& b, const Params& m, v2 imp, v2 point) {  // :68-73
  v2 arm = sub(point, v2{b.px, b.py});
  float torque = crs(arm, imp);
  b.vx = b.vx + imp.x / m.mass;
  b.vy = b.vy + imp.y / m.mass;
  b.w = b.w + torque / m.inertia;
}
// resolve_collision (:52-151) split in two.  Every operand that does not
// depend on the two bodies' velocities -- the contact, the positions (the
// resolution changes velocities only) and the parameters -- is folded into
// ResPre, so the collider's sequential pass over the bodies carries only the
// velocity-dependent part.  The expressions and their evaluation order are
// the reference's; pre + seq is bit-identical to the one-piece form.
// Exact reciprocals of a body's mass and inertia (scene tables): r with
// x / d == x * r bit for bit for every x -- d = +-inf (r = +-0), +-0 (r =
// +-inf) or a normal power of two with a normal reciprocal -- or NaN when
// the division must be performed.
struct Rcp {
  float m, i;
};
CX_DEV Rcp no_rcp() { return Rcp{qnan(), qnan()}; }
// x / d; RCP: the scene guarantees d's exact reciprocal r (x * r, bit-identical)
template <bool RCP>
CX_DEV float div_r(float x, float d, float r) {
  if (RCP) return x * r;
  return x / d;
}
struct ResPre {
  v2 n, r1, r2, pen;  // pen / |pen|; cp - p1; cp - p2 (== velocity_at / apply_impulse arms); pen
  float den, pterm, ne, mu;  // (1/m1 + 1/m2) + ang; (0.3 |pen|) / 0.01; -(1 + e); (mu1 + mu2) / 2
};
// the penetration term's constants (baumgarte_term 0.3 and the divisor 0.01,
// cotix/_collision_resolution.py:105,115; cotix_params)
struct Baum {
  float k, dt;
};
CX_HD Baum baum_default() { return Baum{0.3f, 0.01f}; }
template <bool RCP = false>
CX_DEV ResPre resolve_pre(const Dyn& b1, const Params& m1, Rcp q1, const Dyn& b2, const Params& m2, Rcp q2, v2 pen,
                          v2 cp, Baum bm = baum_default()) {
  ResPre p;
  const float pn = nrm(pen);
  p.n = v2{pen.x / pn, pen.y / pn};
  const float e = fmin_(m1.elast, m2.elast);
  p.r1 = sub(cp, v2{b1.px, b1.py});
  p.r2 = sub(cp, v2{b2.px, b2.py});
  const float lev1 = p.r1.x * p.r1.x + p.r1.y * p.r1.y, lev2 = p.r2.x * p.r2.x + p.r2.y * p.r2.y;
  const float ang = div_r<RCP>(lev1, m1.inertia, q1.i) + div_r<RCP>(lev2, m2.inertia, q2.i);
  p.den = (div_r<RCP>(1.0f, m1.mass, q1.m) + div_r<RCP>(1.0f, m2.mass, q2.m)) + ang;
  p.pterm = (bm.k * nrm(pen)) / bm.dt;
  p.ne = -(1.0f + e);
  p.mu = (m1.fric + m2.fric) / 2.0f;
  p.pen = pen;
  return p;
}
// the velocity-dependent part on (vx, vy, w) of both bodies; false when the
// bodies move apart (:140-146) and nothing is applied
template <bool RCP = false>
CX_DEV bool resolve_seq(float& vx1, float& vy1, float& w1, const Params& m1, Rcp q1, float& vx2, float& vy2,
                        float& w2, const Params& m2, Rcp q2, const ResPre& p) {
  const v2 v1 = v2{vx1 + (-p.r1.y) * w1, vy1 + p.r1.x * w1};  // velocity_at(b1, cp)
  const v2 v2_ = v2{vx2 + (-p.r2.y) * w2, vy2 + p.r2.x * w2};
  const v2 relv = sub(v2_, v1);
  // moving apart (:140-146): nothing is applied, so the impulse (its divisions
  // and sqrt) is not computed -- the same early exit as below, taken first
  if (dot(p.pen, relv) < 0.0f) return false;
  const float vn = dot(relv, p.n);
  const float nim = p.ne * vn - p.pterm;
  const float ni = nim / p.den;
  v2 imp = scl(p.n, ni);
  const v2 vd = v2{relv.x + vn * p.n.x, relv.y + vn * p.n.y};
  const float vdn = nrm(vd);
  const v2 vdu = v2{vd.x / vdn, vd.y / vdn};
  float idr = (-vdn) / p.den;
  idr = clip_(idr, 0.0f, ni * p.mu);
  imp = add(imp, scl(vdu, idr));
  // apply_impulse(b1, -imp, cp), apply_impulse(b2, imp, cp)  (:68-73)
  const v2 i1 = neg(imp);
  const float t1 = crs(p.r1, i1), t2 = crs(p.r2, imp);
  vx1 = vx1 + div_r<RCP>(i1.x, m1.mass, q1.m);
  vy1 = vy1 + div_r<RCP>(i1.y, m1.mass, q1.m);
  w1 = w1 + div_r<RCP>(t1, m1.inertia, q1.i);
  vx2 = vx2 + div_r<RCP>(imp.x, m2.mass, q2.m);
  vy2 = vy2 + div_r<RCP>(imp.y, m2.mass, q2.m);
  w2 = w2 + div_r<RCP>(t2, m2.inertia, q2.i);
  return true;
}
CX_DEV bool resolve_collision(Dyn& b1, const Params& m1, Dyn& b2, const Params& m2, v2 pen, v2 cp,
                             Baum bm = baum_default()) {  // :52-151
  if (vnan(cp)) return false;
  const ResPre p = resolve_pre(b1, m1, no_rcp(), b2, m2, no_rcp(), pen, cp, bm);
  return resolve_seq(b1.vx, b1.vy, b1.w, m1, no_rcp(), b2.vx, b2.vy, b2.w, m2, no_rcp(), p);
}
CX_DEV v2 rotate(v2 v, float ang) {  // _geometry_utils.py:81-88
  float s, c;
  sincos32(ang, &s, &c);
  return v2{c * v.x + (-s) * v.y, s * v.x + c * v.y};
}

}  // namespace cx
