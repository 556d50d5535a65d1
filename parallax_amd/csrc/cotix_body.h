// cotix_body.h -- body-level operators of UniversalShape
// (cotix/_universal_shape.py:87-132), one env per call; shared by the gfx950
// operator kernels (cotix_step.hip) and the host emulation of the tests.
#pragma once
#include "../../include/cotix_amd.h"
#include "cotix_device.h"

namespace cxk {

constexpr int MAXBP = 16;  // parts per body
struct BodyParts {
  int body, n;
  int kind[MAXBP], nv[MAXBP], goff[MAXBP];
};

CX_DEV cx::WrappedShape wrapped_part(const BodyParts& bp, int k, const float* lg, float c, float sn, float px,
                                     float py) {
  cx::WrappedShape w;
  w.s.kind = bp.kind[k];
  w.s.n = bp.nv[k];
  const int nw = bp.kind[k] == cx::KIND_POLY ? 2 * bp.nv[k] : (bp.kind[k] == cx::KIND_AABB ? 4 : 3);
  for (int q = 0; q < 2 * cx::MAXV; ++q) w.s.w[q] = q < nw ? lg[bp.goff[k] + q] : 0.0f;
  w.c = c;
  w.sn = sn;
  w.px = px;
  w.py = py;
  return w;
}
CX_DEV void body_frame(const float* dyn, int B, int body, int g, float* c, float* sn, float* px, float* py) {
  const float* d = dyn + (size_t)body * 6 * B + g;
  *px = d[0];
  *py = d[(size_t)B];
  cx::sincos32(d[4 * (size_t)B], sn, c);  // HomogenuousTransformer (cotix/_geometry_utils.py:91-112)
}

// collides_with (GJK over every part pair, the first colliding pair's simplex
// kept, :87-107), then penetrates_with / penetration_depth (EPA, 48
// iterations, :112-132).  Returns collides; *pen = 0 when not colliding.
CX_DEV bool body_penetration_env(const float* dyn, int B, const float* geom, int gstride, const BodyParts& pa,
                                 const BodyParts& pb, cx::v2 d0, int g, cx::v2* pen) {
  const float* lg = geom + (gstride ? (size_t)g * gstride : (size_t)0);
  float ca, sa, xa, ya, cb, sb, xb, yb;
  body_frame(dyn, B, pa.body, g, &ca, &sa, &xa, &ya);
  body_frame(dyn, B, pb.body, g, &cb, &sb, &xb, &yb);
  bool hit = false;
  int fa = 0, fb = 0;
  cx::v2 simplex[3] = {cx::v2{0.0f, 0.0f}, cx::v2{0.0f, 0.0f}, cx::v2{0.0f, 0.0f}};
  for (int i = 0; i < pa.n; ++i)
    for (int j = 0; j < pb.n; ++j) {
      const cx::WrappedShape A = wrapped_part(pa, i, lg, ca, sa, xa, ya), Bs = wrapped_part(pb, j, lg, cb, sb, xb, yb);
      cx::v2 sx[3];
      const bool r = cx::gjk(A, Bs, d0, sx);
      if (!hit && r) {
        simplex[0] = sx[0];
        simplex[1] = sx[1];
        simplex[2] = sx[2];
        fa = i;
        fb = j;
      }
      hit = hit || r;
    }
  *pen = cx::v2{0.0f, 0.0f};
  if (hit) {
    const cx::WrappedShape A = wrapped_part(pa, fa, lg, ca, sa, xa, ya), Bs = wrapped_part(pb, fb, lg, cb, sb, xb, yb);
    *pen = cx::epa_big(A, Bs, simplex, 48);
  }
  return hit;
}

// AABB.of (cotix/_convex_shapes.py:68-77) of a whole body through its global
// support (get_global_support, cotix/_universal_shape.py:47-59): a working
// version of the reference's possibly_collides_with broadphase (:109-110,
// which calls the non-existent AABB.of_universal).  out = lo.x, lo.y, up.x,
// up.y; returns the error bits (eqx.error_if with EQX_ON_ERROR=nan).
CX_DEV uint32_t body_aabb_env(const float* dyn, int B, const float* geom, int gstride, const BodyParts& pa, int g,
                              float* out) {
  const float* lg = geom + (gstride ? (size_t)g * gstride : (size_t)0);
  float c, sn, px, py;
  body_frame(dyn, B, pa.body, g, &c, &sn, &px, &py);
  const cx::v2 dirs[4] = {cx::v2{-1.0f, 0.0f}, cx::v2{0.0f, -1.0f}, cx::v2{1.0f, 0.0f}, cx::v2{0.0f, 1.0f}};
  float r[4];
  for (int q = 0; q < 4; ++q) {
    cx::v2 best = cx::v2{0.0f, 0.0f};
    float bv = 0.0f;
    bool have = false, nan = false;
    for (int k = 0; k < pa.n; ++k) {  // supports[argmax(dot)]: first NaN, else first maximum
      const cx::v2 sp = cx::support(wrapped_part(pa, k, lg, c, sn, px, py), dirs[q]);
      const float t = cx::dot(sp, dirs[q]);
      if (nan) continue;
      if (!have || cx::isn(t) || t > bv) {
        best = sp;
        bv = t;
        have = true;
        nan = cx::isn(t);
      }
    }
    r[q] = (q % 2 == 0) ? best.x : best.y;
  }
  uint32_t e = 0u;
  if (r[2] <= r[0]) {
    e |= COTIX_ERR_AABB_INVALID;
    r[2] = cx::qnan();
  }
  if (r[3] <= r[1]) {
    e |= COTIX_ERR_AABB_INVALID;
    r[3] = cx::qnan();
  }
  for (int q = 0; q < 4; ++q) out[q] = r[q];
  return e;
}

}  // namespace cxk
