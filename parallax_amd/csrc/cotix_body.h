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
// iterations by default -- cotix_params epa_body_iters --, :112-132).  Returns collides; *pen = 0 when not colliding.
CX_DEV bool body_penetration_env(const float* dyn, int B, const float* geom, int gstride, const BodyParts& pa,
                                 const BodyParts& pb, const cx::NarrowParams& np, int g, cx::v2* pen) {
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
      const bool r = cx::gjk(A, Bs, np.d0, sx, np.gjk_steps);
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
    *pen = cx::epa_big(A, Bs, simplex, np.epa_body);  // solver_iterations=48, :120
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

// ---------------------------------------------------------------------------
// render export: the geometry of env.draw(painter) (cotix/_robocup.py:140-150,
// cotix/_lunar_lander.py:220-225) as a per-env primitive table instead of
// jax.debug.callback draws (cotix/_viz.py:55-75).  Per part, in scene order:
//   Circle  -> 1 primitive  (cx, cy, r, NaN)          Circle.draw, :43-44
//   AABB    -> 4 edge lines (x0, y0, x1, y1)          AABB.drawEdges / get_edges, :82-93,131-133
//   Polygon -> n edge lines (v_k, v_{k-1})            Polygon.drawEdges / get_edges, :160-163,192-194
// of the part transformed by its body (Polygon.transform re-sorts, :181-187).
// Colours and draw order are static (host side, parallax_amd/render.py).
constexpr int MAXRP = 32;  // parts per scene
struct SceneParts {
  int np;
  int body[MAXRP], kind[MAXRP], nv[MAXRP], goff[MAXRP], poff[MAXRP];
};
CX_HD int render_prims(int kind, int nv) { return kind == cx::KIND_CIRCLE ? 1 : (kind == cx::KIND_AABB ? 4 : nv); }
CX_DEV void render_part_env(const float* dyn, int B, const float* geom, int gstride, const SceneParts& sp, int p, int g,
                            float* out) {
  const float* lg = geom + (gstride ? (size_t)g * gstride : (size_t)0) + sp.goff[p];
  float c, sn, px, py;
  body_frame(dyn, B, sp.body[p], g, &c, &sn, &px, &py);
  float* o = out + 4 * sp.poff[p];
  if (sp.kind[p] == cx::KIND_CIRCLE) {  // Circle.transform: position + shift (:37-41)
    o[0] = lg[1] + px;
    o[1] = lg[2] + py;
    o[2] = lg[0];
    o[3] = cx::qnan();
  } else if (sp.kind[p] == cx::KIND_AABB) {  // lower/upper + shift (:113-117); vs = up, (up.x, lo.y), lo, (lo.x, up.y)
    const float lx = lg[0] + px, ly = lg[1] + py, ux = lg[2] + px, uy = lg[3] + py;
    const float vx[4] = {ux, ux, lx, lx}, vy[4] = {uy, ly, ly, uy};
    for (int k = 0; k < 4; ++k) {
      o[4 * k + 0] = vx[k];
      o[4 * k + 1] = vy[k];
      o[4 * k + 2] = vx[(k + 1) & 3];
      o[4 * k + 3] = vy[(k + 1) & 3];
    }
  } else {  // forward_vector of every vertex (the step kernel's phase T arithmetic), then order_clockwise
    const int n = sp.nv[p];
    cx::Poly q;
    for (int k = 0; k < cx::MAXV; ++k) {
      q.x[k] = 0.0f;
      q.y[k] = 0.0f;
      if (k < n) {
        const float x = lg[2 * k], y = lg[2 * k + 1];
        const float t0 = (c * x + (-sn) * y) + px * 1.0f, t1 = (sn * x + c * y) + py * 1.0f;
        const float t2 = (0.0f * x + 0.0f * y) + 1.0f * 1.0f;
        q.x[k] = t2 == 1.0f ? t0 : cx::qnan();
        q.y[k] = t2 == 1.0f ? t1 : cx::qnan();
      }
    }
    const cx::Poly v = cx::order_clockwise(q, n);
    for (int k = 0; k < n; ++k) {
      const int km = k == 0 ? n - 1 : k - 1;
      o[4 * k + 0] = v.x[k];
      o[4 * k + 1] = v.y[k];
      o[4 * k + 2] = v.x[km];
      o[4 * k + 3] = v.y[km];
    }
  }
}

// class_invariant (cotix/_design_by_contract.py:80-107) of a body's dynamic
// state: every word finite ("detect jnp.nans or invalid values early")
CX_DEV uint32_t state_check_env(const float* dyn, int n_bodies, int B, int g) {
  bool bad = false;
  for (int k = 0; k < 6 * n_bodies; ++k) {
    const float v = dyn[(size_t)k * B + g];
    bad = bad | cx::isn(v) | __builtin_isinf(v);
  }
  return bad ? (uint32_t)COTIX_ERR_STATE_NONFINITE : 0u;
}

}  // namespace cxk
