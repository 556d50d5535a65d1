// cotix_grad.h -- reverse-mode derivatives (VJPs) of the continuous part of
// the step, for the differentiable rollout (BASELINE config 5).
//
// Semantics are those of jax.grad through the reference: every branch in
// the analytic contacts and in the resolution is a jax.lax.cond
// (cotix/_contacts.py:30-154, cotix/_collision_resolution.py:52-65,140-146,
// cotix/_colliders.py:333), so only the executed branch is differentiated;
// argmin/argmax selections are constants; lax.max / lax.min (and jnp.clip,
// built from them) send the cotangent to the operand equal to the result and
// split it 1/2-1/2 on a tie (JAX's _balanced_eq JVP rule).  Each function
// recomputes its forward values with the exact f32 code of cotix_device.h,
// so branch decisions are those the forward step took.
//
// Shape gradients use the geometry layout of the forward path: circle
// (r, cx, cy, pad) and AABB (lo.x, lo.y, up.x, up.y); the radius, masses,
// inertias, elasticities and frictions are constants (not differentiated).
#pragma once
#include "cotix_device.h"

namespace cx {

CX_DEV void vjp_max(float x, float y, float g, float* gx, float* gy) {
  const float z = fmax_(x, y);
  const bool ex = x == z, ey = y == z;
  *gx += ex ? (ey ? 0.5f * g : g) : 0.0f;
  *gy += ey ? (ex ? 0.5f * g : g) : 0.0f;
}
CX_DEV void vjp_min(float x, float y, float g, float* gx, float* gy) {
  const float z = fmin_(x, y);
  const bool ex = x == z, ey = y == z;
  *gx += ex ? (ey ? 0.5f * g : g) : 0.0f;
  *gy += ey ? (ex ? 0.5f * g : g) : 0.0f;
}
// jnp.clip(x, lo, hi) = minimum(maximum(x, lo), hi)
CX_DEV void vjp_clip(float x, float lo, float hi, float g, float* gx, float* glo, float* ghi) {
  float gt = 0.0f;
  vjp_min(fmax_(x, lo), hi, g, &gt, ghi);
  vjp_max(x, lo, gt, gx, glo);
}
// d(v / |v|): cotangent g of the unit vector -> cotangent of v
CX_DEV v2 vjp_unit(v2 v, v2 g) {
  const float n = nrm(v);
  const float gn = -dot(g, v) / (n * n);
  return v2{g.x / n + gn * v.x / n, g.y / n + gn * v.y / n};
}

// aabb_vs_aabb (cotix/_contacts.py:61-96), contact branch
CX_DEV void aabb_vs_aabb_vjp(const Shape& a, const Shape& b, v2 gpen, v2 gcp, float* ga, float* gb) {
  const float alx = a.d(0), aly = a.d(1), aux = a.d(2), auy = a.d(3);
  const float blx = b.d(0), bly = b.d(1), bux = b.d(2), buy = b.d(3);
  const float me = -1e-8f;
  const float X[4] = {auy - bly, buy - aly, aux - blx, bux - alx};
  float dep[4];
  for (int q = 0; q < 4; ++q) dep[q] = fmax_(X[q], me);
  // (the direction and the picked words by selects: a constant array indexed
  // per lane is a global-memory read, whose s_waitcnt vmcnt(0) would also wait
  // for every store and prefetch in flight)
  const int k = argmin_first(dep, 4);
  const float gmd = gpen.x * pick4(k, 0.0f, 0.0f, -1.0f, 1.0f) + gpen.y * pick4(k, -1.0f, 1.0f, 0.0f, 0.0f);
  float gdep = 0.0f, gX = 0.0f, dummy = 0.0f;
  vjp_max(0.0f, pick4(k, dep[0], dep[1], dep[2], dep[3]), gmd, &dummy, &gdep);  // jnp.clip(depth, a_min=0)
  vjp_max(pick4(k, X[0], X[1], X[2], X[3]), me, gdep, &gX, &dummy);
  switch (k) {
    case 0: ga[3] += gX; gb[1] -= gX; break;
    case 1: gb[3] += gX; ga[1] -= gX; break;
    case 2: ga[2] += gX; gb[0] -= gX; break;
    default: gb[2] += gX; ga[0] -= gX; break;
  }
  const float hx = gcp.x / 2.0f, hy = gcp.y / 2.0f;  // cp = (min(up) + max(lo)) / 2
  vjp_min(aux, bux, hx, &ga[2], &gb[2]);
  vjp_min(auy, buy, hy, &ga[3], &gb[3]);
  vjp_max(alx, blx, hx, &ga[0], &gb[0]);
  vjp_max(aly, bly, hy, &ga[1], &gb[1]);
}

// circle_vs_circle (cotix/_contacts.py:30-58), contact branch
CX_DEV void circle_vs_circle_vjp(const Shape& a, const Shape& b, v2 gpen, v2 gcp, float* ga, float* gb) {
  const v2 ap = v2{a.d(1), a.d(2)}, bp = v2{b.d(1), b.d(2)};
  const float ar = a.d(0), br = b.d(0);
  const v2 delta = sub(ap, bp);
  const float dist = nrm(delta);
  const bool zero = dist == 0.0f;
  const v2 dir = zero ? v2{1.0f, 0.0f} : divs(delta, dist);
  const float mn = fmin_(dist - (ar + br), 0.0f);
  const v2 cp0 = divs(add(add(bp, scl(dir, br - ar)), ap), 2.0f);
  const bool sides = dot(sub(ap, cp0), sub(bp, cp0)) <= 0.0f;
  v2 gap = v2{0.0f, 0.0f}, gbp = v2{0.0f, 0.0f};
  const v2 gpr = neg(gpen);  // pen = -(dir * mn)
  v2 gdir = scl(gpr, mn);
  float gdist = 0.0f, dummy = 0.0f;
  vjp_min(dist - (ar + br), 0.0f, dot(gpr, dir), &gdist, &dummy);
  if (sides) {
    const v2 h = divs(gcp, 2.0f);
    gbp = add(gbp, h);
    gap = add(gap, h);
    gdir = add(gdir, scl(h, br - ar));
  } else if (circle_contains(a, bp)) {
    gbp = add(gbp, gcp);
  } else {
    gap = add(gap, gcp);
  }
  v2 gdelta = v2{0.0f, 0.0f};
  if (!zero) {
    gdelta = divs(gdir, dist);
    gdist += -dot(gdir, delta) / (dist * dist);
  }
  gdelta = add(gdelta, scl(divs(delta, dist), gdist));  // d|delta|
  gap = add(gap, gdelta);
  gbp = sub(gbp, gdelta);
  ga[1] += gap.x;
  ga[2] += gap.y;
  gb[1] += gbp.x;
  gb[2] += gbp.y;
}

// circle_vs_aabb (cotix/_contacts.py:99-154), contact branch
CX_DEV void circle_vs_aabb_vjp(const Shape& a, const Shape& b, v2 gpen, v2 gcp, float* ga, float* gb) {
  const v2 ap = v2{a.d(1), a.d(2)};
  const float r = a.d(0);
  const v2 lo = v2{b.d(0), b.d(1)}, up = v2{b.d(2), b.d(3)};
  const v2 bc = v2{(lo.x + up.x) / 2.0f, (lo.y + up.y) / 2.0f};
  const v2 disp = sub(ap, bc);
  const v2 l = sub(lo, bc), h = sub(up, bc);
  const v2 ccp = add(bc, v2{clip_(disp.x, l.x, h.x), clip_(disp.y, l.y, h.y)});
  const v2 vs[4] = {lo, v2{lo.x, up.y}, up, v2{up.x, lo.y}};
  bool perfect = false;
  for (int k = 0; k < 4; ++k) perfect = perfect || (nrm(sub(vs[k], ccp)) < 1e-6f);
  v2 gap = v2{0.0f, 0.0f}, glo = v2{0.0f, 0.0f}, gup = v2{0.0f, 0.0f};
  v2 gccp = gcp;
  if (perfect) {  // pen = -(ap + r * unit(ccp - ap) - ccp)
    const v2 d = sub(ccp, ap);
    gap = sub(gap, gpen);
    gccp = add(gccp, gpen);
    const v2 gd = vjp_unit(d, scl(gpen, -r));
    gccp = add(gccp, gd);
    gap = sub(gap, gd);
  } else {  // pen = -shift[k] * dir[k]
    const float sh[4] = {(ap.y + r) - lo.y, up.y - (ap.y - r), (ap.x + r) - lo.x, up.x - (ap.x - r)};
    const int k = argmin_first(sh, 4);  // (selects, not a constant array: see aabb_vs_aabb_vjp)
    const float g = -(gpen.x * pick4(k, 0.0f, 0.0f, 1.0f, -1.0f) + gpen.y * pick4(k, 1.0f, -1.0f, 0.0f, 0.0f));
    switch (k) {
      case 0: gap.y += g; glo.y -= g; break;
      case 1: gup.y += g; gap.y -= g; break;
      case 2: gap.x += g; glo.x -= g; break;
      default: gup.x += g; gap.x -= g; break;
    }
  }
  // ccp = bc + clip(ap - bc, lo - bc, up - bc)
  v2 gbc = gccp, gdisp = v2{0.0f, 0.0f}, gl = v2{0.0f, 0.0f}, gh = v2{0.0f, 0.0f};
  vjp_clip(disp.x, l.x, h.x, gccp.x, &gdisp.x, &gl.x, &gh.x);
  vjp_clip(disp.y, l.y, h.y, gccp.y, &gdisp.y, &gl.y, &gh.y);
  gap = add(gap, gdisp);
  gbc = sub(sub(sub(gbc, gdisp), gl), gh);
  glo = add(add(glo, gl), divs(gbc, 2.0f));
  gup = add(add(gup, gh), divs(gbc, 2.0f));
  ga[1] += gap.x;
  ga[2] += gap.y;
  gb[0] += glo.x;
  gb[1] += glo.y;
  gb[2] += gup.x;
  gb[3] += gup.y;
}

// reverse of run_contact for the analytic contacts
CX_DEV void contact_vjp(int fn, const Shape& a, const Shape& b, v2 gpen, v2 gcp, float* ga, float* gb) {
  switch (fn) {
    case FN_AABB_AABB: aabb_vs_aabb_vjp(a, b, gpen, gcp, ga, gb); break;
    case FN_CIRCLE_CIRCLE: circle_vs_circle_vjp(a, b, gpen, gcp, ga, gb); break;
    case FN_CIRCLE_AABB: circle_vs_aabb_vjp(a, b, gpen, gcp, ga, gb); break;
    default: break;  // polygon contacts are not differentiated (rejected on the host)
  }
}

// ---------------------------------------------------------------------------
// GJK / EPA contacts (polygon_vs_polygon cotix/_contacts.py:294-315,
// aabb_vs_polygon :270-291), contact branch.  EPA's supports are vertices of a
// polygon or corners of an AABB chosen by argmax (constants), so the
// penetration depends on the shapes only through the two Minkowski points of
// EPA's final edge (_closest_point_on_edge_to_point of that edge,
// cotix/_collisions.py:156-166,271-273); the contact point is the mean of the
// included contact_from_edges terms (:205-267, inclusion = the forward's
// containment / intersection tests, constants).  Cotangents are accumulated
// per vertex (cvx_vert order: polygon slots, AABB corners).
// ---------------------------------------------------------------------------
struct VGrad {
  float x[MAXV], y[MAXV];
  CX_MF void zero() {
#pragma unroll
    for (int k = 0; k < MAXV; ++k) x[k] = y[k] = 0.0f;
  }
  CX_MF void add(int k, v2 g) {  // k varies per lane: select chain, no scratch
#pragma unroll
    for (int q = 0; q < MAXV; ++q) {
      x[q] += q == k ? g.x : 0.0f;
      y[q] += q == k ? g.y : 0.0f;
    }
  }
};
// closest_on_edge_to_origin(a, b) (cotix_device.h) -> cotangents of a, b
CX_DEV void closest_vjp(v2 a, v2 b, v2 g, v2* ga, v2* gb) {
  const v2 d = sub(a, b);
  const float len = sumsq(d);
  if (len == 0.0f) {  // 0 - a
    *ga = sub(*ga, g);
    return;
  }
  const v2 pb = sub(v2{0.0f, 0.0f}, b);
  const float num = dot(pb, d), t = num / len, tc = clip_(t, 0.0f, 1.0f);
  const v2 gproj = neg(g);  // r = 0 - proj, proj = b + d * tc
  v2 gd = scl(gproj, tc);
  float gt = 0.0f, glo = 0.0f, ghi = 0.0f;
  vjp_clip(t, 0.0f, 1.0f, dot(gproj, d), &gt, &glo, &ghi);
  const float gnum = gt / len, glen = -gt * num / (len * len);
  gd = add(gd, scl(pb, gnum));
  gd = add(gd, scl(d, 2.0f * glen));
  const v2 gpb = scl(d, gnum);
  *ga = add(*ga, gd);
  *gb = sub(add(*gb, sub(gproj, gpb)), gd);
}
// the Minkowski point pt = vert_A(i) - vert_B(j): the first (i, j), A-major,
// whose difference equals pt (the oracle's rule, oracle/cotix_oracle/grad.py)
CX_DEV void minkowski_vjp(const Shape& A, const Shape& B, v2 pt, v2 g, VGrad& ga, VGrad& gb) {
  const int na = cvx_count(A), nb = cvx_count(B);
  int fi = -1, fj = -1;
#pragma unroll
  for (int i = 0; i < MAXV; ++i)
#pragma unroll
    for (int j = 0; j < MAXV; ++j)
      if (i < na && j < nb && fi < 0) {
        const v2 d = sub(cvx_vert(A, i), cvx_vert(B, j));
        if (d.x == pt.x && d.y == pt.y) {
          fi = i;
          fj = j;
        }
      }
  if (fi < 0) return;  // (not reached: EPA's points are Minkowski vertex pairs)
  ga.add(fi, g);
  gb.add(fj, neg(g));
}
// edge_vs_edge (cotix_device.h), intersecting branch: x = p + r t,
// t = crs(q - p, s) / crs(r, s); cotangent gx -> the four endpoints
CX_DEV void edge_vs_edge_vjp(v2 pa0, v2 pa1, v2 qb0, v2 qb1, v2 gx, v2* ga0, v2* ga1, v2* gb0, v2* gb1) {
  const v2 p = pa0, r = sub(pa1, pa0), q = qb0, s = sub(qb1, qb0), w = sub(q, p);
  const float c = r.x * s.y - s.x * r.y, nn = w.x * s.y - s.x * w.y, t = nn / c;
  v2 gp = gx, gr = scl(gx, t), gw = v2{0.0f, 0.0f}, gs = v2{0.0f, 0.0f};
  const float gt = dot(gx, r), gn = gt / c, gc = -gt * nn / (c * c);
  // crs(u, v) = u.x v.y - v.x u.y: d/du = (v.y, -v.x), d/dv = (-u.y, u.x)
  gw = add(gw, scl(v2{s.y, -s.x}, gn));
  gs = add(gs, scl(v2{-w.y, w.x}, gn));
  gr = add(gr, scl(v2{s.y, -s.x}, gc));
  gs = add(gs, scl(v2{-r.y, r.x}, gc));
  const v2 gq = gw;
  gp = sub(gp, gw);
  *ga1 = add(*ga1, gr);
  *ga0 = add(add(*ga0, gp), neg(gr));
  *gb1 = add(*gb1, gs);
  *gb0 = add(add(*gb0, gq), neg(gs));
}
// vertex k / edge k of a convex shape for a run-time k (select chains on the
// registers: no scratch copy of the shape); edge k = (v_k, v_prev(k))
CX_DEV v2 cvx_vert_r(const Shape& s, int k) {
  if (s.kind == KIND_AABB)
    return v2{(k == 0 || k == 1) ? s.w[2] : s.w[0], (k == 0 || k == 3) ? s.w[3] : s.w[1]};
  return vert(s, k);
}
CX_DEV int cvx_edge_prev(const Shape& s, int k) {
  if (s.kind == KIND_AABB) return (k + 1) & 3;
  return k == 0 ? s.n - 1 : k - 1;
}
// one pass: every included term's VJP with the cotangent gcp, then / n
// (cp = acc / n is linear in the terms).  The vertex and edge loops are
// unrolled to MAXV with k < n guards (as contact_from_edges): vertex picks
// and cotangent slots are compile-time indices (no select chains) except the
// wrap-around edge's last vertex.
CX_DEV void contact_from_edges_vjp(const Shape& A, const Shape& B, v2 gcp, VGrad& ga, VGrad& gb) {
  const int na = cvx_count(A), nb = cvx_count(B);
  const v2 lastA = A.kind == KIND_AABB ? v2{0.0f, 0.0f} : vert(A, A.n - 1);
  const v2 lastB = B.kind == KIND_AABB ? v2{0.0f, 0.0f} : vert(B, B.n - 1);
  VGrad ca, cb;
  ca.zero();
  cb.zero();
  float n = 0.0f;  // the forward's term count
#pragma unroll
  for (int k = 0; k < MAXV; ++k)
    if (k < na && shape_contains(B, cvx_vert(A, k))) {
      ca.x[k] += gcp.x;
      ca.y[k] += gcp.y;
      n = n + 1.0f;
    }
#pragma unroll
  for (int k = 0; k < MAXV; ++k)
    if (k < nb && shape_contains(A, cvx_vert(B, k))) {
      cb.x[k] += gcp.x;
      cb.y[k] += gcp.y;
      n = n + 1.0f;
    }
#pragma unroll
  for (int jb = 0; jb < MAXV; ++jb)
    if (jb < nb) {
      v2 b0, b1;
      cvx_edge(B, jb, lastB, &b0, &b1);
      const int pb = cvx_edge_prev(B, jb);
#pragma unroll
      for (int ia = 0; ia < MAXV; ++ia)
        if (ia < na) {
          v2 a0, a1;
          cvx_edge(A, ia, lastA, &a0, &a1);
          if (vnan(edge_vs_edge(a0, a1, b0, b1))) continue;
          n = n + 1.0f;
          v2 g0 = v2{0.0f, 0.0f}, g1 = g0, h0 = g0, h1 = g0;
          edge_vs_edge_vjp(a0, a1, b0, b1, gcp, &g0, &g1, &h0, &h1);
          ca.x[ia] += g0.x;
          ca.y[ia] += g0.y;
          ca.add(cvx_edge_prev(A, ia), g1);
          cb.x[jb] += h0.x;
          cb.y[jb] += h0.y;
          cb.add(pb, h1);
        }
    }
  if (!(n > 0.0f)) return;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    ga.x[k] += ca.x[k] / n;
    ga.y[k] += ca.y[k] / n;
    gb.x[k] += cb.x[k] / n;
    gb.y[k] += cb.y[k] / n;
  }
}
// the whole convex contact: re-runs GJK and EPA (the forward's exact code,
// so the final edge is the forward's) and returns the per-vertex cotangents;
// `make` supplies EPA's edge storage (MakeRegs: registers; MakeCol: a
// per-lane LDS column, as the step kernel's phase B)
template <class MakeStore = MakeRegs>
CX_DEV void convex_contact_vjp(const Shape& A, const Shape& B, const NarrowParams& np, v2 gpen, v2 gcp, VGrad& ga,
                               VGrad& gb, MakeStore make = MakeStore{}) {
  // (each half only for a nonzero cotangent: phase GE's unit cotangents
  // take one of the two paths per lane)
  if (gpen.x != 0.0f || gpen.y != 0.0f) {
    v2 simplex[3];
    if (gjk(A, B, np.d0, simplex, np.gjk_steps)) {  // (always, for a resolved contact)
      const int it0 = (A.kind == KIND_AABB) ? (4 + B.n + 1) : (A.n + B.n + 1);
      const int iters = it0 < np.epa_cap ? it0 : np.epa_cap;
      v2 e0, e1;
      if (iters + 3 <= 14) {
        auto es = make.template get<14>();
        epa_edge<14>(A, B, simplex, iters, es, &e0, &e1);
      } else {
        auto es = make.template get<20>();
        epa_edge<20>(A, B, simplex, iters, es, &e0, &e1);
      }
      v2 g0 = v2{0.0f, 0.0f}, g1 = v2{0.0f, 0.0f};
      closest_vjp(e0, e1, gpen, &g0, &g1);
      minkowski_vjp(A, B, e0, g0, ga, gb);
      minkowski_vjp(A, B, e1, g1, ga, gb);
    }
  }
  if (gcp.x != 0.0f || gcp.y != 0.0f) contact_from_edges_vjp(A, B, gcp, ga, gb);
}
// the same from EPA's final edge (e0, e1) as the forward recorded it (the
// rollout's tape, cotix_kernel.h): no GJK / EPA re-run -- the edge is the one
// convex_contact_vjp's re-run would find (the same code on the same shapes)
CX_DEV void convex_contact_vjp_edge(const Shape& A, const Shape& B, v2 e0, v2 e1, v2 gpen, v2 gcp, VGrad& ga,
                                    VGrad& gb) {
  if (gpen.x != 0.0f || gpen.y != 0.0f) {
    v2 g0 = v2{0.0f, 0.0f}, g1 = v2{0.0f, 0.0f};
    closest_vjp(e0, e1, gpen, &g0, &g1);
    minkowski_vjp(A, B, e0, g0, ga, gb);
    minkowski_vjp(A, B, e1, g1, ga, gb);
  }
  if (gcp.x != 0.0f || gcp.y != 0.0f) contact_from_edges_vjp(A, B, gcp, ga, gb);
}

// ---------------------------------------------------------------------------
// LunarLander joints (LunarLander.step, cotix/_lunar_lander.py:176-212; the
// forward is cotix_kernel.h lunar_constraints): four `fixed` impulse pairs,
// then the legs' angular damping.  In: the pre-joint bodies (lander, right
// leg, left leg) and the cotangents of the post-joint ones; out: the
// cotangents of the pre-joint bodies (positions and angles through the
// anchors, velocities through the impulses).
// ---------------------------------------------------------------------------
// d/dangle of rotate(v) = [[c,-s],[s,c]] v (JAX: d sin = cos, d cos = -sin)
CX_DEV float drot_dot(v2 g, v2 v, float s, float c) {
  return g.x * (-s * v.x - c * v.y) + g.y * (c * v.x - s * v.y);
}
CX_DEV void fixed_vjp(const Dyn& b1, const Params& m1, v2 c1, const Dyn& b2, const Params& m2, v2 c2, Dyn& g1, Dyn& g2,
                      v2& gc1, v2& gc2) {
  const float f05 = 0.05f;
  const v2 r1 = sub(c1, v2{b1.px, b1.py}), r2 = sub(c2, v2{b2.px, b2.py});
  const v2 dp = sub(c1, c2);
  const v2 dv = sub(velocity_at(b1, c1), velocity_at(b2, c2));
  const float nd = nrm(dv), k = nd + 0.1f;
  const v2 imp = v2{dp.x * 1.0f + (dv.x * k) * f05, dp.y * 1.0f + (dv.y * k) * f05};
  // apply_impulse(b1, -imp, c1), apply_impulse(b2, imp, c2)
  v2 gimp = v2{-g1.vx / m1.mass + g2.vx / m2.mass, -g1.vy / m1.mass + g2.vy / m2.mass};
  const float gt1 = g1.w / m1.inertia, gt2 = g2.w / m2.inertia;
  v2 gr1 = scl(v2{-imp.y, imp.x}, gt1), gr2 = scl(v2{imp.y, -imp.x}, gt2);  // torque = crs(r, -+imp)
  gimp = add(gimp, scl(v2{r1.y, -r1.x}, gt1));
  gimp = add(gimp, scl(v2{-r2.y, r2.x}, gt2));
  // imp = dp + (dv * k) * 0.05, k = |dv| + 0.1
  const v2 gdp = gimp;
  v2 gdv = scl(gimp, k * f05);
  const float gk = f05 * dot(gimp, dv);
  gdv = add(gdv, scl(divs(dv, nd), gk));
  // dv = velocity_at(b1, c1) - velocity_at(b2, c2); velocity_at = v + perp(c - p) w
  const v2 gu1 = gdv, gu2 = neg(gdv);
  Dyn o1 = g1, o2 = g2;
  o1.vx += gu1.x;
  o1.vy += gu1.y;
  o1.w += -r1.y * gu1.x + r1.x * gu1.y;
  gr1 = add(gr1, v2{gu1.y * b1.w, -gu1.x * b1.w});
  o2.vx += gu2.x;
  o2.vy += gu2.y;
  o2.w += -r2.y * gu2.x + r2.x * gu2.y;
  gr2 = add(gr2, v2{gu2.y * b2.w, -gu2.x * b2.w});
  // r = c - p; dp = c1 - c2
  gc1 = add(gc1, add(gr1, gdp));
  gc2 = add(gc2, sub(gr2, gdp));
  o1.px -= gr1.x;
  o1.py -= gr1.y;
  o2.px -= gr2.x;
  o2.py -= gr2.y;
  g1 = o1;
  g2 = o2;
}

// resolve_collision_notnan (cotix/_collision_resolution.py:76-146) in the
// branch that applies the impulses.  In: the pre-resolution bodies, the
// cotangents g1/g2 of the post-resolution bodies.  Out: g1/g2 become the
// cotangents of the pre-resolution bodies; gpen/gcp those of the contact.
CX_DEV void resolve_vjp(const Dyn& b1, const Params& m1, const Dyn& b2, const Params& m2, v2 pen, v2 cp, Dyn& g1,
                        Dyn& g2, v2& gpen, v2& gcp, Baum bm = baum_default()) {
  // forward values (cotix_device.h resolve_collision)
  const v2 r1 = sub(cp, v2{b1.px, b1.py}), r2 = sub(cp, v2{b2.px, b2.py});
  const v2 v1 = velocity_at(b1, cp), v2_ = velocity_at(b2, cp);
  const v2 relv = sub(v2_, v1);
  const float pn = nrm(pen);
  const v2 n = v2{pen.x / pn, pen.y / pn};
  const float vn = dot(relv, n);
  const float e = fmin_(m1.elast, m2.elast);
  const float lev1 = r1.x * r1.x + r1.y * r1.y, lev2 = r2.x * r2.x + r2.y * r2.y;
  const float ang = lev1 / m1.inertia + lev2 / m2.inertia;
  const float nim = (-(1.0f + e)) * vn - (bm.k * nrm(pen)) / bm.dt;
  const float den = (1.0f / m1.mass + 1.0f / m2.mass) + ang;
  const float ni = nim / den;
  const float mu = (m1.fric + m2.fric) / 2.0f;
  const v2 vd = v2{relv.x + vn * n.x, relv.y + vn * n.y};
  const float vdn = nrm(vd);
  const v2 vdu = v2{vd.x / vdn, vd.y / vdn};
  const float idr0 = (-vdn) / den;
  const float idr = clip_(idr0, 0.0f, ni * mu);
  const v2 imp = add(scl(n, ni), scl(vdu, idr));

  // apply_impulse(b1, -imp, cp); apply_impulse(b2, imp, cp)  (:68-73)
  v2 gimp = v2{-g1.vx / m1.mass + g2.vx / m2.mass, -g1.vy / m1.mass + g2.vy / m2.mass};
  v2 gr1 = v2{0.0f, 0.0f}, gr2 = v2{0.0f, 0.0f};
  {
    const float c1 = g1.w / m1.inertia;  // w1 += crs(r1, -imp) / I1
    gr1 = add(gr1, scl(v2{-imp.y, imp.x}, c1));
    gimp = add(gimp, scl(v2{r1.y, -r1.x}, c1));
    const float c2 = g2.w / m2.inertia;  // w2 += crs(r2, imp) / I2
    gr2 = add(gr2, scl(v2{imp.y, -imp.x}, c2));
    gimp = add(gimp, scl(v2{-r2.y, r2.x}, c2));
  }
  // imp = n * ni + vdu * idr
  v2 gn = scl(gimp, ni);
  float gni = dot(gimp, n);
  v2 gvdu = scl(gimp, idr);
  const float gidr = dot(gimp, vdu);
  // idr = clip(idr0, 0, ni * mu)
  float gidr0 = 0.0f, glo = 0.0f, ghi = 0.0f;
  vjp_clip(idr0, 0.0f, ni * mu, gidr, &gidr0, &glo, &ghi);
  gni += ghi * mu;
  // idr0 = -vdn / den
  float gvdn = -gidr0 / den;
  float gden = gidr0 * vdn / (den * den);
  // vdu = vd / vdn ; vdn = |vd|
  v2 gvd = divs(gvdu, vdn);
  gvdn += -dot(gvdu, vd) / (vdn * vdn);
  gvd = add(gvd, scl(divs(vd, vdn), gvdn));
  // vd = relv + vn * n
  v2 grelv = gvd;
  float gvn = dot(gvd, n);
  gn = add(gn, scl(gvd, vn));
  // ni = nim / den ; den = 1/m1 + 1/m2 + ang ; ang = lev1/I1 + lev2/I2
  const float gnim = gni / den;
  gden += -gni * nim / (den * den);
  gr1 = add(gr1, scl(r1, 2.0f * (gden / m1.inertia)));
  gr2 = add(gr2, scl(r2, 2.0f * (gden / m2.inertia)));
  // nim = -(1 + e) * vn - k * |pen| / dt
  gvn += -(1.0f + e) * gnim;
  float gpn = -(bm.k / bm.dt) * gnim;
  // vn = relv . n
  grelv = add(grelv, scl(n, gvn));
  gn = add(gn, scl(relv, gvn));
  // n = pen / |pen|
  gpen = add(gpen, vjp_unit(pen, gn));
  gpen = add(gpen, scl(divs(pen, pn), gpn));
  // relv = velocity_at(b2, cp) - velocity_at(b1, cp); velocity_at = v + perp(cp - p) * w
  const v2 gv2c = grelv, gv1c = neg(grelv);
  Dyn o1 = g1, o2 = g2;  // pass-through of every field
  o1.vx += gv1c.x;
  o1.vy += gv1c.y;
  o1.w += -r1.y * gv1c.x + r1.x * gv1c.y;
  gr1 = add(gr1, v2{gv1c.y * b1.w, -gv1c.x * b1.w});
  o2.vx += gv2c.x;
  o2.vy += gv2c.y;
  o2.w += -r2.y * gv2c.x + r2.x * gv2c.y;
  gr2 = add(gr2, v2{gv2c.y * b2.w, -gv2c.x * b2.w});
  // r = cp - p
  gcp = add(gcp, add(gr1, gr2));
  o1.px -= gr1.x;
  o1.py -= gr1.y;
  o2.px -= gr2.x;
  o2.py -= gr2.y;
  g1 = o1;
  g2 = o2;
}


// ---------------------------------------------------------------------------
// circle_vs_polygon (cotix/_contacts.py:157-202).  A circle's support is a
// function of the search direction (Circle.get_support, d / |d| * r + c,
// cotix/_convex_shapes.py:22-26), so the penetration depends on the circle
// through EVERY GJK and EPA point the final edge descends from: jax.grad
// differentiates the whole chain.  The forward is re-run with the exact
// arithmetic of cx::gjk / cx::epa_big (same decisions, same bits) while each
// Minkowski point records how its direction was made from earlier points;
// the reverse pass then walks the points in reverse creation order.  The
// polygon supports (argmax vertices) are constants.  Private memory (this
// pair is never on the benchmark scenes' path).
// ---------------------------------------------------------------------------
// direction kinds: CONST d0; NEG -p[a]; FN s * fnormal(p[a] - p[b]) (GJK);
// EPAN normalize(fnormal(p[a] - p[b])) (EPA; the circle support normalizes
// again)
enum : int { CP_CONST = 0, CP_NEG = 1, CP_FN = 2, CP_EPAN = 3 };
constexpr int CP_GJK_MAX = 32;  // the default gjk_max_steps: larger values are refused for gradients
constexpr int CP_NP = 3 + CP_GJK_MAX + 128;
struct CPRec {
  v2 p[CP_NP];
  int16_t pa[CP_NP], pb[CP_NP];
  int8_t kind[CP_NP], sg[CP_NP], vi[CP_NP];
  int n = 0;
};
// the polygon's support index for direction d (support(Shape), polygon branch:
// first NaN, else first maximum of v . d)
CX_DEV int poly_support_idx(const Shape& s, v2 d) {
  float bv = s.w[0] * d.x + s.w[1] * d.y;
  int bk = 0;
  for (int k = 1; k < MAXV; ++k) {
    const float x = s.w[2 * k], y = s.w[2 * k + 1];
    const float t = x * d.x + y * d.y;
    const bool take = (k < s.n) & !isn(bv) & (isn(t) | (t > bv));
    bv = take ? t : bv;
    bk = take ? k : bk;
  }
  return bk;
}
// minkowski(C, P, d) = support(C, d) - support(P, -d), recorded
CX_DEV int cp_point(const Shape& C, const Shape& P, v2 d, int kind, int a, int b, int sg, CPRec& R) {
  const int k = poly_support_idx(P, neg(d));
  const v2 pt = sub(support(C, d), vert(P, k));
  const int id = R.n++;
  R.p[id] = pt;
  R.pa[id] = (int16_t)a;
  R.pb[id] = (int16_t)b;
  R.kind[id] = (int8_t)kind;
  R.sg[id] = (int8_t)sg;
  R.vi[id] = (int8_t)k;
  return id;
}
// GJK (cx::gjk) + EPA (cx::epa_big) of circle C vs polygon P, recorded; false
// when there is no contact.  e0 / e1: the ids of EPA's final edge
CX_DEV bool cp_forward(const Shape& C, const Shape& P, const NarrowParams& np, CPRec& R, int* e0, int* e1) {
  R.n = 0;
  int i0 = cp_point(C, P, np.d0, CP_CONST, -1, -1, 1, R);
  v2 s0 = R.p[i0];
  int i1 = cp_point(C, P, neg(s0), CP_NEG, i0, -1, 1, R);
  v2 s1 = R.p[i1];
  v2 dir = fnormal(sub(s1, s0));
  const int fa = i1, fb = i0;  // dir = +-fnormal(p[i1] - p[i0])
  int sg = 1;
  {
    const bool sw = dot(dir, neg(s1)) > 0.0f;
    const v2 t0 = s0;
    const int j0 = i0;
    s0 = sw ? s1 : s0;
    i0 = sw ? i1 : i0;
    s1 = sw ? t0 : s1;
    i1 = sw ? j0 : i1;
    dir = sw ? dir : neg(dir);
    sg = sw ? 1 : -1;
  }
  int i2 = cp_point(C, P, dir, CP_FN, fa, fb, sg, R);
  v2 s2 = R.p[i2];
  for (int step = 0; step < np.gjk_steps; ++step) {
    bool c1 = dot(s2, dir) <= 0.0f;
    bool c2 = dot(fnormal(sub(s2, s0)), neg(s2)) < 0.0f;
    bool c3 = dot(fnormal(sub(s1, s2)), neg(s2)) < 0.0f;
    if (c1 || (c2 && c3)) break;
    if (R.n >= 3 + CP_GJK_MAX) return false;  // (not reached: gjk_max_steps <= CP_GJK_MAX is checked at launch)
    const v2 c = s2;
    const int ic = i2;
    const v2 acn = fnormal(sub(c, s0)), cbn = fnormal(sub(s1, c));
    const bool ac = dot(acn, neg(c)) >= 0.0f;
    const int pa = ac ? ic : i1, pb = ac ? i0 : ic;  // acn = fnormal(c - s0), cbn = fnormal(s1 - c)
    s1 = ac ? c : s1;
    i1 = ac ? ic : i1;
    s0 = ac ? s0 : c;
    i0 = ac ? i0 : ic;
    dir = ac ? acn : cbn;
    i2 = cp_point(C, P, dir, CP_FN, pa, pb, 1, R);
    s2 = R.p[i2];
  }
  if (!point_in_triangle0(s0, s1, s2)) return false;
  const float area = crs(sub(s1, s0), sub(s2, s0));
  const bool allzero = s0.x == 0.0f && s0.y == 0.0f && s1.x == 0.0f && s1.y == 0.0f && s2.x == 0.0f && s2.y == 0.0f;
  if (allzero || vnan(s0) || vnan(s1) || vnan(s2) || area == 0.0f) return false;
  // EPA (epa_big), edge ids alongside the edges
  constexpr int NE = 131;
  v2 g0[NE], g1[NE];
  int16_t d0[NE], d1[NE];
  float dist[NE];
  const int iters = np.epa_cp, ne = iters + 3;
  const v2 z = v2{0.0f, 0.0f};
  for (int k = 0; k < ne; ++k) {
    g0[k] = z;
    g1[k] = z;
    d0[k] = d1[k] = -1;
  }
  g0[0] = s0; g1[0] = s1; d0[0] = (int16_t)i0; d1[0] = (int16_t)i1;
  g0[1] = s1; g1[1] = s2; d0[1] = (int16_t)i1; d1[1] = (int16_t)i2;
  g0[2] = s2; g1[2] = s0; d0[2] = (int16_t)i2; d1[2] = (int16_t)i0;
  for (int k = 0; k < ne; ++k) dist[k] = edge_dist(g0[k], g1[k]);
  int bei = argmin_first(dist, ne);
  v2 best0 = g0[bei], best1 = g1[bei], newp = s2, prev0 = g0[0], prev1 = g1[0];
  int b0 = d0[bei], b1 = d1[bei];
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
    const int ip = cp_point(C, P, n, CP_EPAN, b0, b1, 1, R);
    newp = R.p[ip];
    g1[bei] = newp;
    d1[bei] = (int16_t)ip;
    dist[bei] = edge_dist(best0, newp);
    g0[i + 3] = newp;
    g1[i + 3] = best1;
    d0[i + 3] = (int16_t)ip;
    d1[i + 3] = (int16_t)b1;
    dist[i + 3] = edge_dist(newp, best1);
    prev0 = best0;
    prev1 = best1;
    bei = argmin_first(dist, ne);
    best0 = g0[bei];
    best1 = g1[bei];
    b0 = d0[bei];
    b1 = d1[bei];
  }
  *e0 = b0;
  *e1 = b1;
  return true;
}
// fnormal(a - b) = (-(a.y - b.y), a.x - b.x): cotangent g -> a, b
CX_DEV void fnormal_diff_vjp(v2 g, v2* ga, v2* gb) {
  ga->x += g.y;
  gb->x -= g.y;
  ga->y -= g.x;
  gb->y += g.x;
}
// the VJP: cotangents (gpen, gcp) of the contact -> the circle's centre (gc)
// and the polygon's world vertices (gv).  False when the re-run finds no
// contact (not reached for a resolved contact)
// (not inlined: its private point record and EPA buffer stay out of the
// calling kernel's register allocation; only this rare pair pays the call)
#if defined(__HIP__)
__device__ __attribute__((noinline))
#else
static
#endif
bool circle_poly_vjp(const Shape& C, const Shape& P, const NarrowParams& np, v2 gpen, v2 gcp, v2* gc, VGrad& gv) {
  CPRec R;
  int e0 = -1, e1 = -1;
  if (!cp_forward(C, P, np, R, &e0, &e1)) return false;
  const float r = C.d(0);
  const v2 pos = v2{C.d(1), C.d(2)};
  v2 g[CP_NP];
  for (int k = 0; k < R.n; ++k) g[k] = v2{0.0f, 0.0f};
  // pen = closest_on_edge_to_origin(e0, e1) (:270-273); a zero edge (never
  // a contact's) has no points
  if (e0 >= 0 && e1 >= 0) closest_vjp(R.p[e0], R.p[e1], gpen, &g[e0], &g[e1]);
  for (int k = R.n - 1; k >= 0; --k) {
    const v2 gp = g[k];
    if (gp.x == 0.0f && gp.y == 0.0f) continue;
    *gc = add(*gc, gp);          // + c
    gv.add(R.vi[k], neg(gp));    // - vertex
    const int kd = R.kind[k], a = R.pa[k], b = R.pb[k];
    // the direction u handed to the circle support, and the point's value
    // through it: p = (u / |u|) * r + c - v
    v2 u;
    v2 fn = v2{0.0f, 0.0f};
    if (kd == CP_CONST) u = np.d0;
    else if (kd == CP_NEG) u = neg(R.p[a]);
    else {
      fn = fnormal(sub(R.p[a], R.p[b]));
      u = kd == CP_EPAN ? divs(fn, nrm(fn)) : (R.sg[k] > 0 ? fn : neg(fn));
    }
    const v2 gu = vjp_unit(u, scl(gp, r));
    if (kd == CP_NEG) {
      g[a] = sub(g[a], gu);
    } else if (kd == CP_FN) {
      const v2 gfn = R.sg[k] > 0 ? gu : neg(gu);
      fnormal_diff_vjp(gfn, &g[a], &g[b]);
    } else if (kd == CP_EPAN) {
      fnormal_diff_vjp(vjp_unit(fn, gu), &g[a], &g[b]);
    }
  }
  // the contact point (:168-197): the polygon edge k = (v_k, v_{k-1}) nearest
  // the centre, or the centre when it is farther than r
  float dists[MAXV];
  v2 disps[MAXV];
  const v2 last = vert(P, P.n - 1);
  for (int k = 0; k < MAXV; ++k) {
    dists[k] = 0.0f;
    disps[k] = v2{0.0f, 0.0f};
    if (k < P.n) {
      const v2 a = v2{P.w[2 * k], P.w[2 * k + 1]}, b = k == 0 ? last : v2{P.w[2 * k - 2], P.w[2 * k - 1]};
      if (a.x == 0.0f && a.y == 0.0f && b.x == 0.0f && b.y == 0.0f) {
        disps[k] = v2{finf(), finf()};
      } else {
        const float len = sumsq(sub(a, b));
        float t = dot(sub(pos, b), sub(a, b)) / len;
        t = clip_(t, 0.0f, 1.0f);
        disps[k] = sub(pos, add(b, scl(sub(a, b), t)));
      }
      dists[k] = sumsq(disps[k]);
    }
  }
  const int k = argmin_first_n<MAXV>(dists, P.n);
  *gc = add(*gc, gcp);  // cp = pos (+ disp)
  float sk = dists[0];
  for (int q = 1; q < MAXV; ++q)
    if (q == k) sk = dists[q];
  if (!(sk > r * r)) {
    const int kb = k == 0 ? P.n - 1 : k - 1;
    const v2 a = vert(P, k), b = vert(P, kb);
    if (!(a.x == 0.0f && a.y == 0.0f && b.x == 0.0f && b.y == 0.0f)) {
      // disp = pos - (b + d * tc), d = a - b, tc = clip(dot(pos - b, d) / |d|^2, 0, 1)
      const v2 d = sub(a, b), pb = sub(pos, b);
      const float len = sumsq(d), num = dot(pb, d), t = num / len, tc = clip_(t, 0.0f, 1.0f);
      const v2 gdisp = gcp, gproj = neg(gdisp);
      *gc = add(*gc, gdisp);
      v2 ga = v2{0.0f, 0.0f}, gb = gproj, gd = scl(gproj, tc);
      float gt = 0.0f, glo = 0.0f, ghi = 0.0f;
      vjp_clip(t, 0.0f, 1.0f, dot(gproj, d), &gt, &glo, &ghi);
      const float gnum = gt / len, glen = -gt * num / (len * len);
      *gc = add(*gc, scl(d, gnum));
      gb = sub(gb, scl(d, gnum));
      gd = add(gd, scl(pb, gnum));
      gd = add(gd, scl(d, 2.0f * glen));
      ga = add(ga, gd);
      gb = sub(gb, gd);
      gv.add(k, ga);
      gv.add(kb, gb);
    }
  }
  return true;
}

}  // namespace cx
