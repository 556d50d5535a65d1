// cotix_kernel.h -- the fused step as phase functions + the scene tables.
//
// Shared by the gfx950 kernel (cotix_step.hip: phases separated by
// __syncthreads) and by the CPU emulation harness of the tests (tests/emu:
// every phase run for all lanes in turn, under AddressSanitizer).
//
// Design (DESIGN.md "Kernels"): one workgroup owns a tile of E environments
// for all n_steps of a launch; the tile's state lives in LDS laid out
// [word][env] (env fastest -> conflict-free, coalesced) and every phase of a
// step is spread over the workgroup's lanes as (item, env) pairs with env
// fastest, so the lanes of a wave run the same item (same contact function,
// same cell) for consecutive envs:
//   A  Euler (+gravity, +action), per-env key chain     (item = body)
//   T  part transforms + order_clockwise                  (item = part)
//   B  distinct narrowphase contacts (+error bits)        (item = contact)
//   C  per-cell "last passing candidate" RNG scan         (item = cell)
//   D  per-body contact choice (jr.choice)                (item = body)
//   E  sequential resolution, LunarLander joints, key     (item = env)
// Phase C replaces the reference's sequential N2 x N1 scatter scan
// (cotix/_colliders.py:208-268) by an exact equivalent: for every cell
// (i, j) only the LAST candidate (in scan order) whose contact is non-NaN
// and whose bernoulli passes determines all_contacts[i, j], so each cell is
// scanned backwards and stops at the first pass; duplicate contacts (the
// same part pair repeated in the candidate lists) are evaluated once.
#pragma once
#include "../../include/cotix_amd.h"
#include "cotix_device.h"

namespace cxk {

constexpr int MAXB = 16, MAXP = 32, MAXC = 256, MAXL = 128, MAXT = 13, MAXCAND = 4096;
constexpr int BLK = 256;

struct SceneDev {
  int nb, np, nc, nl, nt, G, W;  // bodies, parts, contacts, cells, types, geom floats, world floats
  float d0x, d0y;                // GJK start direction (constant)
  cx::Params par[MAXB];
  int part_body[MAXP], part_kind[MAXP], part_n[MAXP], part_goff[MAXP], part_woff[MAXP];
  int c_pa[MAXC], c_pb[MAXC], c_fn[MAXC];
  int cell_i[MAXL], cell_j[MAXL], cell_beg[MAXL], cell_cnt[MAXL];
  int type_n1[MAXT], type_n2[MAXT];
  uint32_t cand[MAXCAND];
};

// kernel arguments (passed by value)
struct KArgs {
  const SceneDev* sc;
  float* dyn;          // [nb][6][B]
  uint32_t* keys;      // [B][2]
  uint32_t* err;       // [B]
  const float* geom;   // [G] or [B][gstride]
  int gstride, B, n_steps;
  float dt;
  int stages;
  const float* action;  // [n_steps][B][2] or null
  int action_body;
  const float* dyn_reset;  // [nb][6][B] or null
  uint32_t* resets;        // [B] or null
  int dbg_skip;            // debug only: bit k skips collider phase k (T=1,B=2,C=4,D=8)
};

struct Lay {
  int dyn, world, con, m, ch, key, sk0, skt, err, S;
};
CX_DEV Lay layout(const SceneDev& s) {
  Lay L;
  L.dyn = 0;
  L.world = L.dyn + s.nb * 6;
  L.con = L.world + s.W;
  L.m = L.con + s.nc * 4;
  L.ch = L.m + s.nb * s.nb;
  L.key = L.ch + s.nb;
  L.sk0 = L.key + 2;
  L.skt = L.sk0 + 2;
  L.err = L.skt + 2 * s.nt;
  L.S = L.err + 1;
  return L;
}
static inline int lds_words(const SceneDev& s) {
  return s.nb * 6 + s.W + s.nc * 4 + s.nb * s.nb + s.nb + 4 + 2 * s.nt + 1;
}

CX_DEV void lunar_constraints(cx::Dyn& lander, cx::Dyn& rleg, cx::Dyn& lleg, const cx::Params& pl,
                              const cx::Params& pr, const cx::Params& pll) {
  // LunarLander.step, cotix/_lunar_lander.py:145-218
  using namespace cx;
  const float f05 = 0.05f;
  v2 lp = v2{lander.px, lander.py};
  v2 llj1 = add(rotate(v2{24.0f * f05, -8.0f * f05}, lander.a), lp);
  v2 llj2 = add(rotate(v2{24.0f * f05, 0.0f * f05}, lander.a), lp);
  v2 lj1 = v2{lleg.px, lleg.py};
  v2 lj2 = add(v2{lleg.px, lleg.py}, rotate(v2{0.0f, 0.4f}, lleg.a));
  v2 lrj1 = add(rotate(v2{-24.0f * f05, -8.0f * f05}, lander.a), lp);
  v2 lrj2 = add(rotate(v2{-24.0f * f05, 0.0f * f05}, lander.a), lp);
  v2 rj1 = v2{rleg.px, rleg.py};
  v2 rj2 = add(v2{rleg.px, rleg.py}, rotate(v2{0.0f, 0.4f}, rleg.a));
  struct J {
    static CX_MF void fixed(Dyn& b1, const Params& m1, v2 c1, Dyn& b2, const Params& m2, v2 c2) {
      const float f05 = 0.05f;
      v2 dp = sub(c1, c2);
      v2 dv = sub(velocity_at(b1, c1), velocity_at(b2, c2));
      float k = nrm(dv) + 0.1f;
      v2 imp = v2{dp.x * 1.0f + (dv.x * k) * f05, dp.y * 1.0f + (dv.y * k) * f05};
      apply_impulse(b1, m1, neg(imp), c1);
      apply_impulse(b2, m2, imp, c2);
    }
  };
  J::fixed(lander, pl, llj1, lleg, pll, lj1);
  J::fixed(lander, pl, llj2, lleg, pll, lj2);
  J::fixed(lander, pl, lrj1, rleg, pr, rj1);
  J::fixed(lander, pl, lrj2, rleg, pr, rj2);
  rleg.w = rleg.w * 0.95f;
  lleg.w = lleg.w * 0.95f;
}

// contact-function sets compiled into a step kernel (scene feature mask)
enum : int { FNS_ANALYTIC = 1, FNS_CONVEX = 2, FNS_CIRCLE_POLY = 4 };
template <int FNSET>
CX_DEV cx::Contact run_contact_set(int fn, const cx::Shape& a, const cx::Shape& b, cx::v2 d0, uint32_t* err) {
  using namespace cx;
  if ((FNSET & FNS_ANALYTIC) != 0) {
    if (fn == FN_AABB_AABB) return aabb_vs_aabb(a, b);
    if (fn == FN_CIRCLE_AABB) return circle_vs_aabb(a, b, err);
    if (fn == FN_CIRCLE_CIRCLE) return circle_vs_circle(a, b);
  }
  if ((FNSET & FNS_CONVEX) != 0) {
    if (fn == FN_POLY_POLY || fn == FN_AABB_POLY) return convex_vs_polygon(a, b, d0);
  }
  if ((FNSET & FNS_CIRCLE_POLY) != 0) {
    if (fn == FN_CIRCLE_POLY) return circle_vs_polygon(a, b, d0);
  }
  return nan_contact();
}

// [word][env] LDS accessors
template <int E>
struct Tile {
  uint32_t* u;
  CX_MF float& f(int off, int e) const { return reinterpret_cast<float*>(u)[off * E + e]; }
  CX_MF uint32_t& w(int off, int e) const { return u[off * E + e]; }
};

template <int E>
CX_DEV void ph_load(const KArgs& a, const SceneDev& sc, const Lay& L, Tile<E> t, int env0, int tid) {
  for (int w = tid; w < sc.nb * 6 * E; w += BLK) {
    int e = w % E, off = w / E, g = env0 + e;
    t.f(L.dyn + off, e) = (g < a.B) ? a.dyn[(size_t)off * a.B + g] : 0.0f;
  }
  for (int e = tid; e < E; e += BLK) {
    int g = env0 + e;
    t.w(L.key, e) = (g < a.B) ? a.keys[2 * (size_t)g] : 0u;
    t.w(L.key + 1, e) = (g < a.B) ? a.keys[2 * (size_t)g + 1] : 0u;
    t.w(L.err, e) = (g < a.B) ? a.err[g] : 0u;
  }
}

// phase A: Euler (cotix/_physics_solvers.py:16-33) + driver extras + key chain
template <int E>
CX_DEV void ph_A(const KArgs& a, const SceneDev& sc, const Lay& L, Tile<E> t, int env0, int tid, int step) {
  using namespace cx;
  const int nb = sc.nb;
  if (a.stages & (COTIX_STAGE_EULER | COTIX_STAGE_GRAVITY)) {
    for (int w = tid; w < nb * E; w += BLK) {
      int e = w % E, b = w / E, g = env0 + e;
      if (g >= a.B) continue;
      const int o = L.dyn + b * 6;
      if (a.stages & COTIX_STAGE_EULER) {
        t.f(o + 0, e) = t.f(o + 0, e) + t.f(o + 2, e) * a.dt;
        t.f(o + 1, e) = t.f(o + 1, e) + t.f(o + 3, e) * a.dt;
        t.f(o + 4, e) = t.f(o + 4, e) + t.f(o + 5, e) * a.dt;
      }
      if ((a.stages & COTIX_STAGE_GRAVITY) && b == 0) {  // examples/test_viz.py:27-31
        t.f(o + 2, e) = t.f(o + 2, e) + 0.0f;
        t.f(o + 3, e) = t.f(o + 3, e) + -0.002f;
      }
      if (a.action != nullptr && b == a.action_body) {
        const float* ac = a.action + ((size_t)step * a.B + g) * 2;
        t.f(o + 2, e) = t.f(o + 2, e) + ac[0];
        t.f(o + 3, e) = t.f(o + 3, e) + ac[1];
      }
    }
  }
  if (a.stages & (COTIX_STAGE_COLLIDER | COTIX_STAGE_ADVANCE_KEY)) {
    for (int e = tid; e < E; e += BLK) {
      key2 k = key2{t.w(L.key, e), t.w(L.key + 1, e)};
      key2 s = split_at(k, 2u, 0u);  // cotix/_colliders.py:142 == next driver key
      t.w(L.sk0, e) = s.a;
      t.w(L.sk0 + 1, e) = s.b;
      for (int q = 0; q < sc.nt; ++q) {  // :175, one split per type key
        s = split_at(s, 2u, 0u);
        t.w(L.skt + 2 * q, e) = s.a;
        t.w(L.skt + 2 * q + 1, e) = s.b;
      }
      for (int q = 0; q < nb * nb; ++q) t.w(L.m + q, e) = 0xFFFFFFFFu;
      for (int q = 0; q < nb; ++q) t.w(L.ch + q, e) = (uint32_t)q;
    }
  }
}

// phase T: shape.transform(body transformer) (cotix/_colliders.py:92-94)
template <int E>
CX_DEV void ph_T(const KArgs& a, const SceneDev& sc, const Lay& L, Tile<E> t, int env0, int tid) {
  using namespace cx;
  for (int w = tid; w < sc.np * E; w += BLK) {
    int e = w % E, p = w / E, g = env0 + e;
    if (g >= a.B) continue;
    const int b = sc.part_body[p], kind = sc.part_kind[p], n = sc.part_n[p];
    const float* lg = a.geom + (a.gstride ? (size_t)g * a.gstride : (size_t)0) + sc.part_goff[p];
    const int o = L.dyn + b * 6, wo = L.world + sc.part_woff[p];
    const float px = t.f(o + 0, e), py = t.f(o + 1, e);
    if (kind != KIND_POLY) {
      // Circle (r, cx, cy, pad): translate only, cotix/_convex_shapes.py:37-41
      // AABB (lo.x, lo.y, up.x, up.y): translate only, :113-117
      // Branch-free on purpose: all four floats are loaded unconditionally
      // (a divergent circle/AABB tail was miscompiled by hipcc 7.2: the
      // circle lanes read an address register only the AABB lanes defined).
      const bool circ = kind == KIND_CIRCLE;
      const float g0 = lg[0], g1 = lg[1], g2 = lg[2], g3 = lg[3];
      t.f(wo + 0, e) = circ ? g0 : g0 + px;
      t.f(wo + 1, e) = circ ? g1 + px : g1 + py;
      t.f(wo + 2, e) = circ ? g2 + py : g2 + px;
      t.f(wo + 3, e) = circ ? g3 : g3 + py;
    } else {  // :181-187 forward_vector then re-sort (Polygon.__init__)
      float s, c;
      sincos32(t.f(o + 4, e), &s, &c);
      float xy[2 * MAXV];
      for (int k = 0; k < n; ++k) {
        float x = lg[2 * k], y = lg[2 * k + 1];
        float t0 = (c * x + (-s) * y) + px * 1.0f;
        float t1 = (s * x + c * y) + py * 1.0f;
        float t2 = (0.0f * x + 0.0f * y) + 1.0f * 1.0f;
        xy[2 * k] = t0 / t2;
        xy[2 * k + 1] = t1 / t2;
      }
      order_clockwise(xy, n);
      for (int k = 0; k < 2 * n; ++k) t.f(wo + k, e) = xy[k];
    }
  }
}

// phase B: distinct contacts (cotix/_colliders.py:149-173)
template <int E, int FNSET>
CX_DEV void ph_B(const KArgs& a, const SceneDev& sc, const Lay& L, Tile<E> t, int env0, int tid) {
  using namespace cx;
  const v2 d0 = v2{sc.d0x, sc.d0y};
  for (int w = tid; w < sc.nc * E; w += BLK) {
    int e = w % E, c = w / E, g = env0 + e;
    if (g >= a.B) continue;
    const int pa = sc.c_pa[c], pb = sc.c_pb[c];
    Shape A, Bs;
    A.kind = sc.part_kind[pa];
    A.n = sc.part_n[pa];
    Bs.kind = sc.part_kind[pb];
    Bs.n = sc.part_n[pb];
    const int na = A.kind == KIND_CIRCLE ? 3 : (A.kind == KIND_AABB ? 4 : 2 * A.n);
    const int nbf = Bs.kind == KIND_CIRCLE ? 3 : (Bs.kind == KIND_AABB ? 4 : 2 * Bs.n);
    for (int k = 0; k < na; ++k) A.d[k] = t.f(L.world + sc.part_woff[pa] + k, e);
    for (int k = 0; k < nbf; ++k) Bs.d[k] = t.f(L.world + sc.part_woff[pb] + k, e);
    uint32_t er = 0u;
    Contact ct = run_contact_set<FNSET>(sc.c_fn[c], A, Bs, d0, &er);
    const int co = L.con + 4 * c;
    t.f(co + 0, e) = ct.pen.x;
    t.f(co + 1, e) = ct.pen.y;
    t.f(co + 2, e) = ct.cp.x;
    t.f(co + 3, e) = ct.cp.y;
    if (er) {
#if defined(__HIP__) || defined(__HIPCC__)
      atomicOr(&t.w(L.err, e), er);
#else
      t.w(L.err, e) |= er;
#endif
    }
  }
}

// phase C: per cell, last passing candidate (cotix/_colliders.py:208-268)
template <int E>
CX_DEV void ph_C(const KArgs& a, const SceneDev& sc, const Lay& L, Tile<E> t, int env0, int tid) {
  using namespace cx;
  for (int w = tid; w < sc.nl * E; w += BLK) {
    int e = w % E, l = w / E, g = env0 + e;
    if (g >= a.B) continue;
    const int beg = sc.cell_beg[l], cnt = sc.cell_cnt[l];
    int res = -1, lt = -1, li2 = -1;
    key2 k2 = key2{0u, 0u};
    for (int q = 0; q < cnt; ++q) {
      const uint32_t cd = sc.cand[beg + q];
      const int i1 = cd & 511u, i2 = (cd >> 9) & 511u, cid = (cd >> 18) & 511u, ty = cd >> 27;
      const float cpx = t.f(L.con + 4 * cid + 2, e), cpy = t.f(L.con + 4 * cid + 3, e);
      if (isn(cpx) || isn(cpy)) continue;  // a NaN candidate never writes
      if (ty != lt || i2 != li2) {
        key2 sk = key2{t.w(L.skt + 2 * ty, e), t.w(L.skt + 2 * ty + 1, e)};
        k2 = split_at(sk, (uint32_t)sc.type_n2[ty], (uint32_t)i2);  // :264
        lt = ty;
        li2 = i2;
      }
      key2 k = split_at(k2, (uint32_t)sc.type_n1[ty], (uint32_t)i1);  // :254
      key2 k1 = split_at(k, 2u, 0u);                                   // :222
      if (bernoulli_half(k1)) {                                        // :223
        res = cid;
        break;
      }
    }
    t.w(L.m + sc.cell_i[l] * sc.nb + sc.cell_j[l], e) = (uint32_t)res;
  }
}

// phase D: choose_random_contact (cotix/_colliders.py:274-295)
template <int E>
CX_DEV void ph_D(const KArgs& a, const SceneDev& sc, const Lay& L, Tile<E> t, int env0, int tid) {
  using namespace cx;
  const int nb = sc.nb, nt = sc.nt;
  for (int w = tid; w < nb * E; w += BLK) {
    int e = w % E, i = w / E, g = env0 + e;
    if (g >= a.B) continue;
    int cnt = 0;
    for (int j = 0; j < nb; ++j) cnt += ((int)t.w(L.m + i * nb + j, e) >= 0) ? 1 : 0;
    int ch = i;
    if (cnt > 0) {
      float p[MAXB], c[MAXB];
      const float fc = (float)cnt;
      for (int j = 0; j < nb; ++j) p[j] = (((int)t.w(L.m + i * nb + j, e) >= 0) ? 1.0f : 0.0f) / fc;
      cumsum_assoc(p, nb, c);
      const int so = nt > 0 ? L.skt + 2 * (nt - 1) : L.sk0;
      key2 ck = split_at(key2{t.w(so, e), t.w(so + 1, e)}, (uint32_t)nb, (uint32_t)i);
      float u = unit_float(bits1(ck));
      float r = c[nb - 1] * (1.0f - u);
      ch = nb;
      for (int j = 0; j < nb; ++j)
        if (!(c[j] < r)) {
          ch = j;
          break;
        }
    }
    t.w(L.ch + i, e) = (uint32_t)ch;
  }
}

// phase E: sequential resolution (:310-336), joints, key update, restarts
template <int E>
CX_DEV void ph_E(const KArgs& a, const SceneDev& sc, const Lay& L, Tile<E> t, int env0, int tid) {
  using namespace cx;
  const int nb = sc.nb;
  for (int e = tid; e < E; e += BLK) {
    int g = env0 + e;
    if (g >= a.B) continue;
    if (a.stages & COTIX_STAGE_COLLIDER) {
      for (int i = 0; i < nb; ++i) {
        const int j = (int)t.w(L.ch + i, e);
        if (j == i || j < 0 || j >= nb) continue;
        const int cid = (int)t.w(L.m + i * nb + j, e);
        if (cid < 0) continue;
        const int co = L.con + 4 * cid, oi = L.dyn + 6 * i, oj = L.dyn + 6 * j;
        Dyn bi = Dyn{t.f(oi, e), t.f(oi + 1, e), t.f(oi + 2, e), t.f(oi + 3, e), t.f(oi + 4, e), t.f(oi + 5, e)};
        Dyn bj = Dyn{t.f(oj, e), t.f(oj + 1, e), t.f(oj + 2, e), t.f(oj + 3, e), t.f(oj + 4, e), t.f(oj + 5, e)};
        resolve_collision(bi, sc.par[i], bj, sc.par[j], v2{t.f(co, e), t.f(co + 1, e)},
                          v2{t.f(co + 2, e), t.f(co + 3, e)});
        t.f(oi + 2, e) = bi.vx;
        t.f(oi + 3, e) = bi.vy;
        t.f(oi + 5, e) = bi.w;
        t.f(oj + 2, e) = bj.vx;
        t.f(oj + 3, e) = bj.vy;
        t.f(oj + 5, e) = bj.w;
      }
    }
    if ((a.stages & COTIX_STAGE_LUNAR) && nb >= 3) {
      Dyn d[3];
      for (int b = 0; b < 3; ++b) {
        const int o = L.dyn + 6 * b;
        d[b] = Dyn{t.f(o, e), t.f(o + 1, e), t.f(o + 2, e), t.f(o + 3, e), t.f(o + 4, e), t.f(o + 5, e)};
      }
      lunar_constraints(d[0], d[1], d[2], sc.par[0], sc.par[1], sc.par[2]);
      for (int b = 0; b < 3; ++b) {
        const int o = L.dyn + 6 * b;
        t.f(o + 2, e) = d[b].vx;
        t.f(o + 3, e) = d[b].vy;
        t.f(o + 5, e) = d[b].w;
      }
    }
    if (a.stages & COTIX_STAGE_ADVANCE_KEY) {  // examples/test_viz.py:39,66
      t.w(L.key, e) = t.w(L.sk0, e);
      t.w(L.key + 1, e) = t.w(L.sk0 + 1, e);
    }
    if (a.dyn_reset != nullptr && t.w(L.err, e) != 0u) {
      // episode end on an error_if trip (the reference raises here): restart
      // the env from its reset state; the key chain continues.
      for (int off = 0; off < nb * 6; ++off) t.f(L.dyn + off, e) = a.dyn_reset[(size_t)off * a.B + g];
      t.w(L.err, e) = 0u;
      if (a.resets) a.resets[g] += 1u;
    }
  }
}

template <int E>
CX_DEV void ph_store(const KArgs& a, const SceneDev& sc, const Lay& L, Tile<E> t, int env0, int tid) {
  for (int w = tid; w < sc.nb * 6 * E; w += BLK) {
    int e = w % E, off = w / E, g = env0 + e;
    if (g < a.B) a.dyn[(size_t)off * a.B + g] = t.f(L.dyn + off, e);
  }
  for (int e = tid; e < E; e += BLK) {
    int g = env0 + e;
    if (g < a.B) {
      a.keys[2 * (size_t)g] = t.w(L.key, e);
      a.keys[2 * (size_t)g + 1] = t.w(L.key + 1, e);
      a.err[g] = t.w(L.err, e);
    }
  }
}

}  // namespace cxk
