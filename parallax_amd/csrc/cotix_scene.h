// cotix_scene.h -- host-side scene compiler: the collider's trace-time work
// (cotix/_colliders.py:86-131) done once per scene.  Host C++ only; shared by
// the library (cotix_step.hip) and the CPU emulation harness (tests/emu).
#pragma once
#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "cotix_kernel.h"

namespace cxk {

// the exact reciprocal of a mass / inertia (cx::Rcp): r with x / d == x * r
// for every x, or NaN when no such r exists
inline float exact_rcp(float d) {
  if (std::isinf(d)) return std::signbit(d) ? -0.0f : 0.0f;
  if (d == 0.0f) return std::signbit(d) ? -INFINITY : INFINITY;
  if (std::isnan(d) || !std::isnormal(d)) return NAN;
  int ex;
  const float m = std::frexp(d, &ex);
  if (std::fabs(m) != 0.5f) return NAN;  // not a power of two
  const float r = 1.0f / d;
  return std::isnormal(r) ? r : NAN;
}

inline int scene_fail(std::string& err, const std::string& m) {
  err = m;
  return -1;
}

inline int registry_fn(int ta, int tb) {
  // _contact_funcs keys (cotix/_colliders.py:21-35), exact types
  using namespace cx;
  if (ta == COTIX_AABB && tb == COTIX_AABB) return FN_AABB_AABB;
  if (ta == COTIX_CIRCLE && tb == COTIX_CIRCLE) return FN_CIRCLE_CIRCLE;
  if (ta == COTIX_CIRCLE && tb == COTIX_AABB) return FN_CIRCLE_AABB;
  if (ta == COTIX_POLYGON && tb == COTIX_POLYGON) return FN_POLY_POLY;
  if (ta == COTIX_AABB && (tb == COTIX_POLYGON || tb == COTIX_POLYGON4 || tb == COTIX_POLYGON6)) return FN_AABB_POLY;
  if (ta == COTIX_CIRCLE && (tb == COTIX_POLYGON || tb == COTIX_POLYGON4 || tb == COTIX_POLYGON6))
    return FN_CIRCLE_POLY;
  if (ta == COTIX_POLYGON4 && (tb == COTIX_POLYGON4 || tb == COTIX_POLYGON6)) return FN_POLY_POLY;
  if (ta == COTIX_POLYGON6 && tb == COTIX_POLYGON6) return FN_POLY_POLY;
  return -1;
}


// the reference's literals (include/cotix_amd.h cotix_params)
inline cotix_params default_params() {
  cotix_params p;
  p.prng_layout = COTIX_PRNG_LEGACY;
  p.baumgarte = 0.3f;      // cotix/_collision_resolution.py:105
  p.baumgarte_dt = 0.01f;  // :115
  p.contact_p = 0.5f;      // cotix/_colliders.py:220
  p.gjk_max_steps = 32;    // cotix/_collisions.py:101
  p.epa_max_iters = 48;    // cotix/_contacts.py:271,295
  p.epa_circle_iters = 128;  // cotix/_contacts.py:162-163
  p.epa_body_iters = 48;   // cotix/_universal_shape.py:120
  return p;
}
inline int check_params(const cotix_params& p, std::string& err) {
  if (p.prng_layout != COTIX_PRNG_LEGACY && p.prng_layout != COTIX_PRNG_PARTITIONABLE)
    return scene_fail(err, "prng_layout must be COTIX_PRNG_LEGACY or COTIX_PRNG_PARTITIONABLE");
  if (p.gjk_max_steps < 0 || p.gjk_max_steps > 4096) return scene_fail(err, "gjk_max_steps outside 0..4096");
  // the reference's error_if rejects fewer than 3 EPA iterations (cotix/_collisions.py:130-135)
  if (p.epa_max_iters < 3 || p.epa_max_iters > 65535) return scene_fail(err, "epa_max_iters outside 3..65535");
  if (p.epa_circle_iters < 3 || p.epa_circle_iters > 128) return scene_fail(err, "epa_circle_iters outside 3..128");
  if (p.epa_body_iters < 3 || p.epa_body_iters > 128) return scene_fail(err, "epa_body_iters outside 3..128");
  return 0;
}
// the scene header's parameter fields
inline void set_params(SceneHdr& s, const cotix_params& p) {
  s.prng = (uint16_t)p.prng_layout;
  const cx::v2 d0 = cx::gjk_d0(p.prng_layout == COTIX_PRNG_PARTITIONABLE);  // random_direction(PRNGKey(1))
  s.d0x = d0.x;
  s.d0y = d0.y;
  s.gjk_steps = (uint16_t)p.gjk_max_steps;
  s.epa_cap = (uint16_t)p.epa_max_iters;
  s.epa_cp = (uint16_t)p.epa_circle_iters;
  s.epa_body = (uint16_t)p.epa_body_iters;
  s.baum = p.baumgarte;
  s.baum_dt = p.baumgarte_dt;
  s.pc = p.contact_p;
}
inline cotix_params params_of(const SceneHdr& s) {
  cotix_params p;
  p.prng_layout = s.prng;
  p.baumgarte = s.baum;
  p.baumgarte_dt = s.baum_dt;
  p.contact_p = s.pc;
  p.gjk_max_steps = s.gjk_steps;
  p.epa_max_iters = s.epa_cap;
  p.epa_circle_iters = s.epa_cp;
  p.epa_body_iters = s.epa_body;
  return p;
}

// Compiles the body/part description into SceneDev tables.  Returns 0 or -1
// (message in err).  n_cand / fnset: candidate count and contact-function set.
// prm: cotix_params (nullable: the reference's literals).
inline int compile_scene(int n_bodies, const float* body_params, int n_parts, const int* part_body,
                         const int* part_type, const int* part_nverts, SceneDev& s, int& n_cand, int& fnset,
                         std::string& err, const cotix_params* prm = nullptr, int flags = 0) {
  const cotix_params par = prm ? *prm : default_params();
  if (check_params(par, err)) return -1;
  if (!body_params || !part_body || !part_type) return scene_fail(err, "null argument");

  if (n_bodies < 1 || n_bodies > MAXB) return scene_fail(err, "n_bodies out of range (1..16)");
  if (n_parts < 1 || n_parts > MAXP) return scene_fail(err, "n_parts out of range (1..32)");
  std::memset(&s, 0, sizeof(s));
  s.nb = n_bodies;
  s.np = n_parts;
  set_params(s, par);  // incl. the GJK start direction (cotix/_collisions.py:287-298)
  std::vector<int> part_bodyv(n_parts), part_kindv(n_parts), part_nv(n_parts), part_goffv(n_parts),
      part_woffv(n_parts);
  std::vector<std::vector<int>> parts_of(n_bodies);
  int goff = 0, woff = 0;
  for (int p = 0; p < n_parts; ++p) {
    int b = part_body[p], t = part_type[p];
    if (b < 0 || b >= n_bodies) return scene_fail(err, "part_body out of range");
    if (p > 0 && b < part_body[p - 1]) return scene_fail(err, "parts must be grouped by body in body order");
    part_bodyv[p] = b;
    if (t == COTIX_CIRCLE) {
      part_kindv[p] = cx::KIND_CIRCLE;
      part_nv[p] = 0;
    } else if (t == COTIX_AABB) {
      part_kindv[p] = cx::KIND_AABB;
      part_nv[p] = 0;
    } else if (t >= COTIX_POLYGON && t <= COTIX_POLYGON6) {
      int n = (t == COTIX_POLYGON) ? (part_nverts ? part_nverts[p] : 0) : t;
      if (n < 3 || n > cx::MAXV) return scene_fail(err, "polygon vertex count must be 3..8");
      part_kindv[p] = cx::KIND_POLY;
      part_nv[p] = n;
    } else {
      return scene_fail(err, "unknown part type");
    }
    int nf = part_kindv[p] == cx::KIND_CIRCLE ? 4 : (part_kindv[p] == cx::KIND_AABB ? 4 : 2 * part_nv[p]);
    part_goffv[p] = goff;
    part_woffv[p] = woff;
    goff += nf;
    woff += nf;
    parts_of[b].push_back(p);
  }
  s.G = goff;
  s.W = woff;
  if (flags & ~COTIX_SCENE_PER_ENV_BODY_PARAMS) return scene_fail(err, "unknown scene flags");
  if (flags & COTIX_SCENE_PER_ENV_BODY_PARAMS) {  // each env's 4 words per body after its part geometry
    s.epar = (uint16_t)(goff + 1);
    s.G = goff + 4 * n_bodies;
  }
  // enumeration, cotix/_colliders.py:86-113 (dict insertion order of type keys)
  std::vector<std::pair<int, int>> tkeys;
  std::vector<std::vector<std::pair<int, int>>> l1, l2;  // (body, part)
  for (int i = 0; i < n_bodies; ++i)
    for (int j = 0; j < n_bodies; ++j) {
      if (i <= j) continue;
      for (int pa : parts_of[i])
        for (int pb : parts_of[j]) {
          int t1 = part_type[pa], t2 = part_type[pb];
          std::pair<int, int> key;
          if (registry_fn(t1, t2) >= 0) key = {t1, t2};
          else if (registry_fn(t2, t1) >= 0) key = {t2, t1};
          else return scene_fail(err, "illegal shape pair (cotix/_colliders.py:103-107)");
          int k = -1;
          for (size_t q = 0; q < tkeys.size(); ++q)
            if (tkeys[q] == key) k = (int)q;
          if (k < 0) {
            k = (int)tkeys.size();
            tkeys.push_back(key);
            l1.emplace_back();
            l2.emplace_back();
          }
          l1[k].push_back({i, pa});
          l2[k].push_back({j, pb});
        }
    }
  if ((int)tkeys.size() > MAXT) return scene_fail(err, "too many type keys");
  s.nt = (int)tkeys.size();
  std::map<std::tuple<int, int, int>, int> cid_of;
  std::map<std::pair<int, int>, std::vector<uint32_t>> cells;  // forward scan order
  std::vector<std::pair<int, int>> cell_order;
  auto get_cid = [&](int a, int b, int fn) -> int {
    auto key = std::make_tuple(a, b, fn);
    auto it = cid_of.find(key);
    if (it != cid_of.end()) return it->second;
    int c = (int)cid_of.size();
    cid_of[key] = c;
    return c;
  };
  std::vector<std::tuple<int, int, int>> clist;
  std::vector<int> tn1(s.nt), tn2(s.nt);
  for (int k = 0; k < s.nt; ++k) {
    int N1 = (int)l1[k].size(), N2 = (int)l2[k].size();
    if (N1 > 511 || N2 > 511) return scene_fail(err, "candidate list longer than 511");
    tn1[k] = N1;
    tn2[k] = N2;
    int fn = registry_fn(tkeys[k].first, tkeys[k].second);
    for (int i2 = 0; i2 < N2; ++i2)
      for (int i1 = 0; i1 < N1; ++i1) {
        int bi = l1[k][i1].first, pa = l1[k][i1].second, bj = l2[k][i2].first, pb = l2[k][i2].second;
        int a = pa, b = pb;
        if (registry_fn(part_type[pa], part_type[pb]) < 0) std::swap(a, b);  // :155-157
        bool cand = bi >= bj;
        if (!cand && fn != cx::FN_CIRCLE_AABB) continue;  // masked & side-effect free
        size_t before = cid_of.size();
        int c = get_cid(a, b, fn);
        if (cid_of.size() != before) clist.push_back(std::make_tuple(a, b, fn));
        if (!cand) continue;
        auto ck = std::make_pair(bi, bj);
        if (!cells.count(ck)) cell_order.push_back(ck);
        cells[ck].push_back((uint32_t)i1 | ((uint32_t)i2 << 9) | ((uint32_t)c << 18) | ((uint32_t)k << 27));
      }
  }
  if ((int)clist.size() > MAXC || (int)clist.size() > 511) return scene_fail(err, "too many distinct contacts");
  s.nc = (int)clist.size();
  if ((int)cells.size() > MAXL) return scene_fail(err, "too many cells");
  s.nl = (int)cells.size();
  // pack the hot tables (word offsets into s.hot, copied to LDS per launch)
  std::vector<uint32_t> hot;
  auto put = [&](uint16_t& off, const std::vector<int>& v) {
    off = (uint16_t)hot.size();
    for (int x : v) hot.push_back((uint32_t)x);
  };
  {
    s.o_par = (int)hot.size();
    for (int q = 0; q < 4 * n_bodies; ++q) {
      uint32_t u;
      std::memcpy(&u, &body_params[q], 4);
      hot.push_back(u);
    }
  }
  {
    s.o_rcp = (int)hot.size();  // exact reciprocals of mass and inertia (cx::Rcp)
    s.rcp_all = 1;
    s.rcp_mask = 0;
    for (int b = 0; b < n_bodies; ++b) s.rcp_mask |= (b < 32 ? 1 << b : 0);
    for (int b = 0; b < n_bodies; ++b)
      for (int q = 0; q < 2; ++q) {
        const float r = exact_rcp(body_params[4 * b + q]);
        if (std::isnan(r)) {
          s.rcp_all = 0;
          if (b < 32) s.rcp_mask &= ~(1 << b);
        }
        uint32_t u;
        std::memcpy(&u, &r, 4);
        hot.push_back(u);
      }
  }
  if (s.epar != 0) {  // the table's reciprocals hold for the template values only: IEEE divisions
    s.rcp_all = 0;
    s.rcp_mask = 0;
  }
  put(s.o_pbody, part_bodyv);
  put(s.o_pkind, part_kindv);
  put(s.o_pn, part_nv);
  put(s.o_pgoff, part_goffv);
  put(s.o_pwoff, part_woffv);
  {  // phase T's polygon vertex items, part order (cxk::ph_TV*)
    // 2 words per vertex (one 8-byte read): part | vertex << 5 | count << 8 |
    // first item of the part << 12 | body << 21, then the vertex's local
    // geometry offset | the part's world offset << 16
    if (hot.size() % 2) hot.push_back(0u);
    s.o_vit = (uint16_t)hot.size();
    int nv = 0;
    for (int p = 0; p < n_parts; ++p) {
      const int first = nv;
      for (int k = 0; k < part_nv[p]; ++k, ++nv) {
        hot.push_back((uint32_t)(p | (k << 5) | (part_nv[p] << 8) | (first << 12) | (part_bodyv[p] << 21)));
        hot.push_back((uint32_t)(part_goffv[p] + 2 * k) | ((uint32_t)part_woffv[p] << 16));
      }
    }
    s.nvt = nv;
    int mv = 0;
    for (int p = 0; p < n_parts; ++p) mv = part_nv[p] > mv ? part_nv[p] : mv;
    s.maxv = (uint16_t)mv;
  }
  std::vector<int> cpa(s.nc), cpb(s.nc), cfn(s.nc);
  for (int c = 0; c < s.nc; ++c) {
    cpa[c] = std::get<0>(clist[c]);
    cpb[c] = std::get<1>(clist[c]);
    cfn[c] = std::get<2>(clist[c]);
  }
  put(s.o_cpa, cpa);
  put(s.o_cpb, cpb);
  put(s.o_cfn, cfn);
  // per contact: world offsets, fn and kinds of both parts in one 2-word descriptor
  if (hot.size() % 2) hot.push_back(0u);  // 8-byte aligned (one ds_read_b64)
  s.o_cdesc = (int)hot.size();
  for (int c = 0; c < s.nc; ++c) {
    const int pa = cpa[c], pb = cpb[c];
    if (part_woffv[pa] > 1023 || part_woffv[pb] > 1023) return scene_fail(err, "world table too large");
    hot.push_back((uint32_t)part_woffv[pa] | ((uint32_t)part_woffv[pb] << 10) | ((uint32_t)cfn[c] << 20) |
                  ((uint32_t)part_kindv[pa] << 23) | ((uint32_t)part_kindv[pb] << 25) |
                  ((uint32_t)(pa == pb) << 27));  // a part paired with itself: penetration never used
    hot.push_back((uint32_t)part_nv[pa] | ((uint32_t)part_nv[pb] << 8) | ((uint32_t)pa << 16) | ((uint32_t)pb << 24));
  }
  {  // per contact the bodies of its two parts (phase AB of the analytic programs)
    std::vector<int> cb(s.nc);
    for (int c = 0; c < s.nc; ++c) cb[c] = part_bodyv[cpa[c]] | (part_bodyv[cpb[c]] << 8);
    put(s.o_cbody, cb);
  }
  s.nmw = (s.nc + 31) / 32;
  std::vector<int> ci, cj, cbeg, ccnt;
  std::vector<uint32_t> cmask;
  std::vector<int> candv;
  for (auto& ck : cell_order) {
    auto& v = cells[ck];
    ci.push_back(ck.first);
    cj.push_back(ck.second);
    cbeg.push_back((int)candv.size());
    ccnt.push_back((int)v.size());
    // types ascend, then (ind2, ind1) ascend in v: reverse = last write first
    for (int q = (int)v.size() - 1; q >= 0; --q) candv.push_back((int)v[q]);
    std::vector<uint32_t> m(s.nmw, 0u);  // the cell's distinct contacts
    for (uint32_t cd : v) {
      int c = (int)((cd >> 18) & 511u);
      m[c >> 5] |= 1u << (c & 31);
    }
    cmask.insert(cmask.end(), m.begin(), m.end());
  }
  if ((int)candv.size() > MAXCAND) return scene_fail(err, "too many candidates");
  put(s.o_ci, ci);
  put(s.o_cj, cj);
  put(s.o_cbeg, cbeg);
  put(s.o_ccnt, ccnt);
  put(s.o_tn1, tn1);
  put(s.o_tn2, tn2);
  put(s.o_cand, candv);
  s.o_cmask = (int)hot.size();
  for (uint32_t x : cmask) hot.push_back(x);
  if ((int)hot.size() > MAXHOT) return scene_fail(err, "scene tables too large");
  s.nhot = (int)hot.size();
  for (size_t q = 0; q < hot.size(); ++q) s.hot[q] = hot[q];
  s.ncand = (int)candv.size();
  int nc_tot = s.ncand;
  n_cand = nc_tot;
  fnset = 0;
  s.poly = 0;
  for (int c = 0; c < s.nc; ++c) s.poly |= (cfn[c] == cx::FN_POLY_POLY || cfn[c] == cx::FN_AABB_POLY) ? 1 : 0;
  s.pminv = 0;  // the broadphase guard's outer loop bound: max over polygon pairs of the smaller edge count
  for (int c = 0; c < s.nc; ++c)
    if (cfn[c] == cx::FN_POLY_POLY || cfn[c] == cx::FN_AABB_POLY) {
      const int ea = part_kindv[cpa[c]] == cx::KIND_POLY ? part_nv[cpa[c]] : 2;
      const int eb = part_kindv[cpb[c]] == cx::KIND_POLY ? part_nv[cpb[c]] : 2;
      const int m = ea < eb ? ea : eb;
      s.pminv = (uint16_t)(m > s.pminv ? m : s.pminv);
    }
  for (int c = 0; c < s.nc; ++c) {
    int fn = cfn[c];
    fnset |= (fn == cx::FN_AABB_AABB || fn == cx::FN_CIRCLE_AABB || fn == cx::FN_CIRCLE_CIRCLE) ? FNS_ANALYTIC
             : fn == cx::FN_CIRCLE_POLY                                                        ? FNS_CIRCLE_POLY
             : fn == cx::FN_AABB_POLY                                                          ? FNS_CONVEX | FNS_AABB_POLY
                                                                                               : FNS_CONVEX;
  }
  s.fnset = fnset;
  return 0;
}

// cotix_eval's judge / control (include/cotix_amd.h) -> the kernel's compact
// arguments: the nonzero weights as (word, w) terms in word order.  nw = the
// scene's state words (n_bodies * 6).
inline int pack_judge(const cotix_judge* j, int nw, int nb, JudgeArgs& out, std::string& err) {
  out = JudgeArgs{};
  if (j == nullptr) return 0;
  out.on = 1;
  for (int k = 0; k < COTIX_MAX_STATE_WORDS; ++k) {
    if (j->rate_w[k] != 0.0f || j->end_w[k] != 0.0f) {
      if (k >= nw) return scene_fail(err, "judge weight on a state word beyond the scene's bodies");
      if (std::isnan(j->rate_w[k]) || std::isnan(j->end_w[k])) return scene_fail(err, "NaN judge weight");
    }
    if (j->rate_w[k] != 0.0f) {
      if (out.nrate == JT) return scene_fail(err, "more than 16 nonzero judge rate weights");
      out.rate_k[out.nrate] = (uint8_t)k;
      out.rate_w[out.nrate++] = j->rate_w[k];
    }
    if (j->end_w[k] != 0.0f) {
      if (out.nend == JT) return scene_fail(err, "more than 16 nonzero judge end-reward weights");
      out.end_k[out.nend] = (uint8_t)k;
      out.end_w[out.nend++] = j->end_w[k];
    }
  }
  if (j->n_regions < 0 || j->n_regions > JR) return scene_fail(err, "judge n_regions outside [0, 4]");
  out.nreg = j->n_regions;
  for (int r = 0; r < out.nreg; ++r) {
    if (j->region_body[r] < 0 || j->region_body[r] >= nb) return scene_fail(err, "judge region body out of range");
    out.rbody[r] = j->region_body[r];
    for (int q = 0; q < 6; ++q) {
      out.lo[r][q] = j->region_lo[r][q];
      out.hi[r][q] = j->region_hi[r][q];
    }
    out.rrew[r] = j->region_reward[r];
  }
  // the rate's pieces over the rate regions (piecewise-linear reward rate)
  if (j->n_rate_regions < 0 || j->n_rate_regions > JR) return scene_fail(err, "judge n_rate_regions outside [0, 4]");
  out.nrr = j->n_rate_regions;
  for (int r = 0; r < JR; ++r) {
    const bool live = r < out.nrr;
    if (live) {
      if (j->rate_region_body[r] < 0 || j->rate_region_body[r] >= nb)
        return scene_fail(err, "judge rate region body out of range");
      out.prbody[r] = j->rate_region_body[r];
      for (int q = 0; q < 6; ++q) {
        out.prlo[r][q] = j->rate_region_lo[r][q];
        out.prhi[r][q] = j->rate_region_hi[r][q];
      }
    }
    for (int k = 0; k < COTIX_MAX_STATE_WORDS; ++k) {
      const float w = j->rate_region_w[r][k];
      if (w == 0.0f) continue;
      if (!live) return scene_fail(err, "judge rate piece for a rate region past n_rate_regions");
      if (k >= nw) return scene_fail(err, "judge rate piece on a state word beyond the scene's bodies");
      if (std::isnan(w)) return scene_fail(err, "NaN judge rate piece weight");
      if (out.npr[r] == JRT) return scene_fail(err, "more than 8 nonzero weights in a rate piece");
      out.pr_k[r][out.npr[r]] = (uint8_t)k;
      out.pr_w[r][out.npr[r]++] = w;
    }
    if (j->rate_region_bias[r] != 0.0f) {
      if (!live) return scene_fail(err, "judge rate piece for a rate region past n_rate_regions");
      out.hasb[r] = 1;
      out.pr_b[r] = j->rate_region_bias[r];
    }
  }
  if (j->done_on_error != 0 && j->done_on_error != 1) return scene_fail(err, "judge done_on_error must be 0 or 1 (zero-initialise the struct)");
  out.doe = j->done_on_error;
  return 0;
}
inline int pack_control(const cotix_control* ct, int nb, CtlArgs& out, std::string& err) {
  out = CtlArgs{};
  if (ct == nullptr) return 0;
  if (ct->body < 0 || ct->body >= nb) return scene_fail(err, "control body out of range");
  out.on = 1;
  out.body = ct->body;
  for (int i = 0; i < 2; ++i) {
    for (int q = 0; q < 6; ++q) {
      out.gain[i][q] = ct->gain[i][q];
      out.target[i][q] = ct->target[i][q];
    }
    out.bias[i] = ct->bias[i];
    out.lo[i] = ct->clip_lo[i];
    out.hi[i] = ct->clip_hi[i];
  }
  // a caller that did not zero-initialise the struct (include/cotix_amd.h)
  // gets an error here rather than a silent clip to garbage bounds
  if (ct->saturate != 0 && ct->saturate != 1) return scene_fail(err, "control saturate must be 0 or 1 (zero-initialise the struct)");
  out.sat = ct->saturate;
  if (out.sat && (std::isnan(out.lo[0]) || std::isnan(out.lo[1]) || std::isnan(out.hi[0]) || std::isnan(out.hi[1])))
    return scene_fail(err, "NaN control clip bound");
  return 0;
}

}  // namespace cxk
