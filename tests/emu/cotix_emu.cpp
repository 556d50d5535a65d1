// TEST INFRASTRUCTURE ONLY -- host emulation of the fused HIP step kernel.
//
// Compiles parallax_amd/csrc/cotix_kernel.h (the kernel's phase functions and
// wave programs) for the host and runs each wave's program on 64 lanes as
// SIMT fibers (cotix_simt.h): the GPU's own code path, its cross-lane
// operations (ballots, permutes, pair exchanges) and phase barriers resolved
// as collective points.  Used to (a) check the kernel logic against the
// oracle on CPU and (b) run it under AddressSanitizer/UBSan (GPU sanitizers
// are unavailable).
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../parallax_amd/csrc/cotix_body.h"
#include "../../parallax_amd/csrc/cotix_kernel.h"
#include "../../parallax_amd/csrc/cotix_scene.h"
#include "cotix_simt.h"

namespace {
std::string g_err;
bool g_split_bwd = false;
bool g_key_helper = false;
struct EmuScene {
  cxk::SceneDev s;
  int n_cand = 0, fnset = 0;
};

// the lane's phase runner: the GPU's WaveRun (cotix_step_kernel.hip) -- an
// order point (every lane's wave-uniform reads between phases precede every
// lane's next phase), the phase on this lane, then the wave barrier; staged
// phases keep their state in the lane's own frame and order their stages by
// lockstep points
struct HostRun {
  int lane;
  template <class F>
  void operator()(int, F f) const {
    cxk::lockstep();
    f(lane);
    cxk::wave_sync();
  }
  template <class S, class F1, class F2, class F3>
  void staged(int ph, F1 fetch, F2 mid, F3 finish) const {
    (*this)(ph, [&](int l) {
      S s;
      fetch(l, s);
      cxk::lockstep();
      mid(l);
      cxk::lockstep();
      finish(l, s);
    });
  }
};

// the step wave's side of the key helper on the host: the helper's next
// window is computed at the step wave's barrier (cxk::KeyHelper)
template <int EW>
struct HostKeyHelp {
  static constexpr bool on = true;
  int kwalt;
  cxk::KeyHelper<EW>* h;
  const cxk::KArgs* a;
  const cxk::Ctx* c;
  const HostRun* run;
  bool* init;
  void bar() const {
    if (!*init) cxk::key_helper_init<EW>(*a, *c, *h, *run);
    *init = true;
    cxk::key_helper_next<EW>(*a, *c, *h, *run);
  }
};

// one wave at a time (waves are independent), through the kernel's own
// wave programs (cxk::run_wave / run_wave_backward) on 64 fiber lanes
template <int EW>
void run_blocks(const cxk::KArgs& a, int mode) {
  const cxk::SceneDev& sc = *a.sc;
  const cxk::Ctx c = cxk::make_ctx<EW>(sc);
  const int nwaves = (a.B + EW - 1) / EW;
  // the wave's tile and scratch (a multiple of EW words), then the split
  // backward's second tile (mode 5) or the key helper's window buffer (mode 6)
  const int rw = cxk::help_region_words<EW>(c), x2 = std::max(c.L.S * EW, cxk::KWIN * c.L.kww * EW);
  std::vector<uint32_t> lds((size_t)sc.nhot + (size_t)rw + (size_t)x2);
  for (int q = 0; q < sc.nhot; ++q) lds[q] = sc.hot[q];
  for (int wv = 0; wv < nwaves; ++wv) {
    std::fill(lds.begin() + sc.nhot, lds.end(), 0x7FBADBADu);  // poison (a NaN pattern)
    const cxk::Tile<EW> t{lds.data() + sc.nhot, lds.data(), lds.data() + sc.nhot + (size_t)c.L.S * EW};
    uint32_t* const x2b = lds.data() + sc.nhot + rw;
    const cxk::Tile<EW> t1{x2b, lds.data(), t.ws};
    // the kernel instantiation the library launches (cxk::launch_fnset)
    const int F = cxk::launch_fnset(sc.fnset, mode == 5 ? 4 : mode == 6 ? 0 : mode);
    const int env0 = wv * EW;
    cxk_simt::run([&](int lane) {
      const HostRun run{lane};
      if (mode == 6) {  // the step with a key helper: its window computed at the step wave's barrier
        cxk::KeyHelper<EW> kh;
        kh.tm = t;
        kh.th = cxk::Tile<EW>{x2b - c.L.kw * EW, lds.data(), nullptr};
        kh.env0 = env0;
        bool init = false;
        const HostKeyHelp<EW> help{(int)(x2b - t.u) / EW - c.L.kw, &kh, &a, &c, &run, &init};
        cxk::run_wave<EW, 1, false, false, false>(a, c, t, env0, run, false, help);
      } else if (mode == 5)  // the split tape backward: each step's producer part, then its consumer's
        c.nb == 5 ? cxk::run_backward_split<EW, 5>(a, c, t, t1, env0, run, 3, [] {})
                  : cxk::run_backward_split<EW, 7>(a, c, t, t1, env0, run, 3, [] {});
      else if (mode == 4)
        F == 1 ? cxk::run_wave_backward_tape<EW, 1>(a, c, t, env0, run)
               : cxk::run_wave_backward_tape<EW, 15>(a, c, t, env0, run);
      else if (mode == 2)
        F == 1 ? cxk::run_wave_backward<EW, 1>(a, c, t, env0, run) : cxk::run_wave_backward<EW, 15>(a, c, t, env0, run);
      else if (mode == 1)
        F == 1 ? cxk::run_wave<EW, 1, true>(a, c, t, env0, run) : cxk::run_wave<EW, 15, true>(a, c, t, env0, run);
      else if (mode == 3)
        F == 1 ? cxk::run_wave<EW, 1, false, true>(a, c, t, env0, run)
               : cxk::run_wave<EW, 15, false, true>(a, c, t, env0, run);
      else if (F == 1)
        cxk::run_wave<EW, 1, false>(a, c, t, env0, run);
      else if (F == 3)
        cxk::run_wave<EW, 3, false>(a, c, t, env0, run);
      else if (F == 11)
        cxk::run_wave<EW, 11, false>(a, c, t, env0, run);
      else
        cxk::run_wave<EW, 15, false>(a, c, t, env0, run);
    });
  }
}
void run_any(const cxk::KArgs& a, int E, int mode) {
  // the GPU's key helper (cotix_step.hip launch) where it applies and is asked for
  if (mode == 0 && g_key_helper && E == 4 && a.n_steps > cxk::KWIN &&
      cxk::launch_fnset(a.sc->fnset, 0) == cxk::FNS_ANALYTIC)
    mode = 6;
  if (E == 1) run_blocks<1>(a, mode);
  else if (E == 4) run_blocks<4>(a, mode);
  else if (E == 8) run_blocks<8>(a, mode);
  else run_blocks<2>(a, mode);
}
}  // namespace

extern "C" {
const char* emu_last_error(void) { return g_err.c_str(); }

int emu_scene_create_ex2(int n_bodies, const float* body_params, int n_parts, const int* part_body,
                         const int* part_type, const int* part_nverts, const cotix_params* params, int flags,
                         void** out) {
  EmuScene* s = new EmuScene();
  if (cxk::compile_scene(n_bodies, body_params, n_parts, part_body, part_type, part_nverts, s->s, s->n_cand,
                         s->fnset, g_err, params, flags)) {
    delete s;
    return -1;
  }
  *out = s;
  return 0;
}
int emu_scene_create_ex(int n_bodies, const float* body_params, int n_parts, const int* part_body,
                        const int* part_type, const int* part_nverts, const cotix_params* params, void** out) {
  return emu_scene_create_ex2(n_bodies, body_params, n_parts, part_body, part_type, part_nverts, params, 0, out);
}
int emu_scene_create(int n_bodies, const float* body_params, int n_parts, const int* part_body, const int* part_type,
                     const int* part_nverts, void** out) {
  return emu_scene_create_ex(n_bodies, body_params, n_parts, part_body, part_type, part_nverts, nullptr, out);
}

int emu_scene_destroy(void* s) {
  delete static_cast<EmuScene*>(s);
  return 0;
}

int emu_step(void* scene, float* dyn, uint32_t* keys, uint32_t* err, const float* geom, int gstride, int B,
             int n_steps, float dt, int stages, const float* action, int action_body, const float* dyn_reset,
             uint32_t* resets, int E) {
  EmuScene* s = static_cast<EmuScene*>(scene);
  cxk::KArgs a{};
  a.sc = &s->s;
  a.dyn = dyn;
  a.keys = keys;
  a.err = err;
  a.geom = geom;
  a.gstride = gstride;
  a.B = B;
  a.n_steps = n_steps;
  a.dt = dt;
  a.stages = stages;
  a.action = action;
  a.action_body = action_body;
  a.dyn_reset = dyn_reset;
  a.reset_mode = dyn_reset ? 1 : 0;
  a.resets = resets;
  run_any(a, E, 0);
  return 0;
}

int emu_step_ex(void* scene, float* dyn, uint32_t* keys, uint32_t* err, const float* geom, int gstride, int B,
                int n_steps, float dt, int stages, const float* action, int action_body, const float* dyn_reset,
                uint32_t* resets, int32_t* chosen, int32_t* cells, int E) {
  EmuScene* s = static_cast<EmuScene*>(scene);
  cxk::KArgs a{};
  a.sc = &s->s;
  a.dyn = dyn;
  a.keys = keys;
  a.err = err;
  a.geom = geom;
  a.gstride = gstride;
  a.B = B;
  a.n_steps = n_steps;
  a.dt = dt;
  a.stages = stages;
  a.action = action;
  a.action_body = action_body;
  a.dyn_reset = dyn_reset;
  a.reset_mode = dyn_reset ? 1 : 0;
  a.resets = resets;
  a.trace_chosen = chosen;
  a.trace_cells = cells;
  run_any(a, E, 0);
  return 0;
}

// cotix_eval on the host (same argument checks as the library's entry point)
int emu_eval(void* scene, float* dyn, uint32_t* keys, uint32_t* err, const float* geom, int gstride, int B, int n_nfe,
             int wfe, float dt, int stages, const cotix_judge* judge, const cotix_control* control,
             const float* action, int action_body, float* reward, uint32_t* finished, int reset_mode,
             const float* dyn_reset, uint32_t* resets, float* obs, int E) {
  EmuScene* s = static_cast<EmuScene*>(scene);
  if (reset_mode == 1 && judge) return g_err = "reset_mode 1 with a judge", -1;
  if (reset_mode != 0 && !dyn_reset) return g_err = "reset_mode needs dyn_reset", -1;
  if (judge && (!reward || !finished)) return g_err = "a judge needs reward and finished", -1;
  if (B == 0 || n_nfe == 0 || wfe == 0) return 0;
  cxk::KArgs a{};
  const int nb = s->s.nb;
  if (cxk::pack_judge(judge, nb * 6, nb, a.judge, g_err) || cxk::pack_control(control, nb, a.ctl, g_err)) return -1;
  a.sc = &s->s;
  a.dyn = dyn;
  a.keys = keys;
  a.err = err;
  a.geom = geom;
  a.gstride = gstride;
  a.B = B;
  a.n_steps = n_nfe * wfe;
  a.nfe_len = wfe;
  a.dt = dt;
  a.stages = stages;
  a.action = action;
  a.action_held = 1;
  a.action_body = action_body;
  a.reward = reward;
  a.finished = finished;
  a.reset_mode = reset_mode;
  a.dyn_reset = dyn_reset;
  a.resets = resets;
  a.obs = obs;
  run_any(a, E, (a.judge.on || a.ctl.on) ? 3 : 0);
  return 0;
}

int emu_rollout_tape_words(void* scene) {
  const cxk::SceneDev& s = static_cast<EmuScene*>(scene)->s;
  return cxk::tape_words(s.nb, s.nc, s.poly);
}
int emu_rollout(void* scene, float* dyn, uint32_t* keys, uint32_t* err, const float* geom, int gstride, int B,
                int n_steps, float dt, int stages, const float* action, int action_body, const float* ret_w, float* ret,
                float* saved_dyn, uint32_t* saved_keys, uint32_t* tape, int E) {
  EmuScene* s = static_cast<EmuScene*>(scene);
  cxk::KArgs a{};
  a.sc = &s->s;
  a.dyn = dyn;
  a.keys = keys;
  a.err = err;
  a.geom = geom;
  a.gstride = gstride;
  a.B = B;
  a.n_steps = n_steps;
  a.dt = dt;
  a.stages = stages;
  a.action = action;
  a.action_body = action_body;
  a.save_dyn = saved_dyn;
  a.save_keys = saved_keys;
  a.tape = tape;
  a.tw = emu_rollout_tape_words(scene);
  a.ret = ret;
  for (int k = 0; k < s->s.nb * 6; ++k) a.ret_w[k] = ret_w[k];
  run_any(a, E, 1);
  return 0;
}

int emu_rollout_backward(void* scene, const float* saved_dyn, const uint32_t* saved_keys, const uint32_t* tape,
                         const float* geom, int gstride, int B, int n_steps, float dt, int stages, const float* action,
                         int action_body, const float* ret_w, float* grad_action, float* grad_dyn0, int E) {
  EmuScene* s = static_cast<EmuScene*>(scene);
  if ((s->fnset & cxk::FNS_CIRCLE_POLY) && s->s.gjk_steps > cx::CP_GJK_MAX) {  // (the library's admission, cotix_step.hip)
    g_err = "differentiable rollout: circle x polygon gradients record every GJK point: gjk_max_steps <= 32";
    return -1;
  }
  if ((stages & COTIX_STAGE_LUNAR) && !(s->fnset & ~1)) {
    g_err = "differentiable rollout: the LunarLander joint stage needs the polygon program";
    return -1;
  }
  cxk::KArgs a{};
  a.sc = &s->s;
  a.geom = geom;
  a.gstride = gstride;
  a.B = B;
  a.n_steps = n_steps;
  a.dt = dt;
  a.stages = stages & ~COTIX_STAGE_BROADPHASE;  // (the library's re-play, cotix_step.hip)
  a.action = action;
  a.action_body = action_body;
  a.save_dyn = const_cast<float*>(saved_dyn);
  a.save_keys = const_cast<uint32_t*>(saved_keys);
  a.tape = const_cast<uint32_t*>(tape);
  a.tw = emu_rollout_tape_words(scene);
  a.grad_action = grad_action;
  a.grad_dyn = grad_dyn0;
  for (int k = 0; k < s->s.nb * 6; ++k) a.ret_w[k] = ret_w[k];
  // the GPU's split backward (cotix_step.hip launch) where it applies and is asked for
  const bool split = g_split_bwd && tape && E == 4 && cxk::launch_fnset(s->fnset, 4) == cxk::FNS_ANALYTIC &&
                     cxk::split_bwd_ok<4>(a, cxk::make_ctx<4>(s->s));
  run_any(a, E, tape ? (split ? 5 : 4) : 2);
  return 0;
}
// 1: the step launches run the step program with the key helper
// (run_wave + KeyHelper) where the library would; 0 (default): run_wave alone
int emu_set_key_helper(int on) {
  g_key_helper = on != 0;
  return 0;
}
// 1: emu_rollout_backward runs the split tape backward (run_backward_split)
// where the library would; 0 (default): run_wave_backward_tape
int emu_set_split_bwd(int on) {
  g_split_bwd = on != 0;
  return 0;
}

static cx::Shape emu_shape(const float* p) {
  cx::Shape S;
  S.kind = (int)p[0];
  S.n = (int)p[1];
  for (int k = 0; k < 16; ++k) S.w[k] = p[2 + k];
  return S;
}
static cx::NarrowParams emu_narrow(const cotix_params* prm) {
  const cotix_params p = prm ? *prm : cxk::default_params();
  return cx::NarrowParams{cx::gjk_d0(p.prng_layout == COTIX_PRNG_PARTITIONABLE), p.gjk_max_steps, p.epa_max_iters,
                          p.epa_circle_iters, p.epa_body_iters};
}
int emu_contacts_ex(int fn, int n, const float* a, const float* b, float* out, uint32_t* err,
                    const cotix_params* prm) {
  const cx::NarrowParams np = emu_narrow(prm);
  for (int i = 0; i < n; ++i) {
    const cx::Shape A = emu_shape(a + 18 * i), Bs = emu_shape(b + 18 * i);
    uint32_t er = 0;
    cx::Contact c = cx::run_contact(fn, A, Bs, np, &er);
    out[4 * i] = c.pen.x;
    out[4 * i + 1] = c.pen.y;
    out[4 * i + 2] = c.cp.x;
    out[4 * i + 3] = c.cp.y;
    if (err) err[i] = er;
  }
  return 0;
}
int emu_contacts(int fn, int n, const float* a, const float* b, float* out, uint32_t* err) {
  return emu_contacts_ex(fn, n, a, b, out, err, nullptr);
}
// the GJK / EPA operators (host builds of cotix_gjk / cotix_epa)
int emu_gjk(int n, const float* a, const float* b, int32_t* hit, float* simplex, const cotix_params* prm) {
  const cx::NarrowParams np = emu_narrow(prm);
  for (int i = 0; i < n; ++i) {
    const cx::Shape A = emu_shape(a + 18 * i), Bs = emu_shape(b + 18 * i);
    cx::v2 sx[3];
    const bool h = cx::gjk(A, Bs, np.d0, sx, np.gjk_steps);
    hit[i] = h ? 1 : 0;
    for (int k = 0; k < 3; ++k) {
      simplex[6 * i + 2 * k] = h ? sx[k].x : sx[k].x * cx::qnan();
      simplex[6 * i + 2 * k + 1] = h ? sx[k].y : sx[k].y * cx::qnan();
    }
  }
  return 0;
}
int emu_epa(int n, const float* a, const float* b, const float* simplex, int iters, float* pen) {
  if (iters < 3 || iters > 128) return -1;
  for (int i = 0; i < n; ++i) {
    const cx::Shape A = emu_shape(a + 18 * i), Bs = emu_shape(b + 18 * i);
    const float* s = simplex + 6 * i;
    const cx::v2 sx[3] = {cx::v2{s[0], s[1]}, cx::v2{s[2], s[3]}, cx::v2{s[4], s[5]}};
    const cx::v2 p = cx::epa_big(A, Bs, sx, iters);
    pen[2 * i] = p.x;
    pen[2 * i + 1] = p.y;
  }
  return 0;
}
}

// random_direction(key) and the GJK start direction (cotix_gjk_ex's device code)
extern "C" int emu_gjk_start(int n, const uint32_t* keys, const float* init, int part, float* out) {
  for (int i = 0; i < n; ++i) {
    cx::v2 d = cx::gjk_d0(part != 0);
    if (keys) d = cx::random_direction(cx::key2{keys[2 * i], keys[2 * i + 1]}, part != 0);
    if (init) d = cx::gjk_start(d, cx::v2{init[2 * i], init[2 * i + 1]});
    out[2 * i] = d.x;
    out[2 * i + 1] = d.y;
  }
  return 0;
}

extern "C" int emu_order_clockwise(float* xy, int n, int nv) {
  for (int i = 0; i < n; ++i) {
    float v[2 * cx::MAXV] = {};
    for (int k = 0; k < 2 * nv; ++k) v[k] = xy[(size_t)i * 2 * nv + k];
    cx::order_clockwise(v, nv);
    for (int k = 0; k < 2 * nv; ++k) xy[(size_t)i * 2 * nv + k] = v[k];
  }
  return 0;
}

// body-level operators on the host (same device code as the gfx950 kernels)
static int emu_body_parts(const EmuScene* es, int body, cxk::BodyParts* bp) {
  const cxk::SceneDev& s = es->s;
  bp->body = body;
  bp->n = 0;
  for (int p = 0; p < s.np; ++p) {
    if ((int)s.hot[s.o_pbody + p] != body) continue;
    if (bp->n >= cxk::MAXBP) return -1;
    bp->kind[bp->n] = (int)s.hot[s.o_pkind + p];
    bp->nv[bp->n] = (int)s.hot[s.o_pn + p];
    bp->goff[bp->n] = (int)s.hot[s.o_pgoff + p];
    ++bp->n;
  }
  return bp->n > 0 ? 0 : -1;
}
extern "C" int emu_body_penetration(void* scene, const float* dyn, const float* geom, int gstride, int B, int ba,
                                    int bb, int* collides, float* pen) {
  const EmuScene* es = static_cast<EmuScene*>(scene);
  cxk::BodyParts pa, pb;
  if (emu_body_parts(es, ba, &pa) || emu_body_parts(es, bb, &pb)) return -1;
  for (int g = 0; g < B; ++g) {
    cx::v2 p;
    collides[g] = cxk::body_penetration_env(dyn, B, geom, gstride, pa, pb, cxk::narrow_of(es->s), g, &p);
    pen[2 * g] = p.x;
    pen[2 * g + 1] = p.y;
  }
  return 0;
}
extern "C" int emu_body_aabb(void* scene, const float* dyn, const float* geom, int gstride, int B, int body,
                             float* out, uint32_t* err) {
  const EmuScene* es = static_cast<EmuScene*>(scene);
  cxk::BodyParts pa;
  if (emu_body_parts(es, body, &pa)) return -1;
  for (int g = 0; g < B; ++g) err[g] |= cxk::body_aabb_env(dyn, B, geom, gstride, pa, g, out + 4 * g);
  return 0;
}

#ifdef COTIX_STATS
// workload counters (tools/collider_stats.py): read and reset
extern "C" int emu_stats(unsigned long long* out) {
  out[0] = cxk::g_stats.wave_steps;
  out[1] = cxk::g_stats.active_items;
  out[2] = cxk::g_stats.rounds;
  out[3] = cxk::g_stats.resolutions;
  out[4] = cxk::g_stats.f_items;
  out[5] = cxk::g_stats.b_items;
  out[6] = cxk::g_stats.draws;
  out[7] = cxk::g_stats.valid_draws;
  out[8] = cxk::g_stats.r1_left;
  out[9] = cxk::g_stats.lvl_env;
  out[10] = cxk::g_stats.lvl_wave;
  out[11] = cxk::g_stats.e1_slots;
  out[12] = cxk::g_stats.valid_cands;
  out[13] = cxk::g_stats.fit64;
  out[14] = cxk::g_stats.bp_cand;
  out[15] = cxk::g_stats.bp_guard_fail;
  out[16] = cxk::g_stats.epa_runs;
  cxk::g_stats = cxk::Stats{};
  return 17;
}
#endif

// the kernels' deterministic f32 transcendentals (tests: vs the oracle)
extern "C" int emu_sincos(const float* x, int n, float* s, float* c) {
  for (int i = 0; i < n; ++i) cx::sincos32(x[i], &s[i], &c[i]);
  return 0;
}
extern "C" int emu_atan2(const float* y, const float* x, int n, float* out) {
  for (int i = 0; i < n; ++i) out[i] = cx::atan2_32(y[i], x[i]);
  return 0;
}

// render export and state check (host builds of cotix_render / cotix_check_state)
extern "C" int emu_render(void* scene, const float* dyn, const float* geom, int gstride, int B, float* prims) {
  const cxk::SceneDev& s = static_cast<EmuScene*>(scene)->s;
  if (s.np > cxk::MAXRP) return -1;
  cxk::SceneParts sp;
  sp.np = s.np;
  int off = 0;
  for (int p = 0; p < s.np; ++p) {
    sp.body[p] = (int)s.hot[s.o_pbody + p];
    sp.kind[p] = (int)s.hot[s.o_pkind + p];
    sp.nv[p] = (int)s.hot[s.o_pn + p];
    sp.goff[p] = (int)s.hot[s.o_pgoff + p];
    sp.poff[p] = off;
    off += cxk::render_prims(sp.kind[p], sp.nv[p]);
  }
  if (prims == nullptr) return off;  // count query
  for (int g = 0; g < B; ++g)
    for (int p = 0; p < s.np; ++p) cxk::render_part_env(dyn, B, geom, gstride, sp, p, g, prims + (size_t)g * off * 4);
  return off;
}
extern "C" int emu_check_state(const float* dyn, int nb, int B, uint32_t* err) {
  for (int g = 0; g < B; ++g) err[g] |= cxk::state_check_env(dyn, nb, B, g);
  return 0;
}

// scene header fields the step kernel specializes on (cxk::SceneDims)
extern "C" int emu_scene_dims(void* scene, int* out) {
  const cxk::SceneHdr& h = static_cast<EmuScene*>(scene)->s;
  const int v[] = {h.nb, h.np, h.nc, h.nl, h.nt, h.G, h.W, h.nmw, h.poly, h.rcp_all, (int)h.rcp_mask, h.nvt, h.fnset};
  for (int k = 0; k < 13; ++k) out[k] = v[k];
  return 13;
}
// the step-kernel specialization the launcher picks for the scene (cxk::spec_of)
extern "C" int emu_scene_spec(void* scene) { return cxk::spec_of(static_cast<EmuScene*>(scene)->s); }

// the scene's header as a C++ initializer in declaration order (floats as
// exact hex literals): tools/gen_spec_hdrs.py writes the specializations'
// constant headers (cotix_spec_hdrs.h) from it; returns the length, -1 if
// buf is too small
static void hdr_put(std::string& o, const char* name, uint16_t v) { o += std::string("/*") + name + "*/ " + std::to_string(v) + ", "; }
static void hdr_put(std::string& o, const char* name, uint32_t v) {
  o += std::string("/*") + name + "*/ " + std::to_string(v) + "u, ";
}
static void hdr_put(std::string& o, const char* name, float v) {
  char b[64];
  std::snprintf(b, sizeof b, "%af", (double)v);
  o += std::string("/*") + name + "*/ " + b + ", ";
}
// the scene's hot tables (tooling: table inspection); returns nhot
extern "C" int emu_scene_hot(void* scene, uint32_t* out, int n) {
  const cxk::SceneDev& s = static_cast<EmuScene*>(scene)->s;
  for (int q = 0; q < s.nhot && q < n; ++q) out[q] = s.hot[q];
  return s.nhot;
}
extern "C" int emu_scene_hdr_text(void* scene, char* buf, int n) {
  const cxk::SceneHdr& h = static_cast<EmuScene*>(scene)->s;
  std::string o = "{";
#define EMU_HDR_PUT(T, f) hdr_put(o, #f, h.f);
  CXK_HDR_FIELDS(EMU_HDR_PUT)
#undef EMU_HDR_PUT
  o.resize(o.size() - 2);
  o += "}";
  if ((int)o.size() + 1 > n) return -1;
  std::memcpy(buf, o.c_str(), o.size() + 1);
  return (int)o.size();
}
// LDS bytes of the step kernel's workgroup (cxk::lds_bytes, 4 waves) for the scene at `ew` envs per wave
extern "C" long emu_lds_bytes(void* scene, int ew) {
  return (long)cxk::lds_bytes(static_cast<EmuScene*>(scene)->s, 4, ew);
}
extern "C" long emu_lds_bytes_w(void* scene, int ew, int wpb) {
  return (long)cxk::lds_bytes(static_cast<EmuScene*>(scene)->s, wpb, ew);
}

// circle x polygon: the gradient's recorded re-run (cx::cp_forward) against
// the forward contact (cx::circle_vs_polygon) -- same penetration bits
extern "C" int emu_circle_poly_check(int n, const float* a, const float* b, float* pen_fwd, float* pen_rec) {
  const cx::NarrowParams np = cx::narrow_default();
  for (int i = 0; i < n; ++i) {
    cx::Shape C, P;
    C.kind = cx::KIND_CIRCLE;
    C.n = 0;
    P.kind = cx::KIND_POLY;
    P.n = (int)b[18 * i + 1];
    for (int k = 0; k < 2 * cx::MAXV; ++k) {
      C.w[k] = a[18 * i + 2 + k];
      P.w[k] = b[18 * i + 2 + k];
    }
    const cx::Contact ct = cx::circle_vs_polygon(C, P, np);
    pen_fwd[2 * i] = ct.pen.x;
    pen_fwd[2 * i + 1] = ct.pen.y;
    cx::CPRec R;
    int e0 = -1, e1 = -1;
    cx::v2 pr = cx::v2{cx::qnan(), cx::qnan()};
    if (cx::cp_forward(C, P, np, R, &e0, &e1) && e0 >= 0 && e1 >= 0) pr = cx::closest_on_edge_to_origin(R.p[e0], R.p[e1]);
    else if (cx::cp_forward(C, P, np, R, &e0, &e1)) pr = cx::v2{0.0f, 0.0f};
    pen_rec[2 * i] = pr.x;
    pen_rec[2 * i + 1] = pr.y;
  }
  return 0;
}
