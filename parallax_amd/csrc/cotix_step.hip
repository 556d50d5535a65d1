// cotix_step.hip -- MI355X (gfx950) operator kernels of the cotix per-step hot
// path and the C-ABI declared in include/cotix_amd.h.  The fused step kernel
// is cotix_step_kernel.hip (one translation unit per envs-per-wave tiling,
// compiled in parallel); its phases live in cotix_kernel.h (design notes there
// and in DESIGN.md).
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/cotix_amd.h"
#include "cotix_device.h"
#include "cotix_body.h"
#include "cotix_kernel.h"
#include "cotix_launch.h"
#include "cotix_scene.h"

using cxk::FNS_ANALYTIC;
using cxk::FNS_CIRCLE_POLY;
using cxk::FNS_CONVEX;
using cxk::SceneDev;

namespace {
thread_local std::string g_err;
int fail(const std::string& m) {
  g_err = m;
  return -1;
}
int hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) return fail(std::string(what) + ": " + hipGetErrorString(e));
  return 0;
}
}  // namespace

struct cotix_scene {
  SceneDev host;
  SceneDev* dev = nullptr;
  int n_candidates = 0;
  int fnset = 0;
  // kernel variant (cotix_scene_set_variant): envs per wave and whether the
  // reference scenes' specializations may be used -- every variant computes
  // the same bits; the defaults are the measured best (envs per wave: 4, or
  // the largest tiling whose LDS fits, lds_default_ew)
  int envs_per_wave = 4;
  int specialize = 1;
};
// a workgroup's LDS at `ew` envs per wave and `wpb` waves (cxk::lds_bytes:
// the hot tables + wpb tiles and wave scratches) and the hardware's 160 KiB
// per CU
constexpr size_t LDS_CAP = 160 * 1024;
static size_t scene_lds_w(const cotix_scene* sc, int ew, int wpb) { return cxk::lds_bytes(sc->host, wpb, ew); }
// waves per workgroup of a tiling: WPB (one per SIMD), or for a scene whose
// tiles do not fit four at a time 2, then 1 -- a workgroup of one wave holds
// one tile and the tables; 0: not even that fits (the scene's hard cap)
static int scene_wpb(const cotix_scene* sc, int ew) {
  for (int w : {cxl::WPB, 2, 1})
    if (scene_lds_w(sc, ew, w) <= LDS_CAP) return w;
  return 0;
}
static size_t scene_lds(const cotix_scene* sc, int ew) {
  const int w = scene_wpb(sc, ew);
  return scene_lds_w(sc, ew, w ? w : 1);
}
// the default tiling of a scene: 4 envs per wave (the measured best), else
// the largest of 2, 1 whose workgroup of WPB waves fits the LDS, else one env
// per wave in workgroups of 2 or 1 waves; 0: none fits
static int lds_default_ew(const cotix_scene* sc) {
#ifdef COTIX_EW4_ONLY
  return scene_lds_w(sc, 4, cxl::WPB) <= LDS_CAP ? 4 : 0;
#else
  for (int ew : {4, 2, 1})
    if (scene_lds_w(sc, ew, cxl::WPB) <= LDS_CAP) return ew;
  return scene_wpb(sc, 1) ? 1 : 0;
#endif
}
// the specialization a launch of this scene uses (cxk::SPEC_*)
static int scene_spec(const cotix_scene* scene) {
  return scene->specialize ? cxk::spec_of(scene->host) : cxk::SPEC_GENERIC;
}

namespace {

// ---------------------------------------------------------------------------
// operator kernels
// ---------------------------------------------------------------------------
__device__ __forceinline__ cx::Shape load_shape(const float* p) {
  cx::Shape s;
  s.kind = (int)p[0];
  s.n = (int)p[1];
#pragma unroll
  for (int k = 0; k < 2 * cx::MAXV; ++k) s.w[k] = p[2 + k];
  return s;
}
__global__ void contacts_kernel(int fn, int n, const float* a, const float* b, float* out, uint32_t* err,
                                cx::NarrowParams np) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const cx::Shape A = load_shape(a + 18 * (size_t)i), Bs = load_shape(b + 18 * (size_t)i);
  uint32_t er = 0u;
  cx::Contact c = cx::run_contact(fn, A, Bs, np, &er);
  out[4 * (size_t)i + 0] = c.pen.x;
  out[4 * (size_t)i + 1] = c.pen.y;
  out[4 * (size_t)i + 2] = c.cp.x;
  out[4 * (size_t)i + 3] = c.cp.y;
  if (err) err[i] = er;
}
using cxk::BodyParts;
using cxk::MAXBP;
__global__ void body_pen_kernel(const float* dyn, int B, const float* geom, int gstride, BodyParts pa, BodyParts pb,
                                cx::NarrowParams np, int* collides, float* pen) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= B) return;
  cx::v2 p;
  collides[g] = cxk::body_penetration_env(dyn, B, geom, gstride, pa, pb, np, g, &p) ? 1 : 0;
  pen[2 * (size_t)g] = p.x;
  pen[2 * (size_t)g + 1] = p.y;
}
__global__ void body_aabb_kernel(const float* dyn, int B, const float* geom, int gstride, BodyParts pa, float* out,
                                 uint32_t* err) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= B) return;
  const uint32_t e = cxk::body_aabb_env(dyn, B, geom, gstride, pa, g, out + 4 * (size_t)g);
  if (err && e) err[g] |= e;
}
__global__ void render_kernel(const float* dyn, int B, const float* geom, int gstride, cxk::SceneParts sp, int nprim,
                              float* prims) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;  // (env, part), part fastest
  if (t >= (long long)B * sp.np) return;
  const int g = (int)(t / sp.np), p = (int)(t % sp.np);
  cxk::render_part_env(dyn, B, geom, gstride, sp, p, g, prims + (size_t)g * nprim * 4);
}
// SoA [nb*6][B] -> per env [B][nb*6]: each thread one output word; the
// block's 256 outputs read 256 / (nb*6) envs of every state row
__global__ void observe_kernel(const float* dyn, int nw, int B, float* obs) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)nw * B) return;
  const int g = (int)(t / nw), k = (int)(t % nw);
  obs[t] = dyn[(size_t)k * B + g];
}
__global__ void check_state_kernel(const float* dyn, int nb, int B, uint32_t* err) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= B) return;
  const uint32_t e = cxk::state_check_env(dyn, nb, B, g);
  if (e) err[g] |= e;
}
__global__ void resolve_kernel(int n, float* d1, const float* p1, float* d2, const float* p2, const float* con,
                               cx::Baum bm) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float* a = d1 + 6 * (size_t)i;
  float* b = d2 + 6 * (size_t)i;
  cx::Dyn x = cx::Dyn{a[0], a[1], a[2], a[3], a[4], a[5]}, y = cx::Dyn{b[0], b[1], b[2], b[3], b[4], b[5]};
  const float* q1 = p1 + 4 * (size_t)i;
  const float* q2 = p2 + 4 * (size_t)i;
  cx::Params m1 = cx::Params{q1[0], q1[1], q1[2], q1[3]}, m2 = cx::Params{q2[0], q2[1], q2[2], q2[3]};
  const float* c = con + 4 * (size_t)i;
  cx::resolve_collision(x, m1, y, m2, cx::v2{c[0], c[1]}, cx::v2{c[2], c[3]}, bm);
  a[2] = x.vx; a[3] = x.vy; a[5] = x.w;
  b[2] = y.vx; b[3] = y.vy; b[5] = y.w;
}
__global__ void threefry_kernel(const uint32_t* k, const uint32_t* c, uint32_t* o, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  cx::key2 r = cx::threefry(cx::key2{k[2 * i], k[2 * i + 1]}, c[2 * i], c[2 * i + 1]);
  o[2 * i] = r.a;
  o[2 * i + 1] = r.b;
}
__global__ void split_kernel(const uint32_t* k, int n, int num, uint32_t* o, int part) {
  long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)n * num) return;
  int i = (int)(t / num), j = (int)(t % num);
  cx::key2 r = cx::split_at_l(cx::key2{k[2 * i], k[2 * i + 1]}, (uint32_t)num, (uint32_t)j, part != 0);
  o[2 * t] = r.a;
  o[2 * t + 1] = r.b;
}
// uniform(key, (count,)): word m of the draw.  Legacy: iota(count) counters
// split in halves (zero pad when odd); partitionable: y0 ^ y1 of block (0, m)
__global__ void uniform_kernel(const uint32_t* k, int n, int count, float lo, float hi, float* o, int part) {
  long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)n * count) return;
  int i = (int)(t / count), m = (int)(t % count);
  cx::key2 key = cx::key2{k[2 * i], k[2 * i + 1]};
  int half = (count + 1) / 2;  // padded counter array split in two halves
  uint32_t w;
  if (part) {
    const cx::key2 r = cx::threefry(key, 0u, (uint32_t)m);
    w = r.a ^ r.b;
  } else {
    w = (m < half) ? cx::threefry(key, (uint32_t)m, (uint32_t)(m + half < count ? m + half : 0)).a
                   : cx::threefry(key, (uint32_t)(m - half), (uint32_t)m).b;
  }
  // the odd pad counter is 0: block (half-1, pad) only feeds word half-1
  o[t] = cx::fmax_(lo, cx::unit_float(w) * (hi - lo) + lo);
}
__global__ void order_cw_kernel(float* xy, int n, int nv) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float v[2 * cx::MAXV];
  for (int k = 0; k < 2 * nv; ++k) v[k] = xy[(size_t)i * 2 * nv + k];
  cx::order_clockwise(v, nv);
  for (int k = 0; k < 2 * nv; ++k) xy[(size_t)i * 2 * nv + k] = v[k];
}
// check_for_collision_convex (cotix/_collisions.py:277-310): hit and the
// simplex, NaN * simplex when there is no collision
// init / keys (cotix_gjk_ex, nullable): per item the initial_direction and
// the key of check_for_collision_convex (cotix/_collisions.py:277-298)
__global__ void gjk_kernel(int n, const float* a, const float* b, int32_t* hit, float* simplex, cx::NarrowParams np,
                           const float* init, const uint32_t* keys, int part) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const cx::Shape A = load_shape(a + 18 * (size_t)i), Bs = load_shape(b + 18 * (size_t)i);
  cx::v2 d0 = np.d0;
  if (keys != nullptr) d0 = cx::random_direction(cx::key2{keys[2 * (size_t)i], keys[2 * (size_t)i + 1]}, part != 0);
  if (init != nullptr) d0 = cx::gjk_start(d0, cx::v2{init[2 * (size_t)i], init[2 * (size_t)i + 1]});
  cx::v2 sx[3];
  const bool h = cx::gjk(A, Bs, d0, sx, np.gjk_steps);
  hit[i] = h ? 1 : 0;
  for (int k = 0; k < 3; ++k) {  // (False, nan * simplex) when there is no collision
    simplex[6 * (size_t)i + 2 * k] = h ? sx[k].x : sx[k].x * cx::qnan();
    simplex[6 * (size_t)i + 2 * k + 1] = h ? sx[k].y : sx[k].y * cx::qnan();
  }
}
// compute_penetration_vector_convex (:313-329): EPA from a given simplex
__global__ void epa_kernel(int n, const float* a, const float* b, const float* simplex, int iters, float* pen) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const cx::Shape A = load_shape(a + 18 * (size_t)i), Bs = load_shape(b + 18 * (size_t)i);
  const float* s = simplex + 6 * (size_t)i;
  const cx::v2 sx[3] = {cx::v2{s[0], s[1]}, cx::v2{s[2], s[3]}, cx::v2{s[4], s[5]}};
  const cx::v2 p = cx::epa_big(A, Bs, sx, iters);
  pen[2 * (size_t)i] = p.x;
  pen[2 * (size_t)i + 1] = p.y;
}
__global__ void euler_kernel(float* dyn, int nb, int B, float dt) {
  long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)nb * B) return;
  int b = (int)(t / B), g = (int)(t % B);
  float* d = dyn + (size_t)b * 6 * B + g;
  d[0] = d[0] + d[2 * (size_t)B] * dt;
  d[(size_t)B] = d[(size_t)B] + d[3 * (size_t)B] * dt;
  d[4 * (size_t)B] = d[4 * (size_t)B] + d[5 * (size_t)B] * dt;
}
__global__ void lunar_kernel(float* dyn, int B, cx::Params p0, cx::Params p1, cx::Params p2) {
  int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= B) return;
  cx::Dyn d[3];
  for (int b = 0; b < 3; ++b) {
    float* q = dyn + (size_t)b * 6 * B + g;
    d[b] = cx::Dyn{q[0], q[(size_t)B], q[2 * (size_t)B], q[3 * (size_t)B], q[4 * (size_t)B], q[5 * (size_t)B]};
  }
  cxk::lunar_constraints(d[0], d[1], d[2], p0, p1, p2);
  for (int b = 0; b < 3; ++b) {
    float* q = dyn + (size_t)b * 6 * B + g;
    q[2 * (size_t)B] = d[b].vx;
    q[3 * (size_t)B] = d[b].vy;
    q[5 * (size_t)B] = d[b].w;
  }
}

}  // namespace

extern "C" {

const char* cotix_last_error(void) { return g_err.c_str(); }
#ifndef COTIX_BUILD_ID
#define COTIX_BUILD_ID "unknown"
#endif
// the build id is a hash of the kernel sources + compile flags (__graft_entry__.build_id):
// profiles/latest_pmc_*.json are keyed to it, so a counter pass of older code is never
// divided by a newer kernel's time (bench.py)
const char* cotix_version(void) { return "cotix_amd 0.2 (gfx950) build " COTIX_BUILD_ID; }


int cotix_params_default(cotix_params* out) {
  if (!out) return fail("null argument");
  *out = cxk::default_params();
  return 0;
}

int cotix_scene_create_ex2(int n_bodies, const float* body_params, int n_parts, const int* part_body,
                           const int* part_type, const int* part_nverts, const cotix_params* params, int flags,
                           cotix_scene** out) {
  if (!out) return fail("null argument");
  cotix_scene* sc = new cotix_scene();
  if (cxk::compile_scene(n_bodies, body_params, n_parts, part_body, part_type, part_nverts, sc->host,
                         sc->n_candidates, sc->fnset, g_err, params, flags)) {
    delete sc;
    return -1;
  }
  // the tiling is a property of the scene: a scene whose tile does not fit
  // the LDS even at one env per wave is rejected here, not at its first launch
  sc->envs_per_wave = lds_default_ew(sc);
  if (sc->envs_per_wave == 0) {
    const size_t need = scene_lds_w(sc, 1, 1);
    delete sc;
    return fail("scene too large for the LDS tile: " + std::to_string(need) + " bytes for one env's tile and the "
                "tables (a workgroup of one wave), the CU has " + std::to_string(LDS_CAP));
  }
  *out = sc;
  return 0;
}

int cotix_scene_create_ex(int n_bodies, const float* body_params, int n_parts, const int* part_body,
                          const int* part_type, const int* part_nverts, const cotix_params* params,
                          cotix_scene** out) {
  return cotix_scene_create_ex2(n_bodies, body_params, n_parts, part_body, part_type, part_nverts, params, 0, out);
}

int cotix_scene_create(int n_bodies, const float* body_params, int n_parts, const int* part_body,
                       const int* part_type, const int* part_nverts, cotix_scene** out) {
  return cotix_scene_create_ex(n_bodies, body_params, n_parts, part_body, part_type, part_nverts, nullptr, out);
}

int cotix_scene_params(const cotix_scene* scene, cotix_params* out) {
  if (!scene || !out) return fail("null argument");
  *out = cxk::params_of(scene->host);
  return 0;
}

int cotix_scene_destroy(cotix_scene* scene) {
  if (!scene) return 0;
  if (scene->dev) (void)hipFree(scene->dev);
  delete scene;
  return 0;
}

int cotix_scene_set_variant(cotix_scene* scene, int envs_per_wave, int specialize) {
  if (!scene) return fail("null scene");
  if (envs_per_wave == 0) envs_per_wave = lds_default_ew(scene);
  if (envs_per_wave != 1 && envs_per_wave != 2 && envs_per_wave != 4 && envs_per_wave != 8)
    return fail("envs_per_wave must be 0 (default), 1, 2, 4 or 8");
#ifdef COTIX_EW4_ONLY
  if (envs_per_wave != 4) return fail("this build carries the 4-envs-per-wave tiling only");
#endif
  if (scene_wpb(scene, envs_per_wave) == 0)
    return fail("envs_per_wave " + std::to_string(envs_per_wave) + ": the scene's workgroup needs " +
                std::to_string(scene_lds(scene, envs_per_wave)) + " bytes of LDS, the CU has " +
                std::to_string(LDS_CAP));
  scene->envs_per_wave = envs_per_wave;
  scene->specialize = specialize ? 1 : 0;
  return 0;
}

int cotix_scene_waves_per_group(const cotix_scene* scene) {
  if (!scene) return fail("null scene");
  return scene_wpb(scene, scene->envs_per_wave);
}

int cotix_scene_variant(const cotix_scene* scene, int* envs_per_wave, int* spec) {
  if (!scene) return fail("null scene");
  if (envs_per_wave) *envs_per_wave = scene->envs_per_wave;
  // the step program's specialization, as the launcher has it
  // (cotix_step_kernel.hip): the reference scenes at 4 and 2 envs per wave,
  // the box world's structure at 4 only
  if (spec) {
    const int ew = scene->envs_per_wave, s = scene_spec(scene);
    *spec = (ew == 4 || (ew == 2 && s != cxk::SPEC_BOX)) ? s : cxk::SPEC_GENERIC;
  }
  return 0;
}

int cotix_scene_geom_floats(const cotix_scene* scene) { return scene ? scene->host.G : fail("null scene"); }

int cotix_scene_info(const cotix_scene* scene, int* n_contacts, int* n_cells, int* n_candidates, int* n_types) {
  if (!scene) return fail("null scene");
  if (n_contacts) *n_contacts = scene->host.nc;
  if (n_cells) *n_cells = scene->host.nl;
  if (n_candidates) *n_candidates = scene->n_candidates;
  if (n_types) *n_types = scene->host.nt;
  return 0;
}

// device copy of the scene tables, made on first use (so scenes compile on
// hosts without a GPU; the first step is therefore not graph-capturable)
static int scene_upload(cotix_scene* sc) {
  if (sc->dev) return 0;
  if (hip_check(hipMalloc(&sc->dev, sizeof(SceneDev)), "hipMalloc(scene)")) return -1;
  return hip_check(hipMemcpy(sc->dev, &sc->host, sizeof(SceneDev), hipMemcpyHostToDevice), "hipMemcpy(scene)");
}


static int check_step_args(const cotix_scene* scene, const float* dyn, const uint32_t* keys, const float* geom,
                           int geom_stride, int B, int n_steps, int stages, const float* action, int action_body) {
  if (!scene || !dyn || !keys) return fail("null argument");
  if ((stages & COTIX_STAGE_COLLIDER) && !geom) return fail("geometry required for the collider stage");
  if (geom_stride != 0 && geom_stride < scene->host.G) return fail("geom_stride smaller than the scene geometry");
  if (B < 0 || n_steps < 0) return fail("negative size");
  if ((stages & COTIX_STAGE_LUNAR) && scene->host.nb < 3) return fail("LunarLander stage needs >= 3 bodies");
  if (action && (action_body < 0 || action_body >= scene->host.nb)) return fail("action_body out of range");
  return 0;
}

// the split tape backward is the default; COTIX_SPLIT_BWD=0 launches MODE 4
// at one wave per env group instead (A/B measurements; the same bits)
static bool split_bwd_enabled() {
  static const int on = [] {
    const char* v = getenv("COTIX_SPLIT_BWD");
    return v == nullptr || atoi(v) != 0 ? 1 : 0;
  }();
  return on != 0;
}
// the key-window helper is the default for the step launches it applies to;
// COTIX_KEY_HELPER=0 launches step_kernel alone (A/B measurements; the same bits)
static bool key_helper_enabled() {
  static const int on = [] {
    const char* v = getenv("COTIX_KEY_HELPER");
    return v == nullptr || atoi(v) != 0 ? 1 : 0;
  }();
  return on != 0;
}
// launch the fused step kernel (mode 0 step, 1 rollout forward, 2 backward re-play, 3 eval with a judge/control)
static int launch(cotix_scene* scene, const cxk::KArgs& ka0, int mode, cotix_stream_t stream) {
  if (scene_upload(scene)) return -1;
#ifdef COTIX_EW4_ONLY
  const int EW = 4;
#else
  const int EW = scene->envs_per_wave;
#endif
  const int wpb = scene_wpb(scene, EW);
  if (wpb == 0) return fail("scene too large for the LDS tile");  // (not reached: checked at create / set_variant)
  const size_t lds = scene_lds_w(scene, EW, wpb);
  cxk::KArgs ka = ka0;
  ka.sc = scene->dev;
  ka.sh = scene->host;  // the header by value (kernel arguments)
#ifdef COTIX_TOOLING  // phase-cost experiments only (cotix_kernel.h CXK_SKIP)
  const char* dbg = getenv("COTIX_DEBUG_SKIP");
  ka.dbg_skip = dbg ? atoi(dbg) : 0;
#endif
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int fs = scene->fnset;
  // scene specialization (compile-time dimensions; reference scenes, whose
  // tiles always fit WPB to a workgroup)
  const int spec = wpb == cxl::WPB ? scene_spec(scene) : cxk::SPEC_GENERIC;
  // the tape backward at two waves per env group where the scene allows it
  // and two tiles per group fit (cxk::run_backward_split; the same bits)
  if (mode == 4 && EW == 4 && wpb == cxl::WPB && split_bwd_enabled() &&
      cxk::launch_fnset(fs, mode) == cxk::FNS_ANALYTIC &&
      cxk::split_bwd_ok<4>(ka, cxk::make_ctx<4>(scene->host)) &&
      scene_lds_w(scene, 4, 2 * cxl::WPB) <= LDS_CAP) {
    const int r = cxl::launch_bwd_split(ka, spec, scene_lds_w(scene, 4, 2 * cxl::WPB), st);
    if (r == 0) return hip_check(hipGetLastError(), "bwd_split_kernel launch");
  }
  // the step program with a key-window helper wave per env group where the
  // launch has more than one key window (cxk::KeyHelper; the same bits)
  if (mode == 0 && EW == 4 && wpb == cxl::WPB && ka.n_steps > cxk::KWIN && key_helper_enabled() &&
      cxk::launch_fnset(fs, mode) == cxk::FNS_ANALYTIC &&
      cxk::help_lds_bytes<4>(scene->host, cxl::WPB) <= LDS_CAP) {
    const int r = cxl::launch_step_help(ka, spec, cxk::help_lds_bytes<4>(scene->host, cxl::WPB), st);
    if (r == 0) return hip_check(hipGetLastError(), "step_help_kernel launch");
  }
  hipError_t e;
#ifdef COTIX_EW4_ONLY  // tooling builds (phase profile, ISA markers): the default tiling only
  e = cxl::launch_step_ew4(ka, fs, mode, lds, st, spec, wpb);
#else
  if (EW == 1) e = cxl::launch_step_ew1(ka, fs, mode, lds, st, spec, wpb);
  else if (EW == 2) e = cxl::launch_step_ew2(ka, fs, mode, lds, st, spec, wpb);
  else if (EW == 8) e = cxl::launch_step_ew8(ka, fs, mode, lds, st, spec, wpb);
  else e = cxl::launch_step_ew4(ka, fs, mode, lds, st, spec, wpb);
#endif
  if (e != hipSuccess) return hip_check(e, "step_kernel launch");
  return hip_check(hipGetLastError(), "step_kernel launch");
}

static int step_impl(cotix_scene* scene, float* dyn, uint32_t* keys, uint32_t* err, const float* geom,
                     int geom_stride, int B, int n_steps, float dt, int stages, const float* action, int action_body,
                     const float* dyn_reset, uint32_t* resets, int32_t* chosen, int32_t* cells,
                     cotix_stream_t stream) {
  if (check_step_args(scene, dyn, keys, geom, geom_stride, B, n_steps, stages, action, action_body)) return -1;
  if (!err) return fail("null argument");
  if (B == 0 || n_steps == 0) return 0;
  cxk::KArgs ka{};
  ka.dyn = dyn;
  ka.keys = keys;
  ka.err = err;
  ka.geom = geom;
  ka.gstride = geom_stride;
  ka.B = B;
  ka.n_steps = n_steps;
  ka.dt = dt;
  ka.stages = stages;
  ka.action = action;
  ka.action_body = action_body;
  ka.dyn_reset = dyn_reset;
  ka.reset_mode = dyn_reset ? 1 : 0;
  ka.resets = resets;
  ka.trace_chosen = chosen;
  ka.trace_cells = cells;
  return launch(scene, ka, 0, stream);
}

int cotix_eval(cotix_scene* scene, float* dyn, uint32_t* keys, uint32_t* err, const float* geom, int geom_stride,
               int B, int n_nfe, int wfe, float dt, int stages, const cotix_judge* judge,
               const cotix_control* control, const float* action, int action_body, float* reward,
               uint32_t* finished, int reset_mode, const float* dyn_reset, uint32_t* resets, float* obs,
               cotix_stream_t stream) {
  if (n_nfe < 0 || wfe < 0) return fail("negative size");
  if (wfe > 0 && n_nfe > INT_MAX / wfe) return fail("n_nfe * wfe overflows");
  if (check_step_args(scene, dyn, keys, geom, geom_stride, B, n_nfe * wfe, stages, action, action_body)) return -1;
  if (!err) return fail("null argument");
  if (reset_mode < 0 || reset_mode > 2) return fail("reset_mode must be 0, 1 or 2");
  if (reset_mode != 0 && !dyn_reset) return fail("reset_mode needs dyn_reset");
  if (reset_mode == 1 && judge) return fail("reset_mode 1 (restart on error) cannot be combined with a judge");
  if (reset_mode == 2 && !finished) return fail("reset_mode 2 needs finished");
  // reset_mode 2 restarts the envs the judge finished; without a judge nothing
  // would clear `finished`, so every later call would restart them again
  if (reset_mode == 2 && !judge) return fail("reset_mode 2 (restart finished envs) needs a judge");
  if (judge && (!reward || !finished)) return fail("a judge needs reward and finished");
  if (B == 0 || n_nfe == 0 || wfe == 0) return 0;
  cxk::KArgs ka{};
  const int nb = scene->host.nb;
  if (cxk::pack_judge(judge, nb * 6, nb, ka.judge, g_err) || cxk::pack_control(control, nb, ka.ctl, g_err)) return -1;
  ka.dyn = dyn;
  ka.keys = keys;
  ka.err = err;
  ka.geom = geom;
  ka.gstride = geom_stride;
  ka.B = B;
  ka.n_steps = n_nfe * wfe;
  ka.nfe_len = wfe;
  ka.dt = dt;
  ka.stages = stages;
  ka.action = action;
  ka.action_held = 1;
  ka.action_body = action_body;
  ka.reward = reward;
  ka.finished = finished;
  ka.reset_mode = reset_mode;
  ka.dyn_reset = dyn_reset;
  ka.resets = resets;
  ka.obs = obs;
  // the judge / control program only when one is on: the plain step program
  // (specialized, fewer registers) serves the rest (obs, held action, resets)
  return launch(scene, ka, (ka.judge.on || ka.ctl.on) ? 3 : 0, stream);
}

int cotix_step(cotix_scene* scene, float* dyn, uint32_t* keys, uint32_t* err, const float* geom, int geom_stride,
               int B, int n_steps, float dt, int stages, const float* action, int action_body,
               cotix_stream_t stream) {
  return step_impl(scene, dyn, keys, err, geom, geom_stride, B, n_steps, dt, stages, action, action_body, nullptr,
                   nullptr, nullptr, nullptr, stream);
}

int cotix_step_autoreset(cotix_scene* scene, float* dyn, uint32_t* keys, uint32_t* err, const float* geom,
                         int geom_stride, int B, int n_steps, float dt, int stages, const float* dyn_reset,
                         uint32_t* resets, cotix_stream_t stream) {
  if (!dyn_reset) return fail("dyn_reset required");
  return step_impl(scene, dyn, keys, err, geom, geom_stride, B, n_steps, dt, stages, nullptr, 0, dyn_reset, resets,
                   nullptr, nullptr, stream);
}

int cotix_step_ex(cotix_scene* scene, float* dyn, uint32_t* keys, uint32_t* err, const float* geom, int geom_stride,
                  int B, int n_steps, float dt, int stages, const float* action, int action_body,
                  const float* dyn_reset, uint32_t* resets, int32_t* chosen, int32_t* cells, cotix_stream_t stream) {
  return step_impl(scene, dyn, keys, err, geom, geom_stride, B, n_steps, dt, stages, action, action_body, dyn_reset,
                   resets, chosen, cells, stream);
}

int cotix_rollout_tape_words(const cotix_scene* scene) {
  if (!scene) return fail("null scene");
  return cxk::tape_words(scene->host.nb, scene->host.nc, scene->host.poly);
}

int cotix_rollout(cotix_scene* scene, float* dyn, uint32_t* keys, uint32_t* err, const float* geom, int geom_stride,
                  int B, int n_steps, float dt, int stages, const float* action, int action_body,
                  const float* ret_weights, float* ret, float* saved_dyn, uint32_t* saved_keys, cotix_stream_t stream) {
  return cotix_rollout_ex(scene, dyn, keys, err, geom, geom_stride, B, n_steps, dt, stages, action, action_body,
                          ret_weights, ret, saved_dyn, saved_keys, nullptr, stream);
}

int cotix_rollout_ex(cotix_scene* scene, float* dyn, uint32_t* keys, uint32_t* err, const float* geom,
                     int geom_stride, int B, int n_steps, float dt, int stages, const float* action, int action_body,
                     const float* ret_weights, float* ret, float* saved_dyn, uint32_t* saved_keys, uint32_t* tape,
                     cotix_stream_t stream) {
  if (check_step_args(scene, dyn, keys, geom, geom_stride, B, n_steps, stages, action, action_body)) return -1;
  if (!err || !ret_weights || !ret || !saved_dyn || !saved_keys) return fail("null argument");
  if (B == 0 || n_steps == 0) return 0;
  cxk::KArgs ka{};
  ka.dyn = dyn;
  ka.keys = keys;
  ka.err = err;
  ka.geom = geom;
  ka.gstride = geom_stride;
  ka.B = B;
  ka.n_steps = n_steps;
  ka.dt = dt;
  ka.stages = stages;
  ka.action = action;
  ka.action_body = action_body;
  ka.save_dyn = saved_dyn;
  ka.save_keys = saved_keys;
  ka.tape = tape;
  ka.tw = cxk::tape_words(scene->host.nb, scene->host.nc, scene->host.poly);
  ka.ret = ret;
  for (int k = 0; k < scene->host.nb * 6; ++k) ka.ret_w[k] = ret_weights[k];
  return launch(scene, ka, 1, stream);
}

int cotix_rollout_backward(cotix_scene* scene, const float* saved_dyn, const uint32_t* saved_keys, const float* geom,
                           int geom_stride, int B, int n_steps, float dt, int stages, const float* action,
                           int action_body, const float* ret_weights, float* grad_action, float* grad_dyn0,
                           cotix_stream_t stream) {
  return cotix_rollout_backward_ex(scene, saved_dyn, saved_keys, nullptr, geom, geom_stride, B, n_steps, dt, stages,
                                   action, action_body, ret_weights, grad_action, grad_dyn0, stream);
}

int cotix_rollout_backward_ex(cotix_scene* scene, const float* saved_dyn, const uint32_t* saved_keys,
                              const uint32_t* tape, const float* geom, int geom_stride, int B, int n_steps, float dt,
                              int stages, const float* action, int action_body, const float* ret_weights,
                              float* grad_action, float* grad_dyn0, cotix_stream_t stream) {
  if (check_step_args(scene, saved_dyn, saved_keys, geom, geom_stride, B, n_steps, stages, action, action_body))
    return -1;
  if (!ret_weights) return fail("null argument");
  if (grad_action && !action) return fail("grad_action needs the action the rollout was run with");
  if ((scene->fnset & cxk::FNS_CIRCLE_POLY) && scene->host.gjk_steps > cx::CP_GJK_MAX)
    return fail("differentiable rollout: circle x polygon gradients record every GJK point: gjk_max_steps <= " +
                std::to_string(cx::CP_GJK_MAX));
  if ((stages & COTIX_STAGE_LUNAR) && !(scene->fnset & ~FNS_ANALYTIC))
    return fail("differentiable rollout: the LunarLander joint stage needs the polygon program (a polygon scene)");
  if (B == 0 || n_steps == 0) return 0;
  cxk::KArgs ka{};
  ka.dyn = nullptr;
  ka.keys = nullptr;
  ka.err = nullptr;
  ka.geom = geom;
  ka.gstride = geom_stride;
  ka.B = B;
  ka.n_steps = n_steps;
  ka.dt = dt;
  // the re-play without the broadphase (an exact filter: the same contacts);
  // its per-edge words overlay the adjoint (cxk::layout)
  ka.stages = stages & ~COTIX_STAGE_BROADPHASE;
  ka.action = action;
  ka.action_body = action_body;
  ka.save_dyn = const_cast<float*>(saved_dyn);
  ka.save_keys = const_cast<uint32_t*>(saved_keys);
  ka.tape = const_cast<uint32_t*>(tape);
  ka.tw = cxk::tape_words(scene->host.nb, scene->host.nc, scene->host.poly);
  ka.grad_action = grad_action;
  ka.grad_dyn = grad_dyn0;
  for (int k = 0; k < scene->host.nb * 6; ++k) ka.ret_w[k] = ret_weights[k];
  return launch(scene, ka, tape ? 4 : 2, stream);
}

int cotix_physics_euler(float* dyn, int n_bodies, int B, float dt, cotix_stream_t stream) {
  if (!dyn) return fail("null argument");
  long long n = (long long)n_bodies * B;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(euler_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), dyn, n_bodies, B, dt);
  return hip_check(hipGetLastError(), "euler_kernel launch");
}

int cotix_collider_resolve(cotix_scene* scene, float* dyn, const uint32_t* keys, uint32_t* err, const float* geom,
                           int geom_stride, int B, cotix_stream_t stream) {
  // the fused kernel with the collider stage only; keys are read, not advanced
  return cotix_step(scene, dyn, const_cast<uint32_t*>(keys), err, geom, geom_stride, B, 1, 0.0f,
                    COTIX_STAGE_COLLIDER, nullptr, 0, stream);
}

int cotix_lunar_constraints(float* dyn, int B, cotix_stream_t stream) {
  if (!dyn) return fail("null argument");
  if (B <= 0) return 0;
  // LunarLander body parameters (cotix/_lunar_lander.py:78-105)
  cx::Params p0{30.0f, 30.0f, 1.0f, 0.1f}, p1{1.0f, 1.0f, 1.0f, 0.1f}, p2{1.0f, 1.0f, 1.0f, 0.1f};
  hipLaunchKernelGGL(lunar_kernel, dim3((B + 255) / 256), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), dyn, B,
                     p0, p1, p2);
  return hip_check(hipGetLastError(), "lunar_kernel launch");
}

static int body_parts(const cotix_scene* scene, int body, BodyParts* bp) {
  const SceneDev& s = scene->host;
  if (body < 0 || body >= s.nb) return fail("body index out of range");
  bp->body = body;
  bp->n = 0;
  for (int p = 0; p < s.np; ++p) {
    if ((int)s.hot[s.o_pbody + p] != body) continue;
    if (bp->n >= MAXBP) return fail("more than 16 parts in a body");
    bp->kind[bp->n] = (int)s.hot[s.o_pkind + p];
    bp->nv[bp->n] = (int)s.hot[s.o_pn + p];
    bp->goff[bp->n] = (int)s.hot[s.o_pgoff + p];
    ++bp->n;
  }
  if (bp->n == 0) return fail("body has no parts");
  return 0;
}

int cotix_body_penetration(const cotix_scene* scene, const float* dyn, const float* geom, int geom_stride, int B,
                           int body_a, int body_b, int* collides, float* pen, cotix_stream_t stream) {
  if (!scene || !dyn || !geom || !collides || !pen) return fail("null argument");
  if (B <= 0) return B == 0 ? 0 : fail("negative size");
  BodyParts pa, pb;
  if (body_parts(scene, body_a, &pa) || body_parts(scene, body_b, &pb)) return -1;
  hipLaunchKernelGGL(body_pen_kernel, dim3((B + 63) / 64), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), dyn,
                     B, geom, geom_stride, pa, pb, cxk::narrow_of(scene->host), collides, pen);
  return hip_check(hipGetLastError(), "body_pen_kernel launch");
}

int cotix_body_aabb(const cotix_scene* scene, const float* dyn, const float* geom, int geom_stride, int B, int body,
                    float* aabb, uint32_t* err, cotix_stream_t stream) {
  if (!scene || !dyn || !geom || !aabb) return fail("null argument");
  if (B <= 0) return B == 0 ? 0 : fail("negative size");
  BodyParts pa;
  if (body_parts(scene, body, &pa)) return -1;
  hipLaunchKernelGGL(body_aabb_kernel, dim3((B + 63) / 64), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), dyn,
                     B, geom, geom_stride, pa, aabb, err);
  return hip_check(hipGetLastError(), "body_aabb_kernel launch");
}

static int scene_parts(const cotix_scene* scene, cxk::SceneParts* sp) {
  const SceneDev& s = scene->host;
  if (s.np > cxk::MAXRP) return fail("more than 32 parts in the scene");
  sp->np = s.np;
  int off = 0;
  for (int p = 0; p < s.np; ++p) {
    sp->body[p] = (int)s.hot[s.o_pbody + p];
    sp->kind[p] = (int)s.hot[s.o_pkind + p];
    sp->nv[p] = (int)s.hot[s.o_pn + p];
    sp->goff[p] = (int)s.hot[s.o_pgoff + p];
    sp->poff[p] = off;
    off += cxk::render_prims(sp->kind[p], sp->nv[p]);
  }
  return off;
}

int cotix_render_count(const cotix_scene* scene) {
  if (!scene) return fail("null scene");
  cxk::SceneParts sp;
  return scene_parts(scene, &sp);
}

int cotix_render(const cotix_scene* scene, const float* dyn, const float* geom, int geom_stride, int B, float* prims,
                 cotix_stream_t stream) {
  if (!scene || !dyn || !geom || !prims) return fail("null argument");
  if (geom_stride != 0 && geom_stride < scene->host.G) return fail("geom_stride smaller than the scene geometry");
  if (B <= 0) return B == 0 ? 0 : fail("negative size");
  cxk::SceneParts sp;
  const int nprim = scene_parts(scene, &sp);
  if (nprim < 0) return -1;
  const long long n = (long long)B * sp.np;
  hipLaunchKernelGGL(render_kernel, dim3((unsigned)((n + 127) / 128)), dim3(128), 0,
                     reinterpret_cast<hipStream_t>(stream), dyn, B, geom, geom_stride, sp, nprim, prims);
  return hip_check(hipGetLastError(), "render_kernel launch");
}

int cotix_observe(const float* dyn, int n_bodies, int B, float* obs, cotix_stream_t stream) {
  if (!dyn || !obs) return fail("null argument");
  if (n_bodies < 0 || B < 0) return fail("negative size");
  const long long n = (long long)n_bodies * 6 * B;
  if (n == 0) return 0;
  hipLaunchKernelGGL(observe_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), dyn, n_bodies * 6, B, obs);
  return hip_check(hipGetLastError(), "observe_kernel launch");
}

int cotix_check_state(const float* dyn, int n_bodies, int B, uint32_t* err, cotix_stream_t stream) {
  if (!dyn || !err) return fail("null argument");
  if (n_bodies < 0 || B < 0) return fail("negative size");
  if (B == 0) return 0;
  hipLaunchKernelGGL(check_state_kernel, dim3((B + 255) / 256), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     dyn, n_bodies, B, err);
  return hip_check(hipGetLastError(), "check_state_kernel launch");
}

// a parameter block (NULL: the defaults), validated, as the narrow phase's / resolution's arguments
static int op_params(const cotix_params* params, cotix_params* out) {
  *out = params ? *params : cxk::default_params();
  return cxk::check_params(*out, g_err);
}
static cx::NarrowParams narrow_params(const cotix_params& p) {
  return cx::NarrowParams{cx::gjk_d0(p.prng_layout == COTIX_PRNG_PARTITIONABLE), p.gjk_max_steps, p.epa_max_iters,
                          p.epa_circle_iters, p.epa_body_iters};
}

int cotix_contacts_ex(int fn, int n, const float* a, const float* b, float* out, uint32_t* err,
                      const cotix_params* params, cotix_stream_t stream) {
  if (!a || !b || !out) return fail("null argument");
  if (fn < 0 || fn > 5) return fail("unknown contact function");
  cotix_params p;
  if (op_params(params, &p)) return -1;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(contacts_kernel, dim3((n + 127) / 128), dim3(128), 0, reinterpret_cast<hipStream_t>(stream), fn,
                     n, a, b, out, err, narrow_params(p));
  return hip_check(hipGetLastError(), "contacts_kernel launch");
}

int cotix_contacts(int fn, int n, const float* a, const float* b, float* out, uint32_t* err, cotix_stream_t stream) {
  return cotix_contacts_ex(fn, n, a, b, out, err, nullptr, stream);
}

int cotix_resolve_ex(int n, float* dyn1, const float* par1, float* dyn2, const float* par2, const float* contact,
                     const cotix_params* params, cotix_stream_t stream) {
  if (!dyn1 || !dyn2 || !par1 || !par2 || !contact) return fail("null argument");
  cotix_params p;
  if (op_params(params, &p)) return -1;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(resolve_kernel, dim3((n + 255) / 256), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), n,
                     dyn1, par1, dyn2, par2, contact, cx::Baum{p.baumgarte, p.baumgarte_dt});
  return hip_check(hipGetLastError(), "resolve_kernel launch");
}

int cotix_resolve(int n, float* dyn1, const float* par1, float* dyn2, const float* par2, const float* contact,
                  cotix_stream_t stream) {
  return cotix_resolve_ex(n, dyn1, par1, dyn2, par2, contact, nullptr, stream);
}

int cotix_gjk_ex(int n, const float* a, const float* b, const float* initial_direction, const uint32_t* keys,
                 int32_t* hit, float* simplex, const cotix_params* params, cotix_stream_t stream) {
  if (!a || !b || !hit || !simplex) return fail("null argument");
  cotix_params p;
  if (op_params(params, &p)) return -1;
  if (n <= 0) return n == 0 ? 0 : fail("negative size");
  hipLaunchKernelGGL(gjk_kernel, dim3((n + 127) / 128), dim3(128), 0, reinterpret_cast<hipStream_t>(stream), n, a, b,
                     hit, simplex, narrow_params(p), initial_direction, keys, p.prng_layout);
  return hip_check(hipGetLastError(), "gjk_kernel launch");
}

int cotix_gjk(int n, const float* a, const float* b, int32_t* hit, float* simplex, const cotix_params* params,
              cotix_stream_t stream) {
  return cotix_gjk_ex(n, a, b, nullptr, nullptr, hit, simplex, params, stream);
}

int cotix_epa(int n, const float* a, const float* b, const float* simplex, int iters, float* pen,
              cotix_stream_t stream) {
  if (!a || !b || !simplex || !pen) return fail("null argument");
  if (iters < 3 || iters > 128) return fail("iters outside 3..128 (cotix/_collisions.py:130-135)");
  if (n <= 0) return n == 0 ? 0 : fail("negative size");
  hipLaunchKernelGGL(epa_kernel, dim3((n + 63) / 64), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), n, a, b,
                     simplex, iters, pen);
  return hip_check(hipGetLastError(), "epa_kernel launch");
}

int cotix_threefry2x32(const uint32_t* keys, const uint32_t* ctr, uint32_t* out, int n, cotix_stream_t stream) {
  if (!keys || !ctr || !out) return fail("null argument");
  if (n <= 0) return 0;
  hipLaunchKernelGGL(threefry_kernel, dim3((n + 255) / 256), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), keys,
                     ctr, out, n);
  return hip_check(hipGetLastError(), "threefry_kernel launch");
}

static int check_layout(int layout) {
  if (layout != COTIX_PRNG_LEGACY && layout != COTIX_PRNG_PARTITIONABLE) return fail("unknown PRNG layout");
  return 0;
}

int cotix_random_split_ex(const uint32_t* keys, int n, int num, int layout, uint32_t* out, cotix_stream_t stream) {
  if (!keys || !out) return fail("null argument");
  if (num <= 0) return fail("num must be positive");
  if (check_layout(layout)) return -1;
  long long t = (long long)n * num;
  if (t <= 0) return 0;
  hipLaunchKernelGGL(split_kernel, dim3((unsigned)((t + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), keys, n, num, out, layout);
  return hip_check(hipGetLastError(), "split_kernel launch");
}

int cotix_random_split(const uint32_t* keys, int n, int num, uint32_t* out, cotix_stream_t stream) {
  return cotix_random_split_ex(keys, n, num, COTIX_PRNG_LEGACY, out, stream);
}

int cotix_random_uniform_ex(const uint32_t* keys, int n, int count, float lo, float hi, int layout, float* out,
                            cotix_stream_t stream) {
  if (!keys || !out) return fail("null argument");
  if (count <= 0) return fail("count must be positive");
  if (check_layout(layout)) return -1;
  long long t = (long long)n * count;
  if (t <= 0) return 0;
  hipLaunchKernelGGL(uniform_kernel, dim3((unsigned)((t + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), keys, n, count, lo, hi, out, layout);
  return hip_check(hipGetLastError(), "uniform_kernel launch");
}

int cotix_random_uniform(const uint32_t* keys, int n, int count, float lo, float hi, float* out,
                         cotix_stream_t stream) {
  return cotix_random_uniform_ex(keys, n, count, lo, hi, COTIX_PRNG_LEGACY, out, stream);
}

int cotix_order_clockwise(float* xy, int n, int nverts, cotix_stream_t stream) {
  if (!xy) return fail("null argument");
  if (nverts < 1 || nverts > cx::MAXV) return fail("nverts must be 1..8");
  if (n <= 0) return 0;
  hipLaunchKernelGGL(order_cw_kernel, dim3((n + 255) / 256), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), xy,
                     n, nverts);
  return hip_check(hipGetLastError(), "order_cw_kernel launch");
}

}  // extern "C"
