// cotix_kernel.h -- the fused step as phase functions + the scene tables.
//
// Shared by the gfx950 kernel (cotix_step.hip) and by the CPU emulation
// harness of the tests (tests/emu: every phase run for all lanes of a wave in
// turn, under AddressSanitizer).
//
// Design (DESIGN.md "Kernels").  A workgroup is WPB independent waves; each
// wave owns a tile of EW environments for all n_steps of a launch and syncs
// only with itself (wave-local ordering, no workgroup barrier per phase), so
// the serial phases of one wave overlap the other waves' work on the SIMD.
// The tile's state lives in LDS laid out [word][env] (env fastest), next to
// a per-workgroup LDS copy of the scene's hot tables.  Every phase is spread
// over the wave's 64 lanes as (item, env) pairs with env fastest:
//   A  Euler (+gravity, +action); per-env key chain     (item = body)
//   T  part transforms + order_clockwise                  (item = part)
//   B  distinct narrowphase contacts (+error bits)        (item = contact)
//   C  per-cell "last passing candidate" RNG scan         (item = cell)
//   D  per-body contact choice (jr.choice)                (item = body)
//   E  sequential resolution, LunarLander joints, key     (item = env)
// Phase C replaces the reference's sequential N2 x N1 scatter scan
// (cotix/_colliders.py:208-268) by an exact equivalent: for every cell
// (i, j) only the LAST candidate (in scan order) whose contact is non-NaN
// and whose bernoulli passes determines all_contacts[i, j], so each cell is
// scanned backwards and stops at the first pass; a cell whose distinct
// contacts are all NaN is skipped outright, and duplicate contacts (the same
// part pair repeated in the candidate lists) are evaluated once.
#pragma once
#include "../../include/cotix_amd.h"
#include "cotix_device.h"
#include "cotix_grad.h"

namespace cxk {

constexpr int MAXB = 16, MAXP = 32, MAXC = 256, MAXL = 128, MAXT = 13, MAXCAND = 16384;
constexpr int MAXHOT = 24576;
constexpr int WAVE = 64;

// workload counters of the host emulation (tools/collider_stats.py); no-ops
// in every other build
#ifdef COTIX_STATS
struct Stats {
  unsigned long long wave_steps, active_items, rounds, resolutions, f_items, b_items, draws, valid_draws, r1_left, lvl_env, lvl_wave, e1_slots;
  unsigned long long valid_cands, fit64;  // valid candidates of the active items; wave-steps where they fit 64 lanes
  unsigned long long bp_cand, bp_guard_fail;  // broadphase: pairs past the gap test; of them, not certified by bp_guard
  unsigned long long epa_runs;                // polygon contacts whose GJK hit (EPA ran, not a self pair)
};
inline Stats g_stats{};
#define CXK_STAT(f, v) (cxk::g_stats.f += (unsigned long long)(v))
#else
#define CXK_STAT(f, v) ((void)0)
#endif
// sub-phase cycle timers of the phase-timing build (tools/phase_prof.py):
// CXK_SUB_T0 / CXK_SUB_T1(k) add the wave's clock delta to slot k (ad-hoc
// instrumentation; slot 4 is cotix_device.h's CX_DSUB_T0 / CX_DSUB_T1)
#if defined(COTIX_PHASE_PROF) && (defined(__HIP__) || defined(__HIPCC__))
static __device__ unsigned long long g_sub_cycles[8];
#define CXK_SUB_T0 const unsigned long long cxk_sub_t0 = clock64()
#define CXK_SUB_T1(k, lane)                                                                       \
  do {                                                                                            \
    const unsigned long long dt_ = clock64() - cxk_sub_t0;                                        \
    if ((lane) == __builtin_amdgcn_readfirstlane(lane)) atomicAdd(&cxk::g_sub_cycles[k], dt_); \
  } while (0)
#else
#define CXK_SUB_T0 ((void)0)
#define CXK_SUB_T1(k, lane) ((void)0)
#endif

// a lambda that must be inlined (a call would put every local it captures by
// reference into scratch memory)
#define CXK_INLINE_LAMBDA __attribute__((always_inline))

// phase-cost experiments of the tooling build (-DCOTIX_TOOLING, KArgs::dbg_skip
// from COTIX_DEBUG_SKIP) skip whole phases; the release library compiles every
// skip out, so no environment variable can change what it computes
#ifdef COTIX_TOOLING
#define CXK_SKIP(a, bit) (((a).dbg_skip & (bit)) != 0)
#else
#define CXK_SKIP(a, bit) false
#endif

// Scene tables.  Everything the step reads per item is packed into hot[]
// (word offsets below) and copied to LDS once per launch.
// the scalar header (offsets, counts) travels in the kernel arguments, so
// phases read it from registers, never from global memory
//
// 16-bit fields: the generic kernel keeps the header in scalar registers for
// the whole launch (every table offset is < MAXHOT, every count < 4096), so
// packing halves its register footprint.  The fields, in declaration order:
//   nb, np, nc, nl, nt, G, W, ncand: bodies, parts, contacts, cells, types,
//     geom / world floats, candidates
//   d0x, d0y: GJK start direction (constant)
//   o_*: word offsets of the hot tables; o_cdesc: per contact 2 words (world
//     offsets of both parts, fn, kinds | vertex counts, part ids); o_cmask: per
//     cell nmw words (bitmask of the cell's distinct contacts); o_cbody: per
//     contact the bodies of its two parts (body_a | body_b << 8); o_vit: per
//     polygon vertex 2 words (part, vertex, count, first item, body | offsets)
//   nmw: contact-mask words = ceil(nc / 32)
//   poly: 1 -- the scene has polygon-polygon / AABB-polygon contacts
//     (deferred contact points)
//   rcp_all: 1 -- every mass and inertia has an exact reciprocal (o_rcp):
//     resolutions multiply; rcp_mask: bit b -- body b's do (bodies < 32)
//   fnset: FNS_* bits of the contact functions the scene uses
//   nhot: hot-table words; nvt: polygon vertices over all parts (phase T's
//     vertex items); maxv: the most vertices of any polygon part (0: none);
//     pminv: max over polygon pairs of the smaller edge count (AABB: 2) --
//     the broadphase guard's loop bounds
//   epar: 0 -- the bodies' (mass, inertia, elasticity, friction) are the
//     scene table's (o_par); else 1 + the word offset, in each env's local
//     geometry (the tile's geo words), of its own 4 words per body
//     (COTIX_SCENE_PER_ENV_BODY_PARAMS; rcp_all and rcp_mask are then 0)
//   prng .. pc: cotix_params (include/cotix_amd.h) -- PRNG layout (1:
//     partitionable), GJK steps, EPA iteration cap / circle x polygon /
//     body-level iterations, Baumgarte factor and divisor, the candidates'
//     bernoulli p
// One list (CXK_HDR_FIELDS) declares them, compares headers (hdr_equal) and
// prints the specializations' constant headers (cotix_spec_hdrs.h).
#define CXK_HDR_FIELDS(X)                                                                                          \
  X(uint16_t, nb) X(uint16_t, np) X(uint16_t, nc) X(uint16_t, nl) X(uint16_t, nt) X(uint16_t, G) X(uint16_t, W)   \
  X(uint16_t, ncand) X(float, d0x) X(float, d0y) X(uint16_t, o_par) X(uint16_t, o_rcp) X(uint16_t, o_pbody)     \
  X(uint16_t, o_pkind) X(uint16_t, o_pn) X(uint16_t, o_pgoff) X(uint16_t, o_pwoff) X(uint16_t, o_cpa)           \
  X(uint16_t, o_cpb) X(uint16_t, o_cfn) X(uint16_t, o_ci) X(uint16_t, o_cj) X(uint16_t, o_cbeg) X(uint16_t, o_ccnt) \
  X(uint16_t, o_tn1) X(uint16_t, o_tn2) X(uint16_t, o_cand) X(uint16_t, o_cdesc) X(uint16_t, o_cmask)          \
  X(uint16_t, o_cbody) X(uint16_t, nmw) X(uint16_t, poly) X(uint16_t, rcp_all) X(uint16_t, fnset)               \
  X(uint16_t, nhot) X(uint16_t, nvt) X(uint16_t, o_vit) X(uint32_t, rcp_mask) X(uint16_t, maxv)                 \
  X(uint16_t, pminv) X(uint16_t, prng) X(uint16_t, gjk_steps) X(uint16_t, epa_cap) X(uint16_t, epa_cp)          \
  X(uint16_t, epa_body) X(float, baum) X(float, baum_dt) X(float, pc) X(uint16_t, epar)
struct SceneHdr {
#define CXK_HDR_DECL(T, n) T n;
  CXK_HDR_FIELDS(CXK_HDR_DECL)
#undef CXK_HDR_DECL
};
// field bits (floats by their bit pattern: -0.0 != 0.0 here)
CX_HD uint32_t hdr_bits(uint16_t v) { return v; }
CX_HD uint32_t hdr_bits(uint32_t v) { return v; }
CX_HD uint32_t hdr_bits(float v) { return __builtin_bit_cast(uint32_t, v); }
CX_HD bool hdr_equal(const SceneHdr& a, const SceneHdr& b) {
  bool eq = true;
#define CXK_HDR_EQ(T, n) eq = eq && hdr_bits(a.n) == hdr_bits(b.n);
  CXK_HDR_FIELDS(CXK_HDR_EQ)
#undef CXK_HDR_EQ
  return eq;
}
CX_HD cx::NarrowParams narrow_of(const SceneHdr& h) {
  return cx::NarrowParams{cx::v2{h.d0x, h.d0y}, (int)h.gjk_steps, (int)h.epa_cap, (int)h.epa_cp, (int)h.epa_body};
}
CX_HD cx::Baum baum_of(const SceneHdr& h) { return cx::Baum{h.baum, h.baum_dt}; }
struct SceneDev : SceneHdr {
  uint32_t hot[MAXHOT];
};

// Scene specializations of the step kernel.  The phases are generic over the
// scene (counts, table offsets and parameters in the header); for the two
// reference scenes, under the default constants in either PRNG layout (and
// the box world's structure, legacy layout), the launcher picks an
// instantiation whose header is a compile-time constant --
// every per-item loop has a known trip count (no exec-mask loop control, no
// index division), the tile layout and every table address fold to
// immediates, the parameters to literals, and no scalar register holds the
// header.  The constant headers are the scene compiler's output for
// cotix/_robocup.py and cotix/_lunar_lander.py (cotix_spec_hdrs.h, written by
// tools/gen_spec_hdrs.py and checked against the compiler by
// tests/test_emu_cpu.py); spec_of() admits a scene only when its whole header
// is bit-identical.
enum : int {
  SPEC_GENERIC = 0,
  SPEC_ROBOCUP = 1,
  SPEC_LUNAR = 2,
  SPEC_ROBOCUP_PART = 3,
  SPEC_LUNAR_PART = 4,
  SPEC_BOX = 5,  // the box world's structure (3 AABB walls, 4 circles): the finite scene of the secondary figures
  SPEC_N = 6
};
}  // namespace cxk
#include "cotix_spec_hdrs.h"  // cxk::SPEC_HDRS[SPEC_N]
namespace cxk {
CX_HD int spec_of(const SceneHdr& h) {
  for (int s = 1; s < SPEC_N; ++s)
    if (hdr_equal(h, SPEC_HDRS[s])) return s;
  return SPEC_GENERIC;
}
// the header a SPEC instantiation runs with: the specialization's constant
// (SPEC > 0 only for a header that spec_of() mapped to SPEC)
template <int SPEC>
CX_HD SceneHdr spec_hdr(const SceneHdr& h) {
  if constexpr (SPEC != SPEC_GENERIC) {
    constexpr SceneHdr k = SPEC_HDRS[SPEC];
    return k;
  } else {
    return h;
  }
}

// device judge and control of cotix_eval (include/cotix_amd.h: cotix_judge,
// cotix_control), compacted by the host: the nonzero weights as (word, w)
// terms in word order -- the sums run over them in that order, starting from
// the first term
constexpr int JT = 16, JR = 4, JRT = 8;
struct JudgeArgs {
  int on, nrate, nend, nreg, doe;
  uint8_t rate_k[JT], end_k[JT];
  float rate_w[JT], end_w[JT];
  int rbody[JR];
  float lo[JR][6], hi[JR][6], rrew[JR];
  // the reward rate's pieces (cotix_judge rate regions): region r over body
  // prbody[r], npr[r] terms (k, w), then the bias when hasb[r]
  int nrr, prbody[JR], npr[JR], hasb[JR];
  float prlo[JR][6], prhi[JR][6];
  uint8_t pr_k[JR][JRT];
  float pr_w[JR][JRT], pr_b[JR];
};
struct CtlArgs {
  int on, body, sat;
  float gain[2][6], target[2][6], bias[2], lo[2], hi[2];
};

// kernel arguments (passed by value)
struct KArgs {
  const SceneDev* sc;
  SceneHdr sh;         // *sc's header (by value: kernel-argument registers)
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
#ifdef COTIX_TOOLING
  int dbg_skip;            // tooling builds only: skip phase T=1, B=2, C=4, D=8, A's key splits=16, E=32, GJK/EPA=64
#endif
  // collider trace (cotix_step_ex; null = off): per step, body and env the
  // chosen partner j* (cotix/_colliders.py:274-295), and per cell (i, j) the
  // reference-scan candidate whose contact all_contacts[i, j] holds (:208-268)
  int32_t* trace_chosen;   // [n_steps][nb][B]
  int32_t* trace_cells;    // [n_steps][nb][nb][B]: i1 | i2 << 9 | type << 18, -1 = empty cell
  // differentiable rollout (cotix_rollout / cotix_rollout_backward)
  float* save_dyn;         // [n_steps][B/4][nb*6][4] (row_at): state before each step, or null
  uint32_t* save_keys;     // [n_steps][B][2]
  float* ret;              // [B] += sum_t sum_k ret_w[k] * state_{t+1}[k] (terms with ret_w[k] == 0 skipped)
  float* grad_action;      // backward: [n_steps][B][2] d ret / d action
  float* grad_dyn;         // backward: [nb*6][B] d ret / d initial state, or null
  float ret_w[MAXB * 6];
  // the rollout's decision tape (cotix_rollout_ex / cotix_rollout_backward_ex;
  // null = off): [n_steps][B/4][tw][4] words (row_at), written by the
  // forward, read by the backward instead of re-playing the collider
  // (tape_words below)
  uint32_t* tape;
  int tw;
  // cotix_eval (AbstractEnvironment.eval, cotix/_envs.py:37-132, fused):
  int reset_mode;          // 1: restart on error bits after a step (dyn_reset); 2: restart envs finished at entry
  int action_held;         // 1: action is [B][2], the same impulse every step (a held control signal)
  float* obs;              // [B][nb][6] final observation, or null
  float* reward;           // [B] in/out: the eval carry's reward (judge on)
  uint32_t* finished;      // [B] in/out: the eval carry's `finished` flag (judge on)
  int nfe_len;             // env-steps per NFE (WFE_scale); n_steps is a multiple of it (judge on)
  JudgeArgs judge;         // device AbstractJudge (judge.on == 0: off)
  CtlArgs ctl;             // device AbstractControl (ctl.on == 0: off)
};

// The rollout's saved rows (save_dyn: nb*6 state words per env-step; tape:
// tw words) in env blocks of 4: row r of step s, env g at
// [((s * ceil(B/4) + g/4) * rows + r) * 4 + g%4].  A wave of 4 envs saves and
// restores its rows as one contiguous run of 16-byte pieces (a [row][B] layout
// puts every row of the wave in a cache line of its own)
CX_HD size_t row_at(int B, int rows, int s, int r, int g) {
  return (((size_t)s * (size_t)((B + 3) >> 2) + (size_t)(g >> 2)) * (size_t)rows + (size_t)r) * 4u + (size_t)(g & 3);
}
// The rollout's decision tape, per env-step (word w of step s, env g at
// tape[row_at(B, tw, s, w, g)]):
//   5 i        body i's resolution (cotix/_colliders.py:310-336): its partner
//              j* | the distinct contact id of cell (i, j*) << 8, or RP_NONE
//              when the body resolves nothing this step
//   5 i + 1..4 that contact (pen.x, pen.y, cp.x, cp.y) -- written only for a
//              resolution
//   5 nb + 4 c (polygon scenes) EPA's final edge (e0, e1) of distinct contact
//              c, written by phase B when EPA ran for it
//   5 nb + 7 i (analytic scenes) the resolution's record: whether its
//              impulse was applied, then the pre-resolution v / w of bodies
//              i and j (REC_W words, the sequential pass of phase E1) --
//              written only for a resolution
// Every value is the forward's own; the backward (MODE 4) restores them
// instead of re-running the key splits, the narrowphase, the RNG scan and the
// choice (and, analytic scenes, the sequential resolution pass), and the VJP
// of a GJK/EPA contact starts from the recorded edge.
constexpr int REC_W = 7;  // per resolution: applied flag, v/w of body i, v/w of body j (pre-resolution)
CX_HD int tape_words(int nb, int nc, int poly) { return 5 * nb + (poly ? 4 * nc : REC_W * nb); }
// the tape carries the resolutions' records (analytic scenes): the forward's
// phase E1 records them (ph_E TREC), the backward skips its phase E
CX_HD bool tape_rec(const SceneHdr& sh) { return sh.poly == 0; }
// the backward's tape words in registers (tape_fetch): per (body, env) item
// its resolution word + contact, and the recorded EPA edge
constexpr int TQ = (MAXB * 8 + WAVE - 1) / WAVE;  // items per lane: nb * EW over 64 lanes (EW <= 8)
// 16 bytes: 4 envs' words of one row (rows_out, restore_rows_fetch)
struct alignas(16) U4 {
  uint32_t v[4];
};
struct TapeRegs {
  uint32_t d[TQ][5];
  uint32_t x[TQ][REC_W];  // polygon scenes: the EPA edge (4 float words); analytic: the resolution's record
};

// per-wave tile layout (words, each x EW envs)
struct Lay {
  int dyn, world, con, m, ch, key, sk0, skt, err, nres, ret, adj, rec, vm, rst, geo, rp, kw, kww, rflag, pose, pcv, pbox,
      pedge, jfin, jal, jr, jpr, jk, je, jsn, S;
};
// key window: the per-step keys of KWIN consecutive steps, precomputed
// together (phase K) -- the collider keys depend on the key chain only, never
// on the physics.  Slot s (KW words): sk0[2], skt[2*nt], then choice uniform[nb].
constexpr int KWIN = 16;
// per resolution (phase E0 -> E1): partner body (or RP_NONE), cx::ResPre, partner mass/inertia
enum : int { RP_J, RP_NX, RP_NY, RP_R1X, RP_R1Y, RP_R2X, RP_R2Y, RP_PX, RP_PY, RP_DEN, RP_PT, RP_NE, RP_MU, RP_MJ, RP_IJ,
             RP_QMJ, RP_QIJ, RP_W };
constexpr uint32_t RP_NONE = 0xFFFFFFFFu;
// PE: words of the broadphase guard's per-edge pseudo-angles (polygon scenes: W / 2, else 0)
CX_HD Lay layout(int nb, int np, int W, int nc, int nt, int G, int PE) {
  Lay L;
  L.dyn = 0;
  L.world = L.dyn + nb * 6;
  L.con = L.world + W + 2 * cx::MAXV;  // slack: shape fetches read 2*MAXV words
  L.m = L.con + nc * 4;  // all_contacts cells: the winning candidate word (o_cand format), ~0 = empty
  L.ch = L.m + nb * nb;
  L.key = L.ch + nb;
  L.sk0 = L.key + 2;
  L.skt = L.sk0 + 2;
  L.err = L.skt + 2 * nt;
  L.nres = L.err + 1;
  L.ret = L.nres + 1;
  L.adj = L.ret + 1;
  L.rec = L.adj + nb * 6;
  L.vm = L.rec + nb * REC_W;        // bit c: contact c has a contact point this step
  L.rst = L.vm + (nc + 31) / 32;    // restart state (autoreset), staged once per launch
  L.geo = L.rst + nb * 6;           // local part geometry (per env), staged once per launch
  L.rp = L.geo + G;                 // resolution operands (E0 -> E1)
  L.kww = 2 + 2 * nt + nb;          // key window slot words
  L.kw = L.rp + nb * RP_W;
  L.rflag = L.kw + KWIN * L.kww;    // this step restarts the env (autoreset)
  L.pose = L.rflag + 1;             // per body: the pose (px, py, angle bits) its world parts were built from
  L.pcv = L.pose + 3 * nb;          // bit b: body b's pose entry is valid (cleared at every launch start)
  L.pbox = L.pcv + 1;               // per part: world AABB (lo.x, lo.y, up.x, up.y), polygon scenes (broadphase)
  // cotix_eval's carry (judge on): finished, already_premature_outted, reward,
  // the premature-out reward, key and err; the premature-out state itself is
  // kept in rst (free in eval: its restarts are taken at entry, reset_mode 2)
  // per world vertex (word offset / 2 of the world parts): the broadphase
  // guard's edge pseudo-angle (ph_TV4, ph_T; written only with
  // COTIX_STAGE_BROADPHASE).  It overlays adj and rec, which only the backward
  // re-play uses, and the backward runs without the broadphase (an exact
  // filter: the same contacts; cotix_rollout_backward clears the stage bit):
  // the LunarLander tile stays within the LDS (a scene with more polygon
  // vertices gets words of its own)
  const bool own = PE > nb * (6 + REC_W);
  L.pedge = own ? L.pbox + 4 * np : L.adj;
  L.jfin = L.pbox + 4 * np + (own ? PE : 0);
  L.jal = L.jfin + 1;
  L.jr = L.jal + 1;
  L.jpr = L.jr + 1;
  L.jk = L.jpr + 1;
  L.je = L.jk + 2;
  L.jsn = L.je + 1;                 // this step's state becomes the premature out
  L.S = L.jsn + 1;
  return L;
}
static inline int tile_words(const SceneHdr& s) {
  return layout(s.nb, s.np, s.W, s.nc, s.nt, s.G, s.poly ? s.W / 2 : 0).S;
}
// per-wave scratch of phase C (words, not per env): pass flags, keep flags,
// active count, two item lists (double buffer), per-item scan positions
enum : int { WS_FLAG = 0, WS_KEEP = 64, WS_KEEP2 = 128, WS_N = 192, WS_LIST = 193 };
// + (polygon scenes) the deferred contact-point area of phase F: per-item
// flags and list (padded to 64), count, per-batch term counts, term results
constexpr int CFB = 8;                           // items per batch
constexpr int CFS = 2 * cx::MAXV + cx::MAXV * cx::MAXV;  // max terms per item
constexpr int EPA_NE = 20;                        // EPA edge column length (epa<20> bound)
struct WsLay {
  int cf_flag, cf_list, cf_n, cf_s, cf_c, cf_res, epa, bl_flag, bl_list, bl_n, bl_mode, bl_epa, bl_pad, vt, words;
};
CX_HD WsLay ws_layout(int nl, int nc, int ew, int poly, int nvt) {
  WsLay w;
  const int pad = ((nc * ew + 63) / 64) * 64;
  w.cf_flag = WS_LIST + 3 * nl * ew;
  w.cf_list = w.cf_flag + pad;
  w.cf_n = w.cf_list + pad;
  w.cf_s = w.cf_n + 1;
  w.cf_c = w.cf_s + CFB;  // per batch item: its containment terms |A| + |B| (F2 runs them apart)
  w.cf_res = w.cf_c + CFB;
  w.epa = w.cf_res + CFB * CFS * 2;  // per-lane EPA edge columns, [4*EPA_NE][64]
  // broadphase (polygon scenes): per-item keep flags (padded to 64) and the B list
  w.bl_pad = pad;
  w.bl_flag = w.epa + 4 * EPA_NE * 64;
  w.bl_list = w.bl_flag + pad;
  w.bl_n = w.bl_list + pad;
  // the B list's lane mapping this step (1: lane pairs) and whether an EPA
  // ran this step (the next step's mode); scheduling only, never results
  w.bl_mode = w.bl_n + 1;
  w.bl_epa = w.bl_n + 2;
  w.words = poly ? w.bl_n + 3 : w.cf_flag;
  // phase T's polygon vertex items (x, y, sort key per vertex, [word][env]):
  // they live only from TV1 to TV3, so they share the EPA columns, which
  // phase B fills afresh each step; else an area of their own
  const int nvw = 3 * nvt * ew;
  w.vt = (poly && nvw <= 4 * EPA_NE * 64) ? w.epa : w.words;
  if (w.vt == w.words) w.words += nvw;
  return w;
}
CX_HD int ws_words(const SceneHdr& s, int ew) { return ws_layout(s.nl, s.nc, ew, s.poly, s.nvt).words; }
// LDS bytes of a workgroup of wpb waves x ew envs
static inline size_t lds_bytes(const SceneHdr& s, int wpb, int ew) {
  return 4 * ((size_t)s.nhot + ((size_t)tile_words(s) * ew + (size_t)ws_words(s, ew)) * wpb);
}

// RL / RG: the lander's / both legs' mass and inertia have exact
// reciprocals (ql, qr, qll; cx::Rcp) -- their divisions become products
template <bool RL = false, bool RG = false>
CX_DEV void lunar_constraints(cx::Dyn& lander, cx::Dyn& rleg, cx::Dyn& lleg, const cx::Params& pl,
                              const cx::Params& pr, const cx::Params& pll, cx::Rcp ql = cx::no_rcp(),
                              cx::Rcp qr = cx::no_rcp(), cx::Rcp qll = cx::no_rcp()) {
  // LunarLander.step, cotix/_lunar_lander.py:145-218.  The anchors are taken
  // before any impulse (impulses change velocities only), so each body's
  // sin/cos (rotate, cotix/_geometry_utils.py:81-88) is evaluated once.
  using namespace cx;
  const float f05 = 0.05f;
  float sl, cl, sr, cr, sll, cll;
  sincos32(lander.a, &sl, &cl);
  sincos32(rleg.a, &sr, &cr);
  sincos32(lleg.a, &sll, &cll);
  auto rot = [](v2 v, float sn, float cs) { return v2{cs * v.x + (-sn) * v.y, sn * v.x + cs * v.y}; };
  v2 lp = v2{lander.px, lander.py};
  v2 llj1 = add(rot(v2{24.0f * f05, -8.0f * f05}, sl, cl), lp);
  v2 llj2 = add(rot(v2{24.0f * f05, 0.0f * f05}, sl, cl), lp);
  v2 lj1 = v2{lleg.px, lleg.py};
  v2 lj2 = add(v2{lleg.px, lleg.py}, rot(v2{0.0f, 0.4f}, sll, cll));
  v2 lrj1 = add(rot(v2{-24.0f * f05, -8.0f * f05}, sl, cl), lp);
  v2 lrj2 = add(rot(v2{-24.0f * f05, 0.0f * f05}, sl, cl), lp);
  v2 rj1 = v2{rleg.px, rleg.py};
  v2 rj2 = add(v2{rleg.px, rleg.py}, rot(v2{0.0f, 0.4f}, sr, cr));
  // apply_impulse (cotix/_bodies.py:68-73) with optional exact reciprocals
  auto apply = [](Dyn& b, const Params& m, Rcp q, bool r, v2 imp, v2 point) {
    const v2 arm = sub(point, v2{b.px, b.py});
    const float torque = crs(arm, imp);
    b.vx = b.vx + (r ? imp.x * q.m : imp.x / m.mass);
    b.vy = b.vy + (r ? imp.y * q.m : imp.y / m.mass);
    b.w = b.w + (r ? torque * q.i : torque / m.inertia);
  };
  auto fixed = [&](Dyn& b1, const Params& m1, Rcp q1, v2 c1, Dyn& b2, const Params& m2, Rcp q2, v2 c2) {
    v2 dp = sub(c1, c2);
    v2 dv = sub(velocity_at(b1, c1), velocity_at(b2, c2));
    float k = nrm(dv) + 0.1f;
    v2 imp = v2{dp.x * 1.0f + (dv.x * k) * f05, dp.y * 1.0f + (dv.y * k) * f05};
    apply(b1, m1, q1, RL, neg(imp), c1);
    apply(b2, m2, q2, RG, imp, c2);
  };
  fixed(lander, pl, ql, llj1, lleg, pll, qll, lj1);
  fixed(lander, pl, ql, llj2, lleg, pll, qll, lj2);
  fixed(lander, pl, ql, lrj1, rleg, pr, qr, rj1);
  fixed(lander, pl, ql, lrj2, rleg, pr, qr, rj2);
  rleg.w = rleg.w * 0.95f;
  lleg.w = lleg.w * 0.95f;
}

// contact-function sets compiled into a step kernel (scene feature mask)
// FNS_CONVEX: polygon x polygon GJK/EPA; FNS_AABB_POLY: AABB x polygon too
// (without it the GJK/EPA supports are compiled for polygons only)
enum : int { FNS_ANALYTIC = 1, FNS_CONVEX = 2, FNS_CIRCLE_POLY = 4, FNS_AABB_POLY = 8 };
// the FNSET instantiation of the step kernel for a scene's function set
// (launcher and host emulation): analytic scenes get the analytic program,
// modes 1 (rollout), 2 / 4 (its backward: re-play / tape) and 3 (eval with a
// judge or control) the full one
CX_HD int launch_fnset(int fs, int mode) {
  if ((fs & ~FNS_ANALYTIC) == 0) return FNS_ANALYTIC;
  if (mode >= 1 && mode <= 4) return FNS_ANALYTIC | FNS_CONVEX | FNS_CIRCLE_POLY | FNS_AABB_POLY;
  if ((fs & ~(FNS_ANALYTIC | FNS_CONVEX)) == 0) return FNS_ANALYTIC | FNS_CONVEX;
  if ((fs & FNS_CIRCLE_POLY) == 0) return FNS_ANALYTIC | FNS_CONVEX | FNS_AABB_POLY;
  return FNS_ANALYTIC | FNS_CONVEX | FNS_CIRCLE_POLY | FNS_AABB_POLY;
}
template <int FNSET>
CX_DEV cx::Contact run_contact_set(int fn, const cx::Shape& a, const cx::Shape& b, const cx::NarrowParams& np,
                                   uint32_t* err, bool self_pair) {
  using namespace cx;
  if ((FNSET & FNS_ANALYTIC) != 0) {
    if (fn == FN_AABB_AABB) return aabb_vs_aabb(a, b);
    if (fn == FN_CIRCLE_AABB) return circle_vs_aabb(a, b, err);
    if (fn == FN_CIRCLE_CIRCLE) return circle_vs_circle(a, b);
  }
  if ((FNSET & FNS_CONVEX) != 0) {
    if (fn == FN_POLY_POLY || fn == FN_AABB_POLY) return convex_vs_polygon(a, b, np, !self_pair);
  }
  if ((FNSET & FNS_CIRCLE_POLY) != 0) {
    if (fn == FN_CIRCLE_POLY) return circle_vs_polygon(a, b, np);
  }
  return nan_contact();
}

// jnp.cumsum via lax.associative_scan (CPU lowering), fully unrolled for a
// compile-time length so the tree lives in registers.
template <int N>
CX_DEV void cumsum_fixed(const float* x, float* out) {
  if constexpr (N < 2) {
    if constexpr (N == 1) out[0] = x[0];
  } else {
    constexpr int M = N / 2;
    float red[M], odd[M];
#pragma unroll
    for (int k = 0; k < M; ++k) red[k] = x[2 * k] + x[2 * k + 1];
    cumsum_fixed<M>(red, odd);
    constexpr int NE = (N % 2 == 0) ? M - 1 : M;
    float even[M + 1];
    even[0] = x[0];
#pragma unroll
    for (int k = 0; k < NE; ++k) even[k + 1] = odd[k] + x[2 * k + 2];
#pragma unroll
    for (int k = 0; k < N; ++k) out[k] = (k % 2 == 0) ? even[k / 2] : odd[k / 2];
  }
}
CX_DEV void cumsum_n(const float* x, int n, float* out) {
  switch (n) {
#define CXK_CS(k) \
  case k:         \
    cumsum_fixed<k>(x, out); \
    break;
    CXK_CS(1) CXK_CS(2) CXK_CS(3) CXK_CS(4) CXK_CS(5) CXK_CS(6) CXK_CS(7) CXK_CS(8)
    CXK_CS(9) CXK_CS(10) CXK_CS(11) CXK_CS(12) CXK_CS(13) CXK_CS(14) CXK_CS(15) CXK_CS(16)
#undef CXK_CS
    default: break;
  }
}

// Cross-lane primitives.  On the GPU they are the hardware's; the host
// emulation (tests/emu/cotix_simt.h) runs a wave's 64 lanes as fibers of the
// same program and resolves each of these as a collective point, so both run
// one code path.
#if !defined(__HIP__)
}  // namespace cxk
namespace cxk_simt {
void sync();
void lockstep();
uint64_t ballot(bool p);
uint32_t bpermute(int src, uint32_t v);
uint32_t pair_swap(uint32_t v);
}  // namespace cxk_simt
namespace cxk {
#define CXK_WAVE_OP static inline __attribute__((always_inline))
#else
#define CXK_WAVE_OP CX_DEV
#endif
// wave-local ordering between phases: every lane's LDS traffic of the
// previous phase is complete and visible to the wave before the next starts.
CXK_WAVE_OP void wave_sync() {
#if defined(__HIP__)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#else
  ::cxk_simt::sync();
#endif
}
// an order point inside a phase: every lane's LDS accesses before it precede
// every lane's after it.  The GPU's lanes run in lockstep and one wave's LDS
// operations execute in program order, so it emits nothing there; the host
// emulation, which runs lanes one after another, waits for the wave.
CXK_WAVE_OP void lockstep() {
#if !defined(__HIP__)
  ::cxk_simt::lockstep();
#endif
}
// a value whose producing global read must complete here (an empty asm that
// reads and writes it: the wait lands at this point, not at a later join)
CXK_WAVE_OP void settle(float& x) {
#if defined(__HIP__)
  asm volatile("" : "+v"(x));
#else
  (void)x;
#endif
}
// 64-bit ballot of p over the wave's active lanes
CXK_WAVE_OP uint64_t ballot(bool p) {
#if defined(__HIP__)
  return (uint64_t)__ballot(p);
#else
  return cxk_simt::ballot(p);
#endif
}
// the value v of lane src (ds_bpermute)
CXK_WAVE_OP uint32_t bpermute(int src, uint32_t v) {
#if defined(__HIP__)
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v);
#else
  return cxk_simt::bpermute(src, v);
#endif
}
// the value v of the lane pair's other lane (DPP quad_perm(1,0,3,2); both
// lanes of the pair active)
CXK_WAVE_OP uint32_t pair_swap_u32(uint32_t v) {
#if defined(__HIP__)
  return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false);
#else
  return cxk_simt::pair_swap(v);
#endif
}
CXK_WAVE_OP float pair_swap_f32(float x) { return __builtin_bit_cast(float, pair_swap_u32(__builtin_bit_cast(uint32_t, x))); }
// an LDS word OR-ed by several lanes of a phase
CXK_WAVE_OP void lds_or(uint32_t& w, uint32_t v) {
#if defined(__HIP__)
  atomicOr(&w, v);
#else
  w |= v;  // lanes run one at a time between collective points
#endif
}

// 64-bit ballot of flags[lane] != 0 over the wave (flags written by an
// earlier phase); called convergently
CX_DEV uint64_t wave_ballot(const uint32_t* flags, int lane) { return ballot(flags[lane] != 0u); }
CX_DEV int popc64(uint64_t m) { return __builtin_popcountll(m); }
// the number of lanes whose flag `mine` is set (every lane gets it); called
// convergently at the top level of a phase
CX_DEV int wave_count_stored(const uint32_t* flags, int lane, bool mine) {
  (void)flags;
  (void)lane;
  return popc64(ballot(mine));
}
CX_DEV uint64_t lanes_below(int lane) { return lane == 0 ? 0ull : ((1ull << lane) - 1ull); }

// LDS views: scene hot tables + this wave's [word][env] tile
template <int EW>
struct Tile {
  uint32_t* u;          // tile base
  const uint32_t* tb;   // hot tables
  uint32_t* ws;         // wave scratch (ws_words)
  CX_MF float& f(int off, int e) const { return reinterpret_cast<float*>(u)[off * EW + e]; }
  CX_MF uint32_t& w(int off, int e) const { return u[off * EW + e]; }
  CX_MF int ti(int off) const { return (int)tb[off]; }
};

struct Ctx {
  int nb, np, nc, nl, nt;
  SceneHdr sh;
  Lay L;
  WsLay W;
};
template <int EW>
CX_HD Ctx make_ctx(const SceneHdr& h) {
  return Ctx{h.nb, h.np, h.nc, h.nl, h.nt, h, layout(h.nb, h.np, h.W, h.nc, h.nt, h.G, h.poly ? h.W / 2 : 0),
             ws_layout(h.nl, h.nc, EW, h.poly, h.nvt)};
}

// the collider scan as one fused phase (ph_M_fused): its (cell, env) items fit
// two rounds of the wave, and its slot words' 12-bit candidate index holds
// every candidate (else the list form C0-C3 runs)
template <int EW>
CX_HD bool scan_fused(const Ctx& c) { return c.nl * EW <= 2 * WAVE && c.sh.ncand <= 4096; }

// local part geometry of the wave's envs: read from HBM once per launch, not
// once per step (per-env LunarLander terrain)
template <int EW>
CX_DEV void ph_geo(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane) {
  if (a.geom == nullptr) return;
  for (int w = lane; w < c.sh.G * EW; w += WAVE) {
    int e = w % EW, k = w / EW, g = env0 + e;
    t.f(c.L.geo + k, e) = (g < a.B) ? a.geom[(a.gstride ? (size_t)g * a.gstride : (size_t)0) + k] : 0.0f;
  }
}

template <int EW>
CX_DEV void k_one_regs(const KArgs& a, const Ctx& c, Tile<EW> t, int lane, uint32_t k0, uint32_t k1);
// the key chain of a one-step launch runs in the prologue, on the keys in
// registers, while the batch of state reads is in flight (ph_load)
CX_DEV bool keys_on(const KArgs& a) {
  return (a.stages & (COTIX_STAGE_COLLIDER | COTIX_STAGE_ADVANCE_KEY)) != 0 && !CXK_SKIP(a, 16);
}
CX_DEV bool k_in_prologue(const KArgs& a) { return keys_on(a) && a.n_steps == 1; }
// the polygon programs' wave-scratch words that live across steps (every
// program's first phase: the forward's load, the backward's adjoint init)
template <int EW>
CX_DEV void ws_poly_init(const Ctx& c, Tile<EW> t, int lane) {
  if (c.sh.poly) {  // phase F's flag array incl. its padding to a multiple of 64
    for (int w = lane; w < c.W.cf_list - c.W.cf_flag; w += WAVE) t.ws[c.W.cf_flag + w] = 0u;
    if (lane == 0) t.ws[c.W.bl_epa] = 0u;  // the first step's B list: one lane per item
  }
}
template <int EW, bool EVAL = false>
CX_DEV void ph_load(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane) {
  ws_poly_init<EW>(c, t, lane);
  // reset_mode 2 (cotix_eval's next-step autoreset): an env finished at entry
  // starts from its reset state (key chain continues, err and finished cleared)
  const bool r2 = a.reset_mode == 2 && a.dyn_reset != nullptr && a.finished != nullptr;
  uint32_t fin = 0u;  // bit e: env e restarts at entry (r2)
  if (r2)
    for (int e = 0; e < EW; ++e) fin |= (env0 + e < a.B && a.finished[env0 + e] != 0u) ? 1u << e : 0u;
  // per env (lane e < EW; EW <= 64): its words, read into registers before
  // the batch below so that every global read of the prologue is in flight
  // together
  const int ge = env0 + lane;
  const bool le = lane < EW && ge < a.B, rs = le && ((fin >> lane) & 1u) != 0u;
  const uint32_t k0 = le ? a.keys[2 * (size_t)ge] : 0u, k1 = le ? a.keys[2 * (size_t)ge + 1] : 0u;
  const uint32_t er = (le && !rs) ? a.err[ge] : 0u;
  // the restart counter, read here with the state (the store then writes it:
  // no read-modify-write round trip at the end of the launch)
  const uint32_t rc = ((le && a.resets != nullptr) ? a.resets[ge] : 0u) + (rs ? 1u : 0u);
  uint32_t jf = 0u;
  float jr = 0.0f;
  if (EVAL && a.judge.on) {
    jf = (le && !rs && a.finished != nullptr) ? (a.finished[ge] != 0u ? 1u : 0u) : 0u;
    jr = (le && a.reward != nullptr) ? a.reward[ge] : 0.0f;
  }
  // the state, the local geometry and the restart state in ONE batch of
  // global reads per lane (all issued before the first LDS store: one HBM
  // round trip instead of one per loop iteration -- the K = 1 launch's
  // fixed cost), item w over [dyn | geo | rst]
  const int nd = c.nb * 6 * EW, ng = a.geom != nullptr ? c.sh.G * EW : 0;
  const int nr = (a.dyn_reset != nullptr && a.reset_mode == 1) ? nd : 0, ntot = nd + ng + nr;
  constexpr int LK = 12;
  for (int base = 0; base < ntot; base += LK * WAVE) {
    float r[LK];
#pragma unroll
    for (int q = 0; q < LK; ++q) {
      const int w = base + q * WAVE + lane;
      const float* src = nullptr;
      if (w < nd) {
        const int e = w % EW, g = env0 + e;
        if (g < a.B) src = (((fin >> e) & 1u) ? a.dyn_reset : a.dyn) + (size_t)(w / EW) * a.B + g;
      } else if (w < nd + ng) {
        const int e = (w - nd) % EW, g = env0 + e;
        if (g < a.B) src = a.geom + (a.gstride ? (size_t)g * a.gstride : (size_t)0) + (w - nd) / EW;
      } else if (w < ntot) {
        const int e = (w - nd - ng) % EW, g = env0 + e;
        if (g < a.B) src = a.dyn_reset + (size_t)((w - nd - ng) / EW) * a.B + g;
      }
      r[q] = src != nullptr ? *src : 0.0f;
    }
    if (base == 0 && k_in_prologue(a)) k_one_regs<EW>(a, c, t, lane, k0, k1);  // uniform; the reads in flight
#pragma unroll
    for (int q = 0; q < LK; ++q) {
      const int w = base + q * WAVE + lane;
      if (w < nd)
        t.f(c.L.dyn + w / EW, w % EW) = r[q];
      else if (w < nd + ng)
        t.f(c.L.geo + (w - nd) / EW, (w - nd) % EW) = r[q];
      else if (w < ntot)
        t.f(c.L.rst + (w - nd - ng) / EW, (w - nd - ng) % EW) = r[q];
    }
  }
  if (lane < EW) {
    const int e = lane;
    t.w(c.L.key, e) = k0;
    t.w(c.L.key + 1, e) = k1;
    t.w(c.L.err, e) = er;
    t.w(c.L.nres, e) = rc;
    t.w(c.L.pcv, e) = 0u;  // no world part built yet in this launch (phase T)
    t.w(c.L.rflag, e) = 0u;  // no restart pending
    if (EVAL && a.judge.on) {
      t.w(c.L.jfin, e) = jf;
      t.f(c.L.jr, e) = jr;
    }
  }
}

// split(key, num)[idx] by a pair of adjacent lanes (h = lane & 1, both
// active): each lane runs the block of one of the key's two words
// (cx::split_word, the same block), then the pair swaps words (pair_swap) --
// half the threefry issue of split_at on the chain's critical path.
// The partitionable layout's split is ONE block (both words), which each
// lane of the pair runs itself (no exchange).
CX_DEV cx::key2 split_at_pair(cx::key2 k, uint32_t num, uint32_t idx, int h, bool part) {
  if (part) return cx::threefry(k, 0u, idx);
  const uint32_t mine = cx::split_word(k, num, 2u * idx + (uint32_t)h);
  const uint32_t other = pair_swap_u32(mine);
  return h ? cx::key2{other, mine} : cx::key2{mine, other};
}

// phase A: Euler (cotix/_physics_solvers.py:16-33) + driver extras + key chain
// phase K: the key window (steps step0 .. step0+n-1), three passes.
// K0 (one lane per env): the driver key chain k_{s+1} = split(k_s)[0] and the
// collider's skey_0 = split(k_s)[0] (cotix/_colliders.py:142,
// examples/test_viz.py:39,66).
// Items (env, half): the chain on a lane pair per env (split_at_pair).
template <int EW>
CX_DEV void ph_K0(const KArgs& a, const Ctx& c, Tile<EW> t, int lane, int n) {
  using namespace cx;
  const Lay& L = c.L;
  for (int w = lane; w < 2 * EW; w += WAVE) {
    const int e = w >> 1, h = w & 1;
    key2 k = key2{t.w(L.key, e), t.w(L.key + 1, e)};
    for (int s = 0; s < n; ++s) {
      const key2 s0 = split_at_pair(k, 2u, 0u, h, c.sh.prng != 0);
      if (h == 0) {
        t.w(L.kw + s * L.kww, e) = s0.a;
        t.w(L.kw + s * L.kww + 1, e) = s0.b;
      }
      if (a.stages & COTIX_STAGE_ADVANCE_KEY) k = s0;
    }
  }
}
// K1 (item = (step, env)): the per-type keys skey = split(skey)[0] (:175)
template <int EW>
CX_DEV void ph_K1(const Ctx& c, Tile<EW> t, int lane, int n) {
  using namespace cx;
  const Lay& L = c.L;
  for (int w = lane; w < n * EW; w += WAVE) {
    const int e = w % EW, o = L.kw + (w / EW) * L.kww;
    key2 k = key2{t.w(o, e), t.w(o + 1, e)};
    for (int q = 0; q < c.nt; ++q) {
      k = split_at_l(k, 2u, 0u, c.sh.prng != 0);
      t.w(o + 2 + 2 * q, e) = k.a;
      t.w(o + 3 + 2 * q, e) = k.b;
    }
  }
}
// K2 (item = (step, body, env)): the uniform of body i's contact choice,
// jr.choice(split(skey, n)[i], p) (:284-295) -> unit float of random_bits
template <int EW>
CX_DEV void ph_K2(const Ctx& c, Tile<EW> t, int lane, int n) {
  using namespace cx;
  const Lay& L = c.L;
  const int nb = c.nb;
  for (int w = lane; w < n * nb * EW; w += WAVE) {
    const int e = w % EW, i = (w / EW) % nb, o = L.kw + (w / EW / nb) * L.kww;
    const int so = c.nt > 0 ? o + 2 + 2 * (c.nt - 1) : o;
    const bool part = c.sh.prng != 0;
    const key2 ck = split_at_l(key2{t.w(so, e), t.w(so + 1, e)}, (uint32_t)nb, (uint32_t)i, part);
    t.f(o + 2 + 2 * c.nt + i, e) = unit_float(bits1_l(ck, part));
  }
}

// a one-step window (K = 1 launches, the RL loop) in ONE pass over (body,
// env) items: each lane derives its body's choice key through the whole
// chain (K0 -> K1 -> K2, the same splits), body 0's lane also writes the
// chain's keys -- no phase syncs or LDS round trips between the three levels.
// The env's collider key comes from lane e's registers (lane permutes), so a
// one-step launch runs this in its prologue (ph_load) while the state reads
// are in flight.  Items ((body, env), half) on lane pairs (split_at_pair),
// in uniform rounds of 64 (the permutes are wave-wide).
template <int EW>
CX_DEV void k_one_regs(const KArgs& a, const Ctx& c, Tile<EW> t, int lane, uint32_t k0, uint32_t k1) {
  using namespace cx;
  const Lay& L = c.L;
  const int nb = c.nb;
  const bool coll = (a.stages & COTIX_STAGE_COLLIDER) != 0;
  const bool part = c.sh.prng != 0;
  const int ni = 2 * (coll ? nb : 1) * EW;
  for (int base = 0; base < ni; base += WAVE) {
    const int w = base + lane, p = w >> 1, h = w & 1, e = p % EW, i = p / EW, o = L.kw;
    const key2 kin = key2{bpermute(e, k0), bpermute(e, k1)};  // env e's collider key (lane e)
    if (w >= ni) continue;
    const bool wr = i == 0 && h == 0;
    key2 k = split_at_pair(kin, 2u, 0u, h, part);  // K0
    if (wr) {
      t.w(o, e) = k.a;
      t.w(o + 1, e) = k.b;
    }
    for (int q = 0; q < c.nt; ++q) {  // K1
      k = split_at_pair(k, 2u, 0u, h, part);
      if (wr) {
        t.w(o + 2 + 2 * q, e) = k.a;
        t.w(o + 3 + 2 * q, e) = k.b;
      }
    }
    if (coll) {  // K2
      const float u = unit_float(bits1_l(split_at_pair(k, (uint32_t)nb, (uint32_t)i, h, part), part));
      if (h == 0) t.f(o + 2 + 2 * c.nt + i, e) = u;
    }
  }
}

// PRE: the step's keys come from the key window (slot `slot`); otherwise
// (backward re-play from saved keys) they are split here.
// Euler (cotix/_physics_solvers.py:16-33) + the driver's velocity terms for
// body b of env e (examples/test_viz.py:27-31; the config-5 action hook)
// the device control's velocity impulse from the body's state before the
// step (cotix_control): dv[i] = sum_q gain[i][q] * (target[i][q] - s[q]) over
// the nonzero gains in q order (from the first term), then + bias[i] if nonzero
template <int EW>
CX_DEV cx::v2 control_dv(const KArgs& a, Tile<EW> t, int o, int e) {
  float dv[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    float acc = 0.0f;
    bool any = false;
#pragma unroll
    for (int q = 0; q < 6; ++q)
      if (a.ctl.gain[i][q] != 0.0f) {  // kernel-argument constant: uniform branch
        const float term = a.ctl.gain[i][q] * (a.ctl.target[i][q] - t.f(o + q, e));
        acc = any ? acc + term : term;
        any = true;
      }
    if (a.ctl.bias[i] != 0.0f) acc = any ? acc + a.ctl.bias[i] : a.ctl.bias[i];
    if (a.ctl.sat) acc = cx::clip_(acc, a.ctl.lo[i], a.ctl.hi[i]);  // the saturating form (jnp.clip)
    dv[i] = acc;
  }
  return cx::v2{dv[0], dv[1]};
}

// Restarts of the autoreset programs (reset_mode 1) are deferred: phase E
// flags the env (rflag) and the next step's phase A (euler_item, DEFER)
// copies the flagged env's restart state before it reads the state -- one
// restart phase (ph_R) after the last step instead of one after every step;
// the values are the ones the copy after the step would have left (nothing
// reads the state in between).  Deferred when phase A runs as a phase of its
// own (Euler or gravity on), and in the staged A/T/B phase where its fetch
// reads the restart state of a pending env (run_wave's SDEFER: kept to the
// RoboCup step, whose register budget holds the select; run_wave's `defer`).
CX_DEV bool restart_deferred(const KArgs& a) {
  return a.dyn_reset != nullptr && a.reset_mode == 1 && (a.stages & (COTIX_STAGE_EULER | COTIX_STAGE_GRAVITY)) != 0;
}

// The action of a step (config 5's per-step dv, the RL loop's held action)
// in the registers of the lane that applies it, read one step ahead (phase A
// would otherwise wait a global round trip every step): lane w = (action
// body, env) item of phase A's first round (nb * EW <= 64, act_prefetch).
struct ActRegs {
  float x = 0.0f, y = 0.0f;
};
template <int EW>
CX_HD bool act_prefetch(const KArgs& a, const Ctx& c) { return a.action != nullptr && c.nb * EW <= WAVE; }
template <int EW>
CX_DEV void act_fetch(const KArgs& a, const Ctx& c, int env0, int lane, int step, ActRegs& r) {
  const int e = lane % EW, g = env0 + e;
  if (lane < c.nb * EW && lane / EW == a.action_body && g < a.B) {
    const float* ac = a.action + ((size_t)(a.action_held ? 0 : step) * a.B + g) * 2;
    r.x = ac[0];
    r.y = ac[1];
  }
}

// The rollout forward's per-step actions, AWIN steps at a time, in the tile's
// restart-state words (free there: the rollout never restarts, and its
// return terms are in registers once ret_fetch has run): one global round
// trip -- and one wait behind the save phase's stores -- per AWIN steps
// instead of per step (act_window_fill; word 2 s + component of step s of the
// window, env e)
constexpr int AWIN = 8;
template <int EW>
CX_DEV bool act_window(const KArgs& a, const Ctx& c) {
  return a.action != nullptr && !a.action_held && c.nb * 6 >= 2 * AWIN;
}
template <int EW>
CX_DEV void act_window_fill(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane, int step0) {
  const int n = a.n_steps - step0 < AWIN ? a.n_steps - step0 : AWIN;
  for (int w = lane; w < 2 * n * EW; w += WAVE) {
    const int e = w % EW, k = w / EW, g = env0 + e;
    const float v = g < a.B ? a.action[((size_t)(step0 + (k >> 1)) * a.B + g) * 2 + (k & 1)] : 0.0f;
    t.f(c.L.rst + k, e) = v;
  }
}

// EVAL: the cotix_eval program (device judge / control); the step programs
// are compiled without them.  DEFER: take a deferred restart first.  ar: the
// item's prefetched action (act_fetch) where has_ar, else read here (by
// value: a pointer that may be null keeps the registers in private memory)
template <int EW, bool EVAL = false, bool DEFER = false>
CX_DEV void euler_item(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int e, int b, int step,
                       bool has_ar = false, ActRegs ar = ActRegs{}) {
  const int o = c.L.dyn + b * 6;
  if (DEFER && restart_deferred(a) && t.w(c.L.rflag, e) != 0u) {  // the body's restart state first
#pragma unroll
    for (int q = 0; q < 6; ++q) t.f(o + q, e) = t.f(c.L.rst + b * 6 + q, e);
  }
  const bool ctl = EVAL && a.ctl.on && b == a.ctl.body;
  const cx::v2 dv = ctl ? control_dv<EW>(a, t, o, e) : cx::v2{0.0f, 0.0f};
  if (!(a.stages & (COTIX_STAGE_EULER | COTIX_STAGE_GRAVITY))) return;  // (ph_A calls only with either)
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
    float ax, ay;
    if (has_ar) {
      ax = ar.x;
      ay = ar.y;
    } else {
      const float* ac = a.action + ((size_t)(a.action_held ? 0 : step) * a.B + env0 + e) * 2;
      ax = ac[0];
      ay = ac[1];
      // the read completes on this path: merged with the register path, the
      // compiler waited at the join (s_waitcnt vmcnt(0)) on BOTH paths -- for
      // every store in flight too (the rollout's saves: ~1.2 k cycles a step)
      settle(ax);
      settle(ay);
    }
    t.f(o + 2, e) = t.f(o + 2, e) + ax;
    t.f(o + 3, e) = t.f(o + 3, e) + ay;
  }
  if (ctl) {  // world.forward(state, signal): the impulse after Euler (cotix/_envs.py:72-75)
    t.f(o + 2, e) = t.f(o + 2, e) + dv.x;
    t.f(o + 3, e) = t.f(o + 3, e) + dv.y;
  }
}
// per-step collider scratch: all_contacts cells empty (:137-140), choice =
// self (m and ch are adjacent in the tile: one flat, branch-free pass), no
// valid contact
template <int EW>
CX_DEV void reset_scratch(const Ctx& c, Tile<EW> t, int lane) {
  const int nm = c.nb * c.nb;
  for (int w = lane; w < (nm + c.nb) * EW; w += WAVE)
    t.u[c.L.m * EW + w] = w < nm * EW ? 0xFFFFFFFFu : (uint32_t)(w / EW - nm);
  for (int w = lane; w < c.sh.nmw * EW; w += WAVE) t.u[c.L.vm * EW + w] = 0u;
}

template <int EW, bool PRE = false, bool EVAL = false, bool DEFER = false>
CX_DEV void ph_A(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane, int step, int slot = 0,
                 bool has_ar = false, ActRegs ar = ActRegs{}) {
  using namespace cx;
  const int nb = c.nb;
  const Lay& L = c.L;
  if (a.stages & (COTIX_STAGE_EULER | COTIX_STAGE_GRAVITY))
    for (int w = lane; w < nb * EW; w += WAVE) {
      const int e = w % EW, b = w / EW;
      if (env0 + e < a.B) euler_item<EW, EVAL, DEFER>(a, c, t, env0, e, b, step, has_ar, ar);
    }
  if (a.stages & (COTIX_STAGE_COLLIDER | COTIX_STAGE_ADVANCE_KEY)) {
    if (!PRE && !CXK_SKIP(a, 16)) {
      // (the backward re-play: the step's keys from its saved key) on a lane
      // pair per env (split_at_pair: each lane one block of each split)
      const bool part = c.sh.prng != 0;
      for (int w = lane; w < 2 * EW; w += WAVE) {
        const int e = w >> 1, h = w & 1;
        key2 k = key2{t.w(L.key, e), t.w(L.key + 1, e)};
        key2 s = split_at_pair(k, 2u, 0u, h, part);  // cotix/_colliders.py:142 == next driver key
        if (h == 0) {
          t.w(L.sk0, e) = s.a;
          t.w(L.sk0 + 1, e) = s.b;
        }
        for (int q = 0; q < c.nt; ++q) {  // :175, one split per type key
          s = split_at_pair(s, 2u, 0u, h, part);
          if (h == 0) {
            t.w(L.skt + 2 * q, e) = s.a;
            t.w(L.skt + 2 * q + 1, e) = s.b;
          }
        }
      }
    }
    reset_scratch<EW>(c, t, lane);
  }
}

// phase T: shape.transform(body transformer) (cotix/_colliders.py:92-94).
// Circles and AABBs: one (part, env) item per lane.  Polygons
// (:181-187 forward_vector then the re-sort of Polygon.__init__) are spread
// over (vertex, env) items in three sub-phases TV1-TV3 (ph_TV*), and a body
// whose pose (position and angle bits) equals the pose its world parts were
// last built from in this launch keeps them: the transform is a function of
// the pose and the launch-constant local geometry only, so the kept parts are
// the bits a recomputation would give (LunarLander: the static terrain).
template <int EW, int FNSET>
CX_DEV void ph_T(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane) {
  using namespace cx;
  const SceneHdr& sc = c.sh;
  for (int w = lane; w < c.np * EW; w += WAVE) {
    int e = w % EW, p = w / EW, g = env0 + e;
    if (g >= a.B) continue;
    const int b = t.ti(sc.o_pbody + p), kind = t.ti(sc.o_pkind + p);
    if (FNSET != FNS_ANALYTIC && kind == KIND_POLY) continue;  // ph_TV*
    const int lgo = c.L.geo + t.ti(sc.o_pgoff + p);  // this part's local geometry in the tile
    const int o = c.L.dyn + b * 6, wo = c.L.world + t.ti(sc.o_pwoff + p);
    const float px = t.f(o + 0, e), py = t.f(o + 1, e);
    // Circle (r, cx, cy, pad): translate only, cotix/_convex_shapes.py:37-41
    // AABB (lo.x, lo.y, up.x, up.y): translate only, :113-117
    // Branch-free on purpose: all four floats are loaded unconditionally
    // (a divergent circle/AABB tail was miscompiled by hipcc 7.2: the
    // circle lanes read an address register only the AABB lanes defined).
    const bool circ = kind == KIND_CIRCLE;
    const float g0 = t.f(lgo, e), g1 = t.f(lgo + 1, e), g2 = t.f(lgo + 2, e), g3 = t.f(lgo + 3, e);
    t.f(wo + 0, e) = circ ? g0 : g0 + px;
    t.f(wo + 1, e) = circ ? g1 + px : g1 + py;
    t.f(wo + 2, e) = circ ? g2 + py : g2 + px;
    t.f(wo + 3, e) = circ ? g3 : g3 + py;
    if (FNSET != FNS_ANALYTIC) {  // the part's world AABB (broadphase, ph_BP0)
      const int bo = c.L.pbox + 4 * p;
      const float w0 = t.f(wo, e), w1 = t.f(wo + 1, e), w2 = t.f(wo + 2, e), w3 = t.f(wo + 3, e);
      // circle (r, cx, cy): center -+ r; AABB (lo, up)
      t.f(bo, e) = circ ? w1 - w0 : w0;
      t.f(bo + 1, e) = circ ? w2 - w0 : w1;
      t.f(bo + 2, e) = circ ? w1 + w0 : w2;
      t.f(bo + 3, e) = circ ? w2 + w0 : w3;
      if (sc.poly && (a.stages & COTIX_STAGE_BROADPHASE)) {
        // the broadphase guard's edge pseudo-angles of an AABB: the axes
        // (get_edges, cotix/_convex_shapes.py:82-93), exactly 0 and 1 (ph_TV4);
        // unused for a circle
        const int po = c.L.pedge + t.ti(sc.o_pwoff + p) / 2;
        t.f(po, e) = 0.0f;
        t.f(po + 1, e) = 1.0f;
      }
    }
  }
}
// body b of env e still has the pose its world parts were built from
template <int EW>
CX_DEV bool pose_kept(const Ctx& c, Tile<EW> t, int b, int e) {
  const Lay& L = c.L;
  const int o = L.dyn + 6 * b, q = L.pose + 3 * b;
  // every word read unconditionally (a short-circuit chain of LDS reads
  // compiles to one round trip per read)
  const uint32_t v = t.w(L.pcv, e), p0 = t.w(o, e), p1 = t.w(o + 1, e), p2 = t.w(o + 4, e);
  const uint32_t q0 = t.w(q, e), q1 = t.w(q + 1, e), q2 = t.w(q + 2, e);
  return (((v >> b) & 1u) != 0u) & (p0 == q0) & (p1 == q1) & (p2 == q2);
}
// TV0 (item = (body, env)): flag the bodies whose world parts must be rebuilt
// this step, then record the poses they will be built from
template <int EW>
CX_DEV void ph_TV0(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane) {
  const Lay& L = c.L;
  for (int w = lane; w < c.nb * EW; w += WAVE) {
    const int e = w % EW, b = w / EW;
    const bool redo = (env0 + e < a.B) & !pose_kept<EW>(c, t, b, e);
    if (w < WAVE) t.ws[WS_FLAG + w] = redo ? 1u : 0u;
    t.w(L.pose + 3 * b, e) = t.w(L.dyn + 6 * b, e);
    t.w(L.pose + 3 * b + 1, e) = t.w(L.dyn + 6 * b + 1, e);
    t.w(L.pose + 3 * b + 2, e) = t.w(L.dyn + 6 * b + 4, e);
  }
  if (lane >= c.nb * EW) t.ws[WS_FLAG + lane] = 0u;
}
// word q (x, y, key) of polygon vertex item v of env e (wave scratch)
template <int EW>
CX_DEV float& vtf(const Ctx& c, Tile<EW> t, int v, int q, int e) {
  return reinterpret_cast<float*>(t.ws)[c.W.vt + (3 * v + q) * EW + e];
}
// TV1-TV3 run over the vertex items in chunks of 64 (item w = (vertex, env),
// env fastest) and rebuild the items of the flagged (body, env) pairs only (a
// part's vertices may straddle chunks: all of them are rebuilt or none); a
// chunk with no flagged item is skipped (wave-uniform).
template <int EW>
CX_DEV uint64_t tv_redo_mask(const Ctx& c, Tile<EW> t, int lane) {
  return c.nb * EW <= WAVE ? wave_ballot(t.ws + WS_FLAG, lane) : ~0ull;
}
template <int EW>
CX_DEV bool tv_item_redo(const Ctx& c, uint64_t redo, int b, int e) {
  return c.nb * EW > WAVE || ((redo >> (b * EW + e)) & 1ull) != 0ull;
}
template <int EW>
CX_DEV bool tv_chunk_runs(const Ctx& c, Tile<EW> t, uint64_t redo, int k) {
  if (c.nb * EW > WAVE) return true;
  const int nw = c.sh.nvt * EW, lo = k * WAVE, hi = (lo + WAVE < nw ? lo + WAVE : nw) - 1;
  const int blo = (int)(t.tb[c.sh.o_vit + 2 * (lo / EW)] >> 21), bhi = (int)(t.tb[c.sh.o_vit + 2 * (hi / EW)] >> 21);
  const int n = (bhi + 1 - blo) * EW;  // item bits of bodies blo..bhi
  const uint64_t m = (n >= 64 ? ~0ull : ((1ull << n) - 1ull)) << (blo * EW);
  return (redo & m) != 0ull;
}
// bit k: chunk k runs (all chunks' table reads issued together)
template <int EW>
CX_DEV uint32_t tv_chunks(const Ctx& c, Tile<EW> t, uint64_t redo) {
  uint32_t runs = 0u;
  for (int k = 0; k * WAVE < c.sh.nvt * EW; ++k) runs |= tv_chunk_runs<EW>(c, t, redo, k) ? 1u << k : 0u;
  return runs;
}
// TV1 (item = (polygon vertex v, env)): the affine map of vertex k of part p
// (HomogenuousTransformer.forward_vector, cotix/_geometry_utils.py:105-112)
// into the vertex item's x, y
template <int EW>
CX_DEV void ph_TV1(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane, uint64_t redo, uint32_t runs) {
  using namespace cx;
  const SceneHdr& sc = c.sh;
  const Lay& L = c.L;
  for (int e = lane; e < EW; e += WAVE) t.w(L.pcv, e) = c.nb >= 32 ? ~0u : ((1u << c.nb) - 1u);
  for (int k0 = 0; k0 * WAVE < sc.nvt * EW; ++k0) {
    if (!((runs >> k0) & 1u)) continue;
    const int w = k0 * WAVE + lane, e = w % EW, v = w / EW;
    if (w >= sc.nvt * EW || env0 + e >= a.B) continue;
    const uint32_t d = t.tb[sc.o_vit + 2 * v], d1 = t.tb[sc.o_vit + 2 * v + 1];
    const int b = (int)(d >> 21), lg = L.geo + (int)(d1 & 0xFFFFu);
    if (!tv_item_redo<EW>(c, redo, b, e)) continue;
    const int o = L.dyn + b * 6;
    const float px = t.f(o + 0, e), py = t.f(o + 1, e);
    float s, cs;
    sincos32(t.f(o + 4, e), &s, &cs);
    const float x = t.f(lg, e), y = t.f(lg + 1, e);
    const float t0 = (cs * x + (-s) * y) + px * 1.0f;
    const float t1 = (s * x + cs * y) + py * 1.0f;
    // w = (0*x + 0*y) + 1*1 is exactly 1 (or NaN when x or y is infinite), so
    // t/w == (w == 1 ? t : NaN) bit for bit
    const float t2 = (0.0f * x + 0.0f * y) + 1.0f * 1.0f;
    vtf<EW>(c, t, v, 0, e) = t2 == 1.0f ? t0 : qnan();
    vtf<EW>(c, t, v, 1, e) = t2 == 1.0f ? t1 : qnan();
  }
}
// TV2: order_clockwise's sort key of the vertex (cotix/_geometry_utils.py:
// 60-67): the sequential mean of the part's vertices, then atan2 about it;
// NaN -> 4 (after every angle, all NaN equal: sort_lt is key order)
template <int EW>
CX_DEV void ph_TV2(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane, uint64_t redo, uint32_t runs) {
  using namespace cx;
  const SceneHdr& sc = c.sh;
  for (int k0 = 0; k0 * WAVE < sc.nvt * EW; ++k0) {
    if (!((runs >> k0) & 1u)) continue;
    const int w = k0 * WAVE + lane, e = w % EW, v = w / EW;
    if (w >= sc.nvt * EW || env0 + e >= a.B) continue;
    const uint32_t d = t.tb[sc.o_vit + 2 * v];
    const int n = (int)((d >> 8) & 15u), v0 = (int)((d >> 12) & 511u);
    if (!tv_item_redo<EW>(c, redo, (int)(d >> 21), e)) continue;
    // every read unconditional (clamped index, the sum selects): guarded
    // reads compile to one LDS round trip per vertex
    float xs[MAXV], ys[MAXV];
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int vk = v0 + (k < n ? k : 0);
      xs[k] = vtf<EW>(c, t, vk, 0, e);
      ys[k] = vtf<EW>(c, t, vk, 1, e);
    }
    float sx = 0.0f, sy = 0.0f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      sx = k < n ? sx + xs[k] : sx;
      sy = k < n ? sy + ys[k] : sy;
    }
    const float fn = (float)n;
    const float mx = sx / fn, my = sy / fn;
    const float ang = atan2_32(vtf<EW>(c, t, v, 1, e) - my, vtf<EW>(c, t, v, 0, e) - mx);
    vtf<EW>(c, t, v, 2, e) = isn(ang) ? 4.0f : ang;
    if (v == v0) {
      // the part's world AABB (broadphase, ph_BP0): hardware min/max (a NaN
      // operand yields the other one), so an all-NaN part gives a NaN box
      // and a NaN vertex is left out -- it contributes only NaN terms to
      // _contact_from_edges; order-independent, so the unsorted vertices do
      float lx = xs[0], ly = ys[0], ux = lx, uy = ly;
#pragma unroll
      for (int k = 1; k < MAXV; ++k) {
        const bool in = k < n;
        lx = in ? __builtin_fminf(lx, xs[k]) : lx;
        ly = in ? __builtin_fminf(ly, ys[k]) : ly;
        ux = in ? __builtin_fmaxf(ux, xs[k]) : ux;
        uy = in ? __builtin_fmaxf(uy, ys[k]) : uy;
      }
      const int bo = c.L.pbox + 4 * (int)(d & 31u);
      t.f(bo, e) = lx;
      t.f(bo + 1, e) = ly;
      t.f(bo + 2, e) = ux;
      t.f(bo + 3, e) = uy;
    }
  }
}
// TV3: the vertex's stable rank among its part's keys -- #{j < k : !(key_k <
// key_j)} + #{j > k : key_j < key_k}, the permutation insertion sort produces
// -- is its slot in the world part
template <int EW>
CX_DEV void ph_TV3(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane, uint64_t redo, uint32_t runs) {
  using namespace cx;
  const SceneHdr& sc = c.sh;
  const Lay& L = c.L;
  for (int k0 = 0; k0 * WAVE < sc.nvt * EW; ++k0) {
    if (!((runs >> k0) & 1u)) continue;
    const int w = k0 * WAVE + lane, e = w % EW, v = w / EW;
    if (w >= sc.nvt * EW || env0 + e >= a.B) continue;
    const uint32_t d = t.tb[sc.o_vit + 2 * v], d1 = t.tb[sc.o_vit + 2 * v + 1];
    const int k = (int)((d >> 5) & 7u), n = (int)((d >> 8) & 15u), v0 = (int)((d >> 12) & 511u);
    if (!tv_item_redo<EW>(c, redo, (int)(d >> 21), e)) continue;
    const float kk = vtf<EW>(c, t, v, 2, e);
    float ks[MAXV];
#pragma unroll
    for (int j = 0; j < MAXV; ++j) ks[j] = vtf<EW>(c, t, v0 + (j < n ? j : 0), 2, e);  // unconditional reads
    int r = 0;
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {  // flat selects (a short-circuit form compiles to branches)
      const int before = ks[j] < kk ? 1 : 0, not_after = kk < ks[j] ? 0 : 1;
      const int in = (j < n ? 1 : 0) & (j != k ? 1 : 0);
      r += in & (j < k ? not_after : before);
    }
    const int wo = L.world + (int)(d1 >> 16) + 2 * r;
    t.f(wo, e) = vtf<EW>(c, t, v, 0, e);
    t.f(wo + 1, e) = vtf<EW>(c, t, v, 1, e);
  }
}
// TV4 (broadphase scenes; item = (world vertex slot k of a rebuilt polygon,
// env)): the shape half of the broadphase guard (DESIGN.md section 3,
// "Broadphase exactness"), once per rebuilt world part instead of per pair.
// Edge k is d_k = v_k - v_k-1 (get_edges, cotix/_convex_shapes.py:160-163);
// the slot stores the pseudo-angle of its line, q = 1 - x in [0, 2) for the
// l1-normalized direction (x, y) = +-d_k / |d_k|_1 with the sign taken so
// that y > 0 or (y == 0, x > 0), when
//  * |d_k|_1 lies in [2^-40, 2^40] (no under/overflow in the products below;
//    false for NaN),
//  * the turn at v_k is strictly counter-clockwise beyond the rounding of the
//    cross product: cross(d_k, d_k+1) > 2^-21 |d_k|_1 |d_k+1|_1 (the world
//    vertices are in order_clockwise's ascending-angle order, so a strictly
//    convex part turns left at every vertex),
//  * a sharp vertex (dot(d_k, d_k+1) < 0: interior angle below 90 degrees) is
//    not too sharp: |cross| >= 2^-7 |d_k|_1 |d_k+1|_1,
// and 2^100 otherwise -- it fails every edge-pair test of ph_BP0, so a part
// with any failing vertex is never certified.
template <int EW>
CX_DEV void ph_TV4(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane, uint64_t redo, uint32_t runs) {
  using namespace cx;
  const SceneHdr& sc = c.sh;
  const Lay& L = c.L;
  for (int k0 = 0; k0 * WAVE < sc.nvt * EW; ++k0) {
    if (!((runs >> k0) & 1u)) continue;
    const int w = k0 * WAVE + lane, e = w % EW, v = w / EW;
    if (w >= sc.nvt * EW || env0 + e >= a.B) continue;
    const uint32_t d = t.tb[sc.o_vit + 2 * v], d1 = t.tb[sc.o_vit + 2 * v + 1];
    const int k = (int)((d >> 5) & 7u), n = (int)((d >> 8) & 15u);
    if (!tv_item_redo<EW>(c, redo, (int)(d >> 21), e)) continue;
    const int wo = L.world + (int)(d1 >> 16);
    const int km = k == 0 ? n - 1 : k - 1, kp = k + 1 == n ? 0 : k + 1;
    const float xm = t.f(wo + 2 * km, e), ym = t.f(wo + 2 * km + 1, e);
    const float x0 = t.f(wo + 2 * k, e), y0 = t.f(wo + 2 * k + 1, e);
    const float xp = t.f(wo + 2 * kp, e), yp = t.f(wo + 2 * kp + 1, e);
    const float dx0 = x0 - xm, dy0 = y0 - ym, dx1 = xp - x0, dy1 = yp - y0;
    const float l0 = __builtin_fabsf(dx0) + __builtin_fabsf(dy0), l1 = __builtin_fabsf(dx1) + __builtin_fabsf(dy1);
    const float cr = dx0 * dy1 - dy0 * dx1, dt = dx0 * dx1 + dy0 * dy1, ll = l0 * l1;
    const bool ok = (n >= 3) & (l0 >= 9.094947017729282e-13f) & (l0 <= 1.099511627776e12f) &  // [2^-40, 2^40]
                    (cr > 4.76837158203125e-07f * ll) &                                      // 2^-21
                    ((dt >= 0.0f) | (__builtin_fabsf(cr) >= 0.0078125f * ll));               // 2^-7
    const bool flip = (dy0 < 0.0f) | ((dy0 == 0.0f) & (dx0 < 0.0f));
    const float q = 1.0f - (flip ? -dx0 : dx0) / l0;
    t.f(L.pedge + (int)(d1 >> 16) / 2 + k, e) = ok ? q : 0x1p100f;  // failed: never certified (ph_BP0)
  }
}

// phase B: distinct contacts (cotix/_colliders.py:149-173); item w =
// (contact, env), env fastest
// _contact_from_edges(P, P) (cotix/_contacts.py:205-267) of a polygon with
// itself has a finite contact point when every coordinate is finite with
// |x| < 2^60 and some pair of adjacent edges is not parallel: for edge a =
// edge k = (v_k, v_{k-1}) and edge b = edge k-1 = (v_{k-1}, v_{k-2}) the
// reference computes q - p = v_{k-1} - v_k = r with the same rounding, so t =
// cross(r, s) / cross(r, s) = 1 and u = cross(r, r) / c = +-0: the
// intersection v_k + r is a term; every term is bounded by the coordinates,
// so their sum cannot overflow.  Returns false when it cannot decide (the
// caller then runs phase F on the item).
CX_DEV bool self_cp_finite(const cx::Shape& P) {
  using namespace cx;
  bool ok = true, any = false;
  const float lim = 1.152921504606846976e18f;  // 2^60
#pragma unroll
  for (int k = 0; k < MAXV; ++k)  // bitwise: no short-circuit branches
    ok = ok & ((k >= P.n) | ((__builtin_fabsf(P.w[2 * k]) < lim) & (__builtin_fabsf(P.w[2 * k + 1]) < lim)));
  // vertex k - 1 and k - 2 (cyclic): v_{k-1} is the previous slot, or the
  // last vertex for k = 0; v_{k-2} the one before that
  v2 prev2 = vert(P, P.n - 2), prev = vert(P, P.n - 1);
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const bool in = k < P.n;
    const v2 vk = v2{P.w[2 * k], P.w[2 * k + 1]};
    const v2 r = sub(prev, vk), sv = sub(prev2, prev);
    const float cr = r.x * sv.y - sv.x * r.y;
    any = any | (in & (cr != 0.0f));
    prev2 = in ? prev : prev2;
    prev = in ? vk : prev;
  }
  return ok & any;
}

// TAPE (rollout forward with a tape): EPA's final edge of the item to the
// tape (step `step`)
template <int EW, int FNSET, bool TAPE = false>
CX_DEV void b_item(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane, int w, int step = 0) {
  using namespace cx;
  const SceneHdr& sc = c.sh;
  const NarrowParams np = narrow_of(sc);
  {
    int e = w % EW, ci = w / EW, g = env0 + e;
    if (g >= a.B) return;
    const uint32_t d0w = t.tb[sc.o_cdesc + 2 * ci], d1w = t.tb[sc.o_cdesc + 2 * ci + 1];
    CXK_STAT(b_items, 1);
    const int fn = (int)((d0w >> 20) & 7u);
    const int wa = c.L.world + (int)(d0w & 1023u), wb = c.L.world + (int)((d0w >> 10) & 1023u);
    Shape A, Bs;
    A.kind = (int)((d0w >> 23) & 3u);
    Bs.kind = (int)((d0w >> 25) & 3u);
    A.n = (int)(d1w & 255u);
    Bs.n = (int)((d1w >> 8) & 255u);
    // one unconditional fetch of both shapes (the world region is followed
    // by 2*MAXV words of slack, so every read stays inside the tile)
    const int nw = FNSET == FNS_ANALYTIC ? 4 : 2 * MAXV;
#pragma unroll
    for (int k = 0; k < 2 * MAXV; ++k) {
      A.w[k] = k < nw ? t.f(wa + k, e) : 0.0f;
      Bs.w[k] = k < nw ? t.f(wb + k, e) : 0.0f;
    }
    uint32_t er = 0u;
    Contact ct;
    if ((FNSET & FNS_CONVEX) != 0 && (fn == FN_POLY_POLY || fn == FN_AABB_POLY)) {
      // GJK (+EPA); the contact point is deferred to phase F (wave-cooperative)
      const bool self = ((d0w >> 27) & 1u) != 0u;
      float* col = reinterpret_cast<float*>(t.ws + c.W.epa + lane);
      v2 edge[2];
      const bool hit = CXK_SKIP(a, 64) ? (ct.pen = v2{0.0f, 0.0f}, true)  // timing only: no GJK / EPA
                       : (FNSET & FNS_AABB_POLY) == 0
                           ? convex_vs_polygon_pen_col<true>(A, Bs, np, !self, &ct.pen, col, WAVE, TAPE ? edge : nullptr)
                           : convex_vs_polygon_pen_col<false>(A, Bs, np, !self, &ct.pen, col, WAVE, TAPE ? edge : nullptr);
      CXK_STAT(epa_runs, hit && !self ? 1 : 0);
      if (TAPE && a.tape != nullptr && hit && !self) {  // (a tape only with the polygon words, tape_words)
        const int o = 5 * c.nb + 4 * ci;
        const float ev[4] = {edge[0].x, edge[0].y, edge[1].x, edge[1].y};
#pragma unroll
        for (int q = 0; q < 4; ++q) a.tape[row_at(a.B, a.tw, step, o + q, g)] = __float_as_uint(ev[q]);
      }
      ct.cp = v2{qnan(), qnan()};
      // a part paired with itself: only the NaN-ness of its contact point is
      // observable (such a cell is only ever chosen as j == i, which
      // resolution skips), and it is decided here exactly (self_cp_finite)
      // instead of by phase F
      if (hit && self && self_cp_finite(A)) ct.cp = v2{0.0f, 0.0f};
      else if (hit) t.ws[c.W.cf_flag + w] = 1u;
      if (hit && !self) t.ws[c.W.bl_epa] = 1u;  // an EPA ran (B-list scheduling of the next step)
    } else {
      ct = run_contact_set<FNSET>(fn, A, Bs, np, &er, ((d0w >> 27) & 1u) != 0u);
    }
    const int co = c.L.con + 4 * ci;
    t.f(co + 0, e) = ct.pen.x;
    t.f(co + 1, e) = ct.pen.y;
    t.f(co + 2, e) = ct.cp.x;
    t.f(co + 3, e) = ct.cp.y;
    if (!(isn(ct.cp.x) || isn(ct.cp.y))) {
      lds_or(t.w(c.L.vm + (ci >> 5), e), 1u << (ci & 31));
    }
    if (er) {
      lds_or(t.w(c.L.err, e), er);
    }
  }
}
// phase B of the analytic program (circle / AABB scenes): the items of up to
// BQ chunks fetch their descriptors and both shapes first, then compute, so
// the LDS latency of a chunk overlaps the others instead of adding up
constexpr int BQ = 4;
template <int EW>
CX_DEV void ph_B_analytic(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane) {
  using namespace cx;
  const SceneHdr& sc = c.sh;
  const int ni = c.nc * EW;
  for (int base = 0; base < ni; base += BQ * WAVE) {
    uint32_t dw[BQ];
    float ga[BQ][4], gb[BQ][4];
#pragma unroll
    for (int q = 0; q < BQ; ++q) {
      const int w0 = base + q * WAVE + lane, w = w0 < ni ? w0 : ni - 1;  // clamped: every read in range
      dw[q] = t.tb[sc.o_cdesc + 2 * (w / EW)];
    }
#pragma unroll
    for (int q = 0; q < BQ; ++q) {
      const int w0 = base + q * WAVE + lane, w = w0 < ni ? w0 : ni - 1;
      const int e = w % EW;
      const int wa = c.L.world + (int)(dw[q] & 1023u), wb = c.L.world + (int)((dw[q] >> 10) & 1023u);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        ga[q][k] = t.f(wa + k, e);
        gb[q][k] = t.f(wb + k, e);
      }
    }
#pragma unroll
    for (int q = 0; q < BQ; ++q) {
      const int w = base + q * WAVE + lane, e = w % EW, ci = w / EW;
      if (w >= ni || env0 + e >= a.B) continue;
      CXK_STAT(b_items, 1);
      Shape A, Bs;
      A.kind = (int)((dw[q] >> 23) & 3u);
      Bs.kind = (int)((dw[q] >> 25) & 3u);
      A.n = Bs.n = 0;
#pragma unroll
      for (int k = 0; k < 2 * MAXV; ++k) {
        A.w[k] = k < 4 ? ga[q][k] : 0.0f;
        Bs.w[k] = k < 4 ? gb[q][k] : 0.0f;
      }
      uint32_t er = 0u;
      const Contact ct = run_contact_set<FNS_ANALYTIC>((int)((dw[q] >> 20) & 7u), A, Bs, narrow_of(sc), &er,
                                                       ((dw[q] >> 27) & 1u) != 0u);
      const int co = c.L.con + 4 * ci;
      t.f(co + 0, e) = ct.pen.x;
      t.f(co + 1, e) = ct.pen.y;
      t.f(co + 2, e) = ct.cp.x;
      t.f(co + 3, e) = ct.cp.y;
      if (!(isn(ct.cp.x) || isn(ct.cp.y))) {
        lds_or(t.w(c.L.vm + (ci >> 5), e), 1u << (ci & 31));
      }
      if (er) {
        lds_or(t.w(c.L.err, e), er);
      }
    }
  }
}
// phases A, T and B as ONE phase for the forward programs of analytic
// (circle / AABB) scenes.  Circles and AABBs transform by translation only
// (cotix/_convex_shapes.py:37-41,113-117), so a contact item builds both world
// parts itself from the launch-constant local geometry and its bodies'
// post-Euler positions -- p + v dt, phase A's expression on the same
// operands -- instead of reading phase T's world parts: every LDS read of the
// phase (descriptors, bodies, local geometry, the pre-Euler state) is issued
// before phase A's writes, one round trip for the three phases, and the
// world parts are never stored (no forward phase of these scenes reads them).
// The phase's per-lane registers between its three stages (fetch, phase A,
// contacts): on the GPU they stay in VGPRs (WaveRun::staged runs the stages
// back to back on the lane); the host emulation keeps one per lane.
// chunks of 64 items prefetched.  Measured (r04e): with 2 the box world
// (84 items) runs fused, 1.03x; RoboCup (160 items, 3 chunks) runs A, T, B
// as phases -- fused it is 0.96x (the fetch holds 3 x 18 words per lane and
// the contact work no longer overlaps phase A's writes)
#ifndef COTIX_AB_CHUNKS  // build-time A/B knob of the tooling (tools/gpu_iter.sh)
#define COTIX_AB_CHUNKS 2
#endif
constexpr int ABQ = COTIX_AB_CHUNKS;
struct ABRegs {
  uint32_t dw[ABQ], bw[ABQ];
  float ga[ABQ][4], gb[ABQ][4], pa[ABQ][4], pb[ABQ][4];  // local geometry; px, py, vx, vy of the bodies
};
template <int EW>
CX_DEV int ab_chunks(const KArgs& a, const Ctx& c) {
  return (a.stages & COTIX_STAGE_COLLIDER) ? (c.nc * EW + WAVE - 1) / WAVE : 0;
}
// stage 1: every LDS read of the phase (the pre-Euler state; DEFER: an env's
// restart state where its restart is pending, run_wave's SDEFER)
template <int EW, bool DEFER = false>
CX_DEV void ab_fetch(const KArgs& a, const Ctx& c, Tile<EW> t, int lane, ABRegs& r) {
  const SceneHdr& sc = c.sh;
  const int ni = c.nc * EW, nch = ab_chunks<EW>(a, c);
#pragma unroll
  for (int q = 0; q < ABQ; ++q) {
    if (q >= nch) continue;  // uniform
    const int w0 = q * WAVE + lane, w = w0 < ni ? w0 : ni - 1;  // clamped: every read in range
    r.dw[q] = t.tb[sc.o_cdesc + 2 * (w / EW)];
    r.bw[q] = t.tb[sc.o_cbody + w / EW];
  }
#pragma unroll
  for (int q = 0; q < ABQ; ++q) {
    if (q >= nch) continue;
    const int w0 = q * WAVE + lane, w = w0 < ni ? w0 : ni - 1, e = w % EW;
    // analytic scenes: a part's world offset is its local-geometry offset (4 words per part)
    const int la = c.L.geo + (int)(r.dw[q] & 1023u), lb = c.L.geo + (int)((r.dw[q] >> 10) & 1023u);
    const int base = DEFER && restart_deferred(a) && t.w(c.L.rflag, e) != 0u ? c.L.rst : c.L.dyn;
    const int oa = base + 6 * (int)(r.bw[q] & 255u), ob = base + 6 * (int)((r.bw[q] >> 8) & 255u);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      r.ga[q][k] = t.f(la + k, e);
      r.gb[q][k] = t.f(lb + k, e);
      r.pa[q][k] = t.f(oa + k, e);
      r.pb[q][k] = t.f(ob + k, e);
    }
  }
}
// one analytic contact item from its descriptor, its parts' local geometry
// and its bodies' post-Euler positions: the translate-only transforms of
// phase T (circle: (r, cx + px, cy + py); AABB: lo + p, up + p), the contact,
// its words and valid bit
template <int EW>
CX_DEV void ab_item(const KArgs& a, const Ctx& c, Tile<EW> t, int e, int ci, uint32_t dw, const float* ga,
                    const float* gb, float pxa, float pya, float pxb, float pyb) {
  using namespace cx;
  CXK_STAT(b_items, 1);
  Shape A, Bs;
  A.kind = (int)((dw >> 23) & 3u);
  Bs.kind = (int)((dw >> 25) & 3u);
  A.n = Bs.n = 0;
  const bool ca = A.kind == KIND_CIRCLE, cb = Bs.kind == KIND_CIRCLE;
#pragma unroll
  for (int k = 0; k < 2 * MAXV; ++k) A.w[k] = Bs.w[k] = 0.0f;
  A.w[0] = ca ? ga[0] : ga[0] + pxa;
  A.w[1] = ca ? ga[1] + pxa : ga[1] + pya;
  A.w[2] = ca ? ga[2] + pya : ga[2] + pxa;
  A.w[3] = ca ? ga[3] : ga[3] + pya;
  Bs.w[0] = cb ? gb[0] : gb[0] + pxb;
  Bs.w[1] = cb ? gb[1] + pxb : gb[1] + pyb;
  Bs.w[2] = cb ? gb[2] + pyb : gb[2] + pxb;
  Bs.w[3] = cb ? gb[3] : gb[3] + pyb;
  uint32_t er = 0u;
  const Contact ct = run_contact_set<FNS_ANALYTIC>((int)((dw >> 20) & 7u), A, Bs, narrow_of(c.sh), &er,
                                                   ((dw >> 27) & 1u) != 0u);
  const int co = c.L.con + 4 * ci;
  t.f(co + 0, e) = ct.pen.x;
  t.f(co + 1, e) = ct.pen.y;
  t.f(co + 2, e) = ct.cp.x;
  t.f(co + 3, e) = ct.cp.y;
  if (!(isn(ct.cp.x) || isn(ct.cp.y))) lds_or(t.w(c.L.vm + (ci >> 5), e), 1u << (ci & 31));
  if (er) lds_or(t.w(c.L.err, e), er);
}
// stage 3: the contacts from the fetched words (post-Euler positions p + v dt,
// euler_item's expression on the same operands)
template <int EW>
CX_DEV void ab_contacts(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane, const ABRegs& r) {
  const int ni = c.nc * EW, nch = ab_chunks<EW>(a, c);
  const bool eul = (a.stages & COTIX_STAGE_EULER) != 0;
#pragma unroll
  for (int q = 0; q < ABQ; ++q) {
    if (q >= nch) continue;
    const int w = q * WAVE + lane, e = w % EW, ci = w / EW;
    if (w >= ni || env0 + e >= a.B) continue;
    const float* pa = r.pa[q];
    const float* pb = r.pb[q];
    ab_item<EW>(a, c, t, e, ci, r.dw[q], r.ga[q], r.gb[q], eul ? pa[0] + pa[2] * a.dt : pa[0],
                eul ? pa[1] + pa[3] * a.dt : pa[1], eul ? pb[0] + pb[2] * a.dt : pb[0],
                eul ? pb[1] + pb[3] * a.dt : pb[1]);
  }
}
// Phase B of the analytic forward programs with more chunks than the fused
// form takes (RoboCup: 160 items, 3 chunks): every launch-constant word of an
// item -- its descriptor, its bodies, both parts' local geometry -- is read
// ONCE per launch into the lane's registers (BConst, before the step loop);
// a step's phase B then reads only its bodies' post-Euler positions (one LDS
// round trip) and builds the world parts itself, so phase T (whose world
// parts no forward phase of these scenes reads otherwise) does not run.
constexpr int HQ = 4;  // chunks of 64 items held in registers
#ifndef COTIX_BCONST_MIN_STEPS  // build-time A/B knob of the tooling: the fewest steps per launch that use it
#define COTIX_BCONST_MIN_STEPS 1
#endif
struct BConst {
  uint32_t dw[HQ], bw[HQ];
  float ga[HQ][4], gb[HQ][4];
};
template <int EW>
CX_DEV int bc_chunks(const Ctx& c) {
  return (c.nc * EW + WAVE - 1) / WAVE;
}
template <int EW>
CX_DEV void bc_fetch(const Ctx& c, Tile<EW> t, int lane, BConst& r) {
  const SceneHdr& sc = c.sh;
  const int ni = c.nc * EW, nch = bc_chunks<EW>(c);
#pragma unroll
  for (int q = 0; q < HQ; ++q) {
    r.dw[q] = r.bw[q] = 0u;
    if (q >= nch) continue;  // uniform
    const int w0 = q * WAVE + lane, w = w0 < ni ? w0 : ni - 1;  // clamped: every read in range
    r.dw[q] = t.tb[sc.o_cdesc + 2 * (w / EW)];
    r.bw[q] = t.tb[sc.o_cbody + w / EW];
  }
#pragma unroll
  for (int q = 0; q < HQ; ++q) {
    if (q >= nch) continue;
    const int w0 = q * WAVE + lane, w = w0 < ni ? w0 : ni - 1, e = w % EW;
    // analytic scenes: a part's world offset is its local-geometry offset (4 words per part)
    const int la = c.L.geo + (int)(r.dw[q] & 1023u), lb = c.L.geo + (int)((r.dw[q] >> 10) & 1023u);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      r.ga[q][k] = t.f(la + k, e);
      r.gb[q][k] = t.f(lb + k, e);
    }
  }
}
template <int EW>
CX_DEV void ph_B_const(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane, const BConst& r) {
  const int ni = c.nc * EW, nch = bc_chunks<EW>(c);
  float px[HQ][2][2];  // every chunk's positions read before any is used (one round trip)
#pragma unroll
  for (int q = 0; q < HQ; ++q) {
    if (q >= nch) continue;
    const int w0 = q * WAVE + lane, w = w0 < ni ? w0 : ni - 1, e = w % EW;
    const int oa = c.L.dyn + 6 * (int)(r.bw[q] & 255u), ob = c.L.dyn + 6 * (int)((r.bw[q] >> 8) & 255u);
    px[q][0][0] = t.f(oa, e);
    px[q][0][1] = t.f(oa + 1, e);
    px[q][1][0] = t.f(ob, e);
    px[q][1][1] = t.f(ob + 1, e);
  }
#pragma unroll
  for (int q = 0; q < HQ; ++q) {
    if (q >= nch) continue;
    const int w = q * WAVE + lane, e = w % EW, ci = w / EW;
    if (w >= ni || env0 + e >= a.B) continue;
    ab_item<EW>(a, c, t, e, ci, r.dw[q], r.ga[q], r.gb[q], px[q][0][0], px[q][0][1], px[q][1][0], px[q][1][1]);
  }
}
template <int EW, int FNSET, bool TAPE = false>
CX_DEV void ph_B(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane, int step = 0) {
  if constexpr (FNSET == FNS_ANALYTIC) {
    ph_B_analytic<EW>(a, c, t, env0, lane);
    return;
  }
  for (int w = lane; w < c.nc * EW; w += WAVE) {
    if ((FNSET & FNS_CONVEX) != 0 && c.sh.poly) t.ws[c.W.cf_flag + w] = 0u;
    b_item<EW, FNSET, TAPE>(a, c, t, env0, lane, w, step);
  }
}

// phase B with the broadphase (COTIX_STAGE_BROADPHASE, polygon scenes; the
// exactness argument is in DESIGN.md section 3).  BP0: a polygon pair
// (polygon x polygon, AABB x polygon) whose world AABBs are separated by
// more than the margin 2^-8 * S + 2^-16 (S = the largest coordinate
// magnitude of the two shapes) and whose world shapes pass bp_guard gets the
// no-contact result without GJK, EPA or contact points -- then no vertex is
// contained and no edge pair intersects in _contact_from_edges
// (cotix/_contacts.py:205-267), with the rounding of f32 included, so the
// reference's contact point is NaN and the candidate never writes.  Every
// other item is flagged for the B list (BP1) that BP2 runs at full lane width.
// The broadphase exactness argument ("Broadphase
// exactness") needs, besides the gap, conditions on the pair's WORLD shapes
// (the f32 vertices the reference works on):
//  (P) every polygon strictly convex with no too-sharp vertex -- checked once
//      per rebuilt part by ph_TV4, which leaves a NaN edge direction when not;
//  (E) no edge of A within |cross(d_a, d_b)| <= 2^-9 |d_a|_1 |d_b|_1 of
//      parallel to an edge of B (AABB edges: the axes).
// (E) on the pseudo-angles q of ph_TV4: for l1-unit vectors a, b in the
// upper half plane and the line distance delta = min(|qa - qb|, 2 - |qa - qb|)
// (<= 1), |cross(a, b)| >= delta - delta^2 / 2 (equality-checked case split in
// DESIGN.md), so delta > 2^-9 + 2^-16 -- with q rounded by at most 2^-22 --
// certifies |cross(d_a, d_b)| > 2^-9 |d_a|_1 |d_b|_1 exactly.  A failed
// vertex's pseudo-angle (2^100) fails the test.  False when it cannot
// certify (the pair takes the full path).
template <int EW>
CX_DEV bool bp_guard(const Ctx& c, Tile<EW> t, int e, int pa, int na, int pb, int nb) {
  using namespace cx;
  // the part with fewer edges on the outer side: at most pminv of them
  // (scene constants; LunarLander 4 x 6)
  const bool sw = nb < na;
  const int p0 = sw ? pb : pa, n0 = sw ? nb : na, p1 = sw ? pa : pb, n1 = sw ? na : nb;
  const int mv = c.sh.maxv > 2 ? c.sh.maxv : 2, m0 = c.sh.pminv > 2 ? c.sh.pminv : 2;
  // every read issued before any test; indices past a part's edge count
  // repeat its edge 0 (a repeated test changes nothing), so the tests need no
  // masks: dq in (T, 2 - T) <=> ||dq| - 1| < 1 - T, and the largest
  // ||dq| - 1| over the pairs decides (a failed vertex's 2^100 gives a huge
  // value against a finite q and 1 against itself: fails either way)
  float qa[MAXV], qb[MAXV];
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    if (j < m0) qa[j] = t.f(p0 + (j < n0 ? j : 0), e);
    if (j < mv) qb[j] = t.f(p1 + (j < n1 ? j : 0), e);
  }
  float m = 0.0f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i)
    if (i < m0) {
#pragma unroll
      for (int j = 0; j < MAXV; ++j)
        if (j < mv) m = __builtin_fmaxf(m, __builtin_fabsf(__builtin_fabsf(qa[i] - qb[j]) - 1.0f));
    }
  return m < 0.9980316162109375f;  // 1 - (2^-9 + 2^-16)
}

// mutation knobs for the tests only (tests/test_broadphase_cpu.py builds the
// host emulation with them); the library is always built with the defaults
#ifndef COTIX_BP_MARGIN_MUL
#define COTIX_BP_MARGIN_MUL 1.0f
#endif
#ifndef COTIX_BP_GUARD
#define COTIX_BP_GUARD 1
#endif
template <int EW>
CX_DEV void ph_BP0(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane) {
  using namespace cx;
  const SceneHdr& sc = c.sh;
  const int ni = c.nc * EW;
  if (lane == 0) {  // this step's B-list mode: lane pairs when the last step ran an EPA (contacts)
    t.ws[c.W.bl_mode] = t.ws[c.W.bl_epa];
    t.ws[c.W.bl_epa] = 0u;
  }
  uint32_t nlist = 0u;  // the B list is compacted here (in-register ballots)
  // BQ chunks at a time: every chunk's descriptors, then every box, are read
  // before any is used (the chunks' LDS latencies overlap)
  for (int base = 0; base < c.W.bl_pad; base += BQ * WAVE) {
    uint32_t d1[BQ], kq[BQ] = {};
    bool poly[BQ];
    float A[BQ][4], B[BQ][4];
#pragma unroll
    for (int q = 0; q < BQ; ++q) {
      const int w0 = base + q * WAVE + lane, w = w0 < ni ? w0 : ni - 1;  // clamped: every read in range
      const uint32_t d0w = t.tb[sc.o_cdesc + 2 * (w / EW)];
      d1[q] = t.tb[sc.o_cdesc + 2 * (w / EW) + 1];
      const int fn = (int)((d0w >> 20) & 7u);
      poly[q] = (fn == FN_POLY_POLY) | (fn == FN_AABB_POLY);
    }
#pragma unroll
    for (int q = 0; q < BQ; ++q) {
      const int w0 = base + q * WAVE + lane, w = w0 < ni ? w0 : ni - 1;
      const int e = w % EW;
      // the parts' world AABBs, built with the world parts in phase T
      const int ba = c.L.pbox + 4 * (int)((d1[q] >> 16) & 255u), bb = c.L.pbox + 4 * (int)(d1[q] >> 24);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        A[q][k] = t.f(ba + k, e);
        B[q][k] = t.f(bb + k, e);
      }
    }
#pragma unroll
    for (int q = 0; q < BQ; ++q) {
      const int w = base + q * WAVE + lane;
      if (w >= c.W.bl_pad) continue;
      uint32_t keep = 0u;
      if (w < ni) {
        t.ws[c.W.cf_flag + w] = 0u;
        const int e = w % EW, ci = w / EW;
        if (env0 + e < a.B) {
          keep = 1u;
          // S and the gap with NaN-propagating max: any NaN box word keeps the full path
          float S = 0.0f;
#pragma unroll
          for (int k = 0; k < 4; ++k) S = cx::fmax_(S, cx::fmax_(__builtin_fabsf(A[q][k]), __builtin_fabsf(B[q][k])));
          const float margin = (S * 0.00390625f + 1.52587890625e-05f) * COTIX_BP_MARGIN_MUL;  // 2^-8 S + 2^-16
          const float gap = cx::fmax_(cx::fmax_(B[q][0] - A[q][2], A[q][0] - B[q][2]),
                                      cx::fmax_(B[q][1] - A[q][3], A[q][1] - B[q][3]));
          bool skip = poly[q] && gap > margin;  // false for NaN
          if (skip) {  // the argument's shape conditions, on the world shapes' edge directions (ph_TV4)
            const uint32_t d0w = t.tb[sc.o_cdesc + 2 * ci];
            const int pa = c.L.pedge + (int)(d0w & 1023u) / 2, pb = c.L.pedge + (int)((d0w >> 10) & 1023u) / 2;
            const int na = ((d0w >> 23) & 3u) == (uint32_t)KIND_POLY ? (int)(d1[q] & 255u) : 2;
            const int nb = ((d0w >> 25) & 3u) == (uint32_t)KIND_POLY ? (int)((d1[q] >> 8) & 255u) : 2;
            skip = COTIX_BP_GUARD ? bp_guard<EW>(c, t, e, pa, na, pb, nb) : true;
            CXK_STAT(bp_cand, 1);
            CXK_STAT(bp_guard_fail, skip ? 0 : 1);
          }
          if (skip) {
            keep = 0u;
            const int co = c.L.con + 4 * ci;
            t.f(co + 0, e) = 0.0f;
            t.f(co + 1, e) = 0.0f;
            t.f(co + 2, e) = qnan();
            t.f(co + 3, e) = qnan();
          }
        }
      }
      t.ws[c.W.bl_flag + w] = keep;
      kq[q] = keep;
    }
#pragma unroll
    for (int q = 0; q < BQ; ++q) {  // chunk by chunk, in item order
      if (base + q * WAVE >= c.W.bl_pad) continue;  // uniform
      const uint64_t mask = ballot(kq[q] != 0u);
      if (kq[q] != 0u) t.ws[c.W.bl_list + nlist + popc64(mask & lanes_below(lane))] = (uint32_t)(base + q * WAVE + lane);
      nlist += (uint32_t)popc64(mask);
    }
  }
  if (lane == 0) t.ws[c.W.bl_n] = nlist;
}
// ---------------------------------------------------------------------------
// GJK + EPA of a polygon pair on a PAIR of adjacent lanes (GPU, polygon-only
// program): lane h = 0 holds polygon A, lane h = 1 polygon B; every
// Minkowski support is one support per lane (A in d on lane 0, B in -d on
// lane 1) whose results the pair swaps with a DPP move, so both lanes form
// the same difference bits and then run the same GJK / EPA arithmetic in
// lockstep (identical values: identical control flow).  Half the support
// work of the one-lane form on the critical path; each lane keeps its own
// EPA edge column.  The host emulation runs the same pair form (its SIMT
// runtime resolves the pair exchanges).
// ---------------------------------------------------------------------------
#ifdef COTIX_NO_PAIR_GJK  // A/B tooling builds only
constexpr bool PAIR_GJK = false;
#else
constexpr bool PAIR_GJK = true;
#endif
CX_DEV float pair_swap(float x) { return pair_swap_f32(x); }
struct PairSide {
  const cx::Shape& mine;  // A on lane 0, B on lane 1
  int h;
};
CX_DEV cx::v2 minkowski(const PairSide& p, const PairSide&, cx::v2 d) {
  const cx::v2 s = cx::support(cx::PolyRef{p.mine}, p.h ? cx::neg(d) : d);
  const cx::v2 o = cx::v2{pair_swap(s.x), pair_swap(s.y)};
  return p.h ? cx::sub(o, s) : cx::sub(s, o);  // support(A, d) - support(B, -d) on both lanes
}
// EPA (cx::epa, cotix/_collisions.py:115-273) on the lane pair: besides the
// supports, the pair splits the two new edges' distances (lane 0 the
// A-side edge, lane 1 the B-side one), the two components of the split
// direction's division, and the argmin over the edge buffer (lane h scans
// the entries k = h mod 2; the halves combine as first NaN, else smallest
// value, then smaller index -- the order the sequential first-min scan
// induces), exchanging the results with DPP moves.  Buffer entries not yet
// written read as the zero edge (no zero-fill of the column).  The same
// expressions on the same operands as cx::epa: bit-identical.
template <int NE>
CX_DEV cx::v2 epa_pair(const PairSide& ps, int h, const cx::v2* simplex, int iters, float* col,
                       cx::v2* edge = nullptr) {
  using namespace cx;
  constexpr int NH = (NE + 1) / 2;
  EdgeCol es{col, WAVE};
  const v2 z = v2{0.0f, 0.0f};
  // this lane's half of the distance cache: dh[j] = dist of entry 2j + h
  float dh[NH];
  es.s0(0, simplex[0]); es.s1(0, simplex[1]);
  es.s0(1, simplex[1]); es.s1(1, simplex[2]);
  es.s0(2, simplex[2]); es.s1(2, simplex[0]);
  uint32_t wm = 7u;  // bit k: entry k holds an edge; the others are the zero edge
  const int ne = iters + 3;
  const v2 sim[3] = {simplex[0], simplex[1], simplex[2]};
  const float dzero = edge_dist(z, z);
  {
    const float d01 = edge_dist(h ? sim[1] : sim[0], h ? sim[2] : sim[1]);  // entry h
    const float d2 = edge_dist(sim[2], sim[0]);                             // entry 2 (lane 0)
#pragma unroll
    for (int j = 0; j < NH; ++j) {
      const int k = 2 * j + h;
      dh[j] = j == 0 ? d01 : (k == 2 ? d2 : ((k < ne) ? dzero : finf()));
    }
  }
  float bd = 0.0f;
  auto argmin_d = [&]() {
    int nanidx = NE, b = h;
    float bv = dh[0];  // ne >= 3: entries 0 and 1 are live
#pragma unroll
    for (int j = 1; j < NH; ++j) {
      const int k = 2 * j + h;
      const bool lt = k < ne && dh[j] < bv;
      bv = lt ? dh[j] : bv;
      b = lt ? k : b;
    }
#pragma unroll
    for (int j = NH - 1; j >= 0; --j) {
      const int k = 2 * j + h;
      nanidx = (k < ne && isn(dh[j])) ? k : nanidx;
    }
    const int onan = (int)pair_swap_u32((uint32_t)nanidx);
    const int ob = (int)pair_swap_u32((uint32_t)b);
    const float obv = pair_swap(bv);
    const int fn = nanidx < onan ? nanidx : onan;
    const bool mine = bv < obv || (!(obv < bv) && b < ob);  // (no NaN among the live entries here)
    bd = fn < NE ? qnan() : (mine ? bv : obv);
    return fn < NE ? fn : (mine ? b : ob);
  };
  // unconditional reads (the column may hold an older item's words), selected
  auto g0 = [&](int k) { const v2 v = es.g0(k); return ((wm >> k) & 1u) ? v : z; };
  auto g1 = [&](int k) { const v2 v = es.g1(k); return ((wm >> k) & 1u) ? v : z; };
  int bei = argmin_d();
  v2 best0 = g0(bei), best1 = g1(bei);
  v2 newp = simplex[2];
  v2 pn = fnormal(sub(simplex[0], simplex[1]));
  pn = divs(pn, nrm(pn));
  float pd = pair_swap(h ? 0.0f : dh[0]);  // dist of entry 0 (lane 0's), on lane 1 ...
  pd = h ? pd : dh[0];                     // ... and lane 0
  bool pz = simplex[0].x == 0.0f && simplex[0].y == 0.0f && simplex[1].x == 0.0f && simplex[1].y == 0.0f;
  for (int i = 0; i < iters; ++i) {
    bool c1 = sumsq(sub(best0, best1)) > 1e-9f;
    bool c2 = crs(best0, best1) >= 0.0f;
    float d = dot(newp, pn);
    float ed = pz ? 0.0f : __builtin_sqrtf(pd);
    bool c4 = (d - ed > 1e-6f) || (d <= 0.0f);
    if (!(c4 && !vnan(best0) && !vnan(best1) && c1 && c2)) break;
    const v2 fnv = fnormal(sub(best0, best1));
    const float len = nrm(fnv);
    const float mc = (h ? fnv.y : fnv.x) / len, oc = pair_swap(mc);  // divs(n, nrm(n)), one component per lane
    const v2 n = h ? v2{oc, mc} : v2{mc, oc};
    newp = minkowski(ps, ps, n);
    const int slot = i + 3;
    // lane 0 the A-side edge (best0, newp), lane 1 the B-side edge (newp, best1)
    const float md = edge_dist(h ? newp : best0, h ? best1 : newp), od = pair_swap(md);
    const float dA = h ? od : md, dB = h ? md : od;
    if (!((wm >> bei) & 1u)) es.s0(bei, z);  // a zero edge taken as the best: its first word stays zero
    es.s1(bei, newp);
    es.s0(slot, newp);
    es.s1(slot, best1);
    wm |= (1u << bei) | (1u << slot);
#pragma unroll
    for (int j = 0; j < NH; ++j) {
      const int k = 2 * j + h;
      if (k == bei) dh[j] = dA;
      if (k == slot) dh[j] = dB;
    }
    pn = n;
    pd = bd;
    pz = best0.x == 0.0f && best0.y == 0.0f && best1.x == 0.0f && best1.y == 0.0f;
    bei = argmin_d();
    best0 = g0(bei);
    best1 = g1(bei);
  }
  if (edge != nullptr) {  // EPA's final edge (the rollout's tape, as cx::epa's)
    edge[0] = best0;
    edge[1] = best1;
  }
  return closest_on_edge_to_origin(best0, best1);
}
CX_DEV bool gjk_epa_pair(const cx::Shape& mine, int h, int na, int nb, const cx::NarrowParams& np, bool need_pen,
                         cx::v2* pen, float* col, cx::v2* edge = nullptr) {
  using namespace cx;
  const PairSide ps{mine, h};
  v2 simplex[3];
  *pen = v2{0.0f, 0.0f};
  if (!gjk(ps, ps, np.d0, simplex, np.gjk_steps)) return false;
  if (!need_pen) return true;
  const int it0 = na + nb + 1, iters = it0 < np.epa_cap ? it0 : np.epa_cap;  // min(48, ...), cotix/_contacts.py:295
  *pen = iters + 3 <= 14 ? epa_pair<14>(ps, h, simplex, iters, col, edge)
                         : epa_pair<20>(ps, h, simplex, iters, col, edge);
  return true;
}
// the B list items of the polygon-only program run on lane pairs
template <int FNSET>
constexpr bool b_pairs() {
  return PAIR_GJK && FNSET == (FNS_ANALYTIC | FNS_CONVEX);
}
// item w on the lane pair (lane, lane ^ 1); h = lane & 1
template <int EW, int FNSET, bool TAPE = false>
CX_DEV void b_item_pair(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane, int w, int step = 0) {
  using namespace cx;
  const SceneHdr& sc = c.sh;
  const int h = lane & 1;
  const int e = w % EW, ci = w / EW, g = env0 + e;
  if (g >= a.B) return;  // both lanes of the pair
  const uint32_t d0w = t.tb[sc.o_cdesc + 2 * ci], d1w = t.tb[sc.o_cdesc + 2 * ci + 1];
  const int fn = (int)((d0w >> 20) & 7u);
  if (fn != FN_POLY_POLY) {  // (not in the reference scenes) the one-lane form on lane 0
    if (h == 0) b_item<EW, FNSET, TAPE>(a, c, t, env0, lane, w, step);
    return;
  }
  CXK_STAT(b_items, h == 0 ? 1 : 0);
  const int na = (int)(d1w & 255u), nb = (int)((d1w >> 8) & 255u);
  const int wo = c.L.world + (int)(h ? (d0w >> 10) & 1023u : d0w & 1023u);
  Shape S;
  S.kind = KIND_POLY;
  S.n = h ? nb : na;
#pragma unroll
  for (int k = 0; k < 2 * MAXV; ++k) S.w[k] = t.f(wo + k, e);  // the tile's world region has 2*MAXV words of slack
  const bool self = ((d0w >> 27) & 1u) != 0u;
  float* col = reinterpret_cast<float*>(t.ws + c.W.epa + lane);
  Contact ct;
  v2 edge[2];
  const bool hit = CXK_SKIP(a, 64) ? (ct.pen = v2{0.0f, 0.0f}, true)  // timing only: no GJK / EPA
                                     : gjk_epa_pair(S, h, na, nb, narrow_of(sc), !self, &ct.pen, col,
                                                    TAPE ? edge : nullptr);
  if (h != 0) return;
  CXK_STAT(epa_runs, hit && !self ? 1 : 0);
  if (TAPE && a.tape != nullptr && hit && !self) {  // EPA's final edge to the tape (b_item's words)
    const int o = 5 * c.nb + 4 * ci;
    const float ev[4] = {edge[0].x, edge[0].y, edge[1].x, edge[1].y};
#pragma unroll
    for (int q = 0; q < 4; ++q) a.tape[row_at(a.B, a.tw, step, o + q, g)] = __float_as_uint(ev[q]);
  }
  ct.cp = v2{qnan(), qnan()};
  if (hit && self && self_cp_finite(S)) ct.cp = v2{0.0f, 0.0f};  // S is A on lane 0 (see b_item)
  else if (hit) t.ws[c.W.cf_flag + w] = 1u;
  if (hit && !self) t.ws[c.W.bl_epa] = 1u;
  const int co = c.L.con + 4 * ci;
  t.f(co + 0, e) = ct.pen.x;
  t.f(co + 1, e) = ct.pen.y;
  t.f(co + 2, e) = ct.cp.x;
  t.f(co + 3, e) = ct.cp.y;
  if (!(isn(ct.cp.x) || isn(ct.cp.y))) lds_or(t.w(c.L.vm + (ci >> 5), e), 1u << (ci & 31));
}
// BP2: round r of the B list, one item per lane (lane pairs: b_pairs)
// pairs: the step's mode (lane pairs pay off when EPA runs -- landers on the
// terrain -- and cost a little on GJK-only lists, e.g. the self pairs in flight)
template <int EW, int FNSET, bool TAPE = false>
CX_DEV void ph_BP2(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane, int r, bool pairs, int step = 0) {
  if (b_pairs<FNSET>() && pairs) {  // (the rollout's tape: EPA's edge from lane 0 of the pair)
    const int k = r * (WAVE / 2) + (lane >> 1);
    if (k < (int)t.ws[c.W.bl_n]) b_item_pair<EW, FNSET, TAPE>(a, c, t, env0, lane, (int)t.ws[c.W.bl_list + k], step);
  } else {
    const int k = r * WAVE + lane;
    if (k < (int)t.ws[c.W.bl_n]) b_item<EW, FNSET, TAPE>(a, c, t, env0, lane, (int)t.ws[c.W.bl_list + k], step);
  }
}

// phase F: deferred polygon contact points (contact_from_edges,
// cotix/_contacts.py:205-267).  Each colliding polygon item (contact, env)
// has |A| + |B| + |A||B| independent terms; batches of CFB items spread their
// terms over the 64 lanes (F2), then one lane per item sums its terms in the
// reference's order (F3), which is bit-identical to the serial loop.
// F0: compact the flagged items of chunk `chunk` into the item list
template <int EW>
CX_DEV void ph_F0(const Ctx& c, Tile<EW> t, int lane, int chunk) {
  const uint64_t mask = wave_ballot(t.ws + c.W.cf_flag + chunk * WAVE, lane);
  const uint32_t base = chunk == 0 ? 0u : t.ws[c.W.cf_n];
  if (t.ws[c.W.cf_flag + chunk * WAVE + lane] != 0u)
    t.ws[c.W.cf_list + base + popc64(mask & lanes_below(lane))] = (uint32_t)(chunk * WAVE + lane);
  if (lane == WAVE - 1) t.ws[c.W.cf_n] = base + (uint32_t)popc64(mask);
}
template <int EW>
CX_DEV void cf_shapes(const Ctx& c, Tile<EW> t, int id, cx::Shape* A, cx::Shape* B, int* wa, int* wb) {
  const SceneHdr& sc = c.sh;
  const int e = id % EW, ci = id / EW;
  const uint32_t d0w = t.tb[sc.o_cdesc + 2 * ci], d1w = t.tb[sc.o_cdesc + 2 * ci + 1];
  A->kind = (int)((d0w >> 23) & 3u);
  B->kind = (int)((d0w >> 25) & 3u);
  A->n = (int)(d1w & 255u);
  B->n = (int)((d1w >> 8) & 255u);
  *wa = c.L.world + (int)(d0w & 1023u);
  *wb = c.L.world + (int)((d0w >> 10) & 1023u);
#pragma unroll
  for (int k = 0; k < 2 * cx::MAXV; ++k) {
    A->w[k] = t.f(*wa + k, e);
    B->w[k] = t.f(*wb + k, e);
  }
}
// F1: term counts of the batch starting at item b
template <int EW>
CX_DEV void ph_F1(const Ctx& c, Tile<EW> t, int lane, int b) {
  if (lane >= CFB) return;
  const int n = (int)t.ws[c.W.cf_n];
  uint32_t cnt = 0u, cc = 0u;
  if (b + lane < n) {
    const int id = (int)t.ws[c.W.cf_list + b + lane];
    const SceneHdr& sc = c.sh;
    const int ci = id / EW;
    const uint32_t d0w = t.tb[sc.o_cdesc + 2 * ci], d1w = t.tb[sc.o_cdesc + 2 * ci + 1];
    const int na = ((d0w >> 23) & 3u) == (uint32_t)cx::KIND_AABB ? 4 : (int)(d1w & 255u);
    const int nb = ((d0w >> 25) & 3u) == (uint32_t)cx::KIND_AABB ? 4 : (int)((d1w >> 8) & 255u);
    cnt = (uint32_t)(na + nb + na * nb);
    cc = (uint32_t)(na + nb);
  }
  t.ws[c.W.cf_s + lane] = cnt;
  t.ws[c.W.cf_c + lane] = cc;
}
// F2: round r of the batch: lane -> one term; the containment terms
// (EDGE = false: vertex k of one shape in the other) and the edge-pair terms
// (EDGE = true) run in rounds of their own, so a round issues one of the two
// code paths, not both (the terms land at their index s either way)
template <int EW, bool EDGE>
CX_DEV void ph_F2(const Ctx& c, Tile<EW> t, int lane, int b, int r) {
  using namespace cx;
  const int g = r * WAVE + lane;
  int pre = 0, item = -1, off = 0;
#pragma unroll
  for (int i = 0; i < CFB; ++i) {
    const int cc = (int)t.ws[c.W.cf_c + i];
    const int si = EDGE ? (int)t.ws[c.W.cf_s + i] - cc : cc;
    if (item < 0 && g < pre + si) {
      item = i;
      off = EDGE ? cc : 0;
    }
    if (item < 0) pre += si;
  }
  if (item < 0) return;
  const int id = (int)t.ws[c.W.cf_list + b + item], e = id % EW;
  Shape A, B;
  int wa, wb;
  cf_shapes<EW>(c, t, id, &A, &B, &wa, &wb);
  // per-lane vertex picks straight from the LDS world tile
  auto va = [&](int k) { return v2{t.f(wa + 2 * k, e), t.f(wa + 2 * k + 1, e)}; };
  auto vb = [&](int k) { return v2{t.f(wb + 2 * k, e), t.f(wb + 2 * k + 1, e)}; };
  const int sidx = off + g - pre;
  const v2 x = EDGE ? cfe_term_edge(A, B, sidx, va, vb) : cfe_term_contain(A, B, sidx, va, vb);
  float* res = reinterpret_cast<float*>(t.ws + c.W.cf_res) + 2 * (item * CFS + sidx);
  res[0] = x.x;
  res[1] = x.y;
}
// F3: one lane per item sums its terms in order -> contact point, valid bit
template <int EW>
CX_DEV void ph_F3(const Ctx& c, Tile<EW> t, int lane, int b) {
  using namespace cx;
  if (lane >= CFB) return;
  const int n = (int)t.ws[c.W.cf_n];
  if (b + lane >= n) return;
  const int id = (int)t.ws[c.W.cf_list + b + lane], e = id % EW, ci = id / EW;
  const int S = (int)t.ws[c.W.cf_s + lane];
  const float* res = reinterpret_cast<const float*>(t.ws + c.W.cf_res) + 2 * lane * CFS;
  float cnt = 0.0f;
  v2 acc = v2{0.0f, 0.0f};
  for (int s0 = 0; s0 < S; s0 += 8) {  // fetch 8 terms, then add them in order
    float xs[8], ys[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      xs[q] = res[2 * (s0 + q)];
      ys[q] = res[2 * (s0 + q) + 1];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (s0 + q < S && !(isn(xs[q]) || isn(ys[q]))) {
        acc = add(acc, v2{xs[q], ys[q]});
        cnt = cnt + 1.0f;
      }
  }
  const v2 cp = cnt > 0.0f ? divs(acc, cnt) : v2{qnan(), qnan()};
  const int co = c.L.con + 4 * ci;
  t.f(co + 2, e) = cp.x;
  t.f(co + 3, e) = cp.y;
  if (!(isn(cp.x) || isn(cp.y))) {
    lds_or(t.w(c.L.vm + (ci >> 5), e), 1u << (ci & 31));
  }
}

// phase C: per cell, last passing candidate (cotix/_colliders.py:208-268).
// The reference scans N2 x N1 candidates forward, each non-NaN one writing
// its cell when its bernoulli draw passes, so a cell ends with its LAST
// passing candidate: we scan each cell's candidates in reverse and stop at
// the first pass.  The scan is wave-cooperative: active (env, cell) items
// are compacted into a list, and every round gives each remaining item
// G = 64 / n lanes that draw G consecutive candidates at once; a ballot
// picks each item's first passing one, unresolved items advance by G.
// C0: activity (a cell whose distinct contacts are all NaN never writes).
template <int EW>
CX_DEV void ph_C0(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane, int chunk) {
  using namespace cx;
  const SceneHdr& sc = c.sh;
  const int id = chunk * WAVE + lane;
  uint32_t flag = 0u;
  if (id < c.nl * EW) {
    const int e = id % EW, l = id / EW;
    if (env0 + e < a.B) {
      bool any = false;
      for (int q = 0; q < sc.nmw; ++q) any |= (t.tb[sc.o_cmask + l * sc.nmw + q] & t.w(c.L.vm + q, e)) != 0u;
      if (any) {
        flag = 1u;
        t.ws[WS_LIST + 2 * c.nl * EW + id] = 0u;  // scan position
      }
    }
  }
  t.ws[WS_FLAG + lane] = flag;
}
// C0b: append this chunk's active items to list 0
template <int EW>
CX_DEV void ph_C0b(const Ctx& c, Tile<EW> t, int lane, int chunk) {
  const uint64_t mask = wave_ballot(t.ws + WS_FLAG, lane);
  const uint32_t base = chunk == 0 ? 0u : t.ws[WS_N];
  if (t.ws[WS_FLAG + lane] != 0u) t.ws[WS_LIST + base + popc64(mask & lanes_below(lane))] = (uint32_t)(chunk * WAVE + lane);
  if (lane == WAVE - 1) t.ws[WS_N] = base + (uint32_t)popc64(mask);  // last lane: the host emulation runs it last
  (void)c;
}
// R1: every lane draws one candidate of its item
template <int EW>
CX_DEV void ph_C1(const KArgs& a, const Ctx& c, Tile<EW> t, int lane, int par, int kso) {
  using namespace cx;
  const SceneHdr& sc = c.sh;
  const int NI = c.nl * EW;
  const uint32_t* list = t.ws + WS_LIST + par * NI;
  const int n = (int)t.ws[WS_N], np = n < WAVE ? n : WAVE, G = WAVE / np;
  const int slot = lane / G, q = lane % G;
  uint32_t pass = 0u;
  if (slot < np) {
    const int id = (int)list[slot], e = id % EW, l = id / EW;
    const int idx = (int)t.ws[WS_LIST + 2 * NI + id] + q;
    if (idx < t.ti(sc.o_ccnt + l)) {
      const uint32_t cd = t.tb[sc.o_cand + t.ti(sc.o_cbeg + l) + idx];
      const int i1 = cd & 511u, i2 = (cd >> 9) & 511u, cid = (cd >> 18) & 511u, ty = cd >> 27;
      const float cpx = t.f(c.L.con + 4 * cid + 2, e), cpy = t.f(c.L.con + 4 * cid + 3, e);
      if (!(isn(cpx) || isn(cpy))) {  // a NaN candidate never writes
        const key2 sk = key2{t.w(kso + 2 + 2 * ty, e), t.w(kso + 3 + 2 * ty, e)};
        const bool part = sc.prng != 0;
        const key2 k2 = split_at_l(sk, (uint32_t)t.ti(sc.o_tn2 + ty), (uint32_t)i2, part);  // :264
        const key2 k = split_at_l(k2, (uint32_t)t.ti(sc.o_tn1 + ty), (uint32_t)i1, part);   // :254
        pass = bernoulli_l(split_at_l(k, 2u, 0u, part), sc.pc, part) ? 1u : 0u;           // :222-223
      }
    }
  }
  (void)a;
  t.ws[WS_FLAG + lane] = pass;
  t.ws[WS_KEEP + lane] = 0u;
}
// R2: per item, the first passing draw writes the cell; else advance
template <int EW>
CX_DEV void ph_C2(const Ctx& c, Tile<EW> t, int lane, int par) {
  const SceneHdr& sc = c.sh;
  const uint64_t mask = wave_ballot(t.ws + WS_FLAG, lane);
  const int NI = c.nl * EW;
  const uint32_t* list = t.ws + WS_LIST + par * NI;
  const int n = (int)t.ws[WS_N], np = n < WAVE ? n : WAVE, G = WAVE / np;
  const int slot = lane / G, q = lane % G;
  if (q == 0 && slot < np) {
    const int id = (int)list[slot], e = id % EW, l = id / EW;
    const uint64_t gm = G == WAVE ? ~0ull : ((1ull << G) - 1ull);
    const uint64_t bits = (mask >> (slot * G)) & gm;
    uint32_t& pos = t.ws[WS_LIST + 2 * NI + id];
    if (bits != 0ull) {
      const int idx = (int)pos + __builtin_ctzll(bits);
      const uint32_t cd = t.tb[sc.o_cand + t.ti(sc.o_cbeg + l) + idx];
      t.w(c.L.m + t.ti(sc.o_ci + l) * c.nb + t.ti(sc.o_cj + l), e) = cd;  // the winning candidate word
    } else {
      pos = pos + (uint32_t)G;
      t.ws[WS_KEEP + slot] = (int)pos < t.ti(sc.o_ccnt + l) ? 1u : 0u;
    }
  }
}
// R3: compact the unresolved items into the other list
template <int EW>
CX_DEV void ph_C3(const Ctx& c, Tile<EW> t, int lane, int par) {
  const uint64_t mask = wave_ballot(t.ws + WS_KEEP, lane);
  const int NI = c.nl * EW;
  const uint32_t* cur = t.ws + WS_LIST + par * NI;
  uint32_t* nxt = t.ws + WS_LIST + (1 - par) * NI;
  const int n = (int)t.ws[WS_N];
  const int kept = popc64(mask);
  if (t.ws[WS_KEEP + lane] != 0u) nxt[popc64(mask & lanes_below(lane))] = cur[lane];
  for (int s2 = WAVE + lane; s2 < n; s2 += WAVE) nxt[kept + s2 - WAVE] = cur[s2];  // not drawn this round
  if (lane == WAVE - 1) t.ws[WS_N] = (uint32_t)(kept + (n > WAVE ? n - WAVE : 0));
}

// Phase C when the (cell, env) items fit two per lane (nl * EW <= 128): the
// whole scan is ONE phase (ph_M_fused).  Items id and id + 64 belong to lane
// id (their "owner"); the pending items are two 64-bit ballot masks.  Each
// round gives the first min(n, 64) pending items (in id order) G = 64 / min(n, 64)
// consecutive lanes ("drawers", at least one) in rank order, each drawing
// the next candidate of its item's scan; an owner then settles each of its
// items that drew from the pass ballot: the first passing draw of its G
// writes the cell (the reference's last passing candidate: the list is in
// reverse scan order), else its scan position advances by G; an item past
// rank 64 waits for a later round (its draws are the same candidates then).  Per-item state (scan position, candidate
// range, cell address) stays in the owner's registers; the owner publishes
// its range to its drawers in one LDS word per rank, and the winning
// candidate word comes back by a lane permute -- per round two dependent LDS
// round trips before the draws (slot word, candidate word), one permute
// after, no barrier.  (Draws on lane pairs -- two threefry blocks of a split
// per lane -- measured no gain, r04j: half the draws per round cost rounds.)
// (a draw's threefry chain does not wait for the candidate's validity: the
// contact-point read overlaps it, and a NaN candidate's draw is discarded --
// a bitwise AND, which the compiler cannot turn into a branch on the read)

// the uniform lanes-per-item G = 64 / n and the drawer's rank slot = lane / G
// without integer division: rcp is within 1 ulp, far inside the margins
// (64 / n is an integer or at least 1/64 from one; (lane + 1/2) / G at least
// 1/(2G) from one)
CX_DEV float rcp_approx(float x) {
#if defined(__HIP__)
  return __builtin_amdgcn_rcpf(x);
#else
  return 1.0f / x;
#endif
}
CX_DEV int lanes_per_item(int n) { return n >= WAVE ? 1 : (int)((float)WAVE * rcp_approx((float)n)); }
// the most items that draw in one round (64: one lane each at least); a
// smaller value is a test build's knob (tests/test_emu_cpu.py: the
// items-past-the-last-rank path with few items)
#ifndef COTIX_SCAN_RANKS
#define COTIX_SCAN_RANKS 64
#endif
CX_DEV int rank_of_lane(int lane, int G) { return (int)(((float)lane + 0.5f) * rcp_approx((float)G)); }

// M0: the item's activity (a cell whose distinct contacts are all NaN never writes)
template <int EW>
CX_DEV bool m0_active(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int id) {
  const SceneHdr& sc = c.sh;
  if (id >= c.nl * EW) return false;
  const int e = id % EW, l = id / EW;
  if (env0 + e >= a.B) return false;
  bool any = false;
  for (int q = 0; q < sc.nmw; ++q) any |= (t.tb[sc.o_cmask + l * sc.nmw + q] & t.w(c.L.vm + q, e)) != 0u;
  return any;
}
// a drawer's candidate: its item's next candidate word (slot word: the item's
// scan base | end << 12 | id << 25), 0xFFFFFFFF past the item's list; pass:
// the candidate's bernoulli draw passed and its contact is not NaN
template <int EW>
CX_DEV uint32_t m_draw(const Ctx& c, Tile<EW> t, uint32_t sw, int q, int kso, bool& pass) {
  using namespace cx;
  const SceneHdr& sc = c.sh;
  pass = false;
  const int base = (int)(sw & 4095u), end = (int)((sw >> 12) & 8191u), id = (int)(sw >> 25);
  const int e = id % EW, idx = base + q;
  if (idx >= end) return 0xFFFFFFFFu;
  const uint32_t cd = t.tb[sc.o_cand + idx];
  const int i1 = cd & 511u, i2 = (cd >> 9) & 511u, cid = (cd >> 18) & 511u, ty = cd >> 27;
  const float cpx = t.f(c.L.con + 4 * cid + 2, e), cpy = t.f(c.L.con + 4 * cid + 3, e);
  const key2 sk = key2{t.w(kso + 2 + 2 * ty, e), t.w(kso + 3 + 2 * ty, e)};
  const bool part = sc.prng != 0;
  const bool valid = !(isn(cpx) || isn(cpy));  // a NaN candidate never writes
  const key2 k2 = split_at_l(sk, (uint32_t)t.ti(sc.o_tn2 + ty), (uint32_t)i2, part);  // :264
  const key2 k = split_at_l(k2, (uint32_t)t.ti(sc.o_tn1 + ty), (uint32_t)i1, part);   // :254
  pass = bernoulli_l(split_at_l(k, 2u, 0u, part), sc.pc, part) & valid;              // :222-223
  CXK_STAT(draws, 1);
  CXK_STAT(valid_draws, valid ? 1 : 0);
  return cd;
}
// an owner's item (owner slot s of lane l: item id = l + 64 s)
struct MItem {
  int cb = 0, ce = 0, cell = 0, pos = 0, e = 0;
};
template <int EW>
CX_DEV MItem m_item(const Ctx& c, Tile<EW> t, int id) {
  const SceneHdr& sc = c.sh;
  MItem it;
  if (id < c.nl * EW) {
    const int l = id / EW;
    it.e = id % EW;
    it.cb = t.ti(sc.o_cbeg + l);
    it.ce = it.cb + t.ti(sc.o_ccnt + l);
    it.cell = c.L.m + t.ti(sc.o_ci + l) * c.nb + t.ti(sc.o_cj + l);
  }
  return it;
}
// an owner's launch-constant words, in registers for the whole launch
// (mc_fetch once, before the step loop): both owner items and the first two
// words of their cells' contact masks (every reference scene: nmw <= 2)
struct MConst {
  MItem it[2];
  uint32_t cm[2][2] = {{0u, 0u}, {0u, 0u}};
};
template <int EW>
CX_DEV void mc_fetch(const Ctx& c, Tile<EW> t, int lane, MConst& m) {
  const SceneHdr& sc = c.sh;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int id = lane + s * WAVE;
    if (s == 1 && c.nl * EW <= WAVE) continue;  // uniform
    m.it[s] = m_item<EW>(c, t, id);
    if (id < c.nl * EW)
      for (int q = 0; q < 2 && q < sc.nmw; ++q) m.cm[s][q] = t.tb[sc.o_cmask + (id / EW) * sc.nmw + q];
  }
}
// the item's activity from the held mask words (nmw <= 2) or the tables
template <int EW>
CX_DEV bool m0_active_c(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int id, const uint32_t* cm) {
  const SceneHdr& sc = c.sh;
  if (sc.nmw > 2) return m0_active<EW>(a, c, t, env0, id);
  if (id >= c.nl * EW) return false;
  const int e = id % EW;
  if (env0 + e >= a.B) return false;
  bool any = false;
  for (int q = 0; q < 2 && q < sc.nmw; ++q) any |= (cm[q] & t.w(c.L.vm + q, e)) != 0u;
  return any;
}
// an owner's item after a round's pass ballot pm: the cell word from the
// winning drawer (wcd, permuted), or the scan advances; returns "still pending"
template <int EW>
CX_DEV bool m_settle(Tile<EW> t, MItem& it, bool drew, uint64_t bits, uint32_t wcd, int G) {
  if (!drew) return true;  // (past the last rank: waits for a later round)
  if (bits != 0ull) {
    t.w(it.cell, it.e) = wcd;  // the winning candidate word
    return false;
  }
  it.pos += G;
  return it.cb + it.pos < it.ce;
}
template <int EW>
CX_DEV void ph_M_fused(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane, int kso, const MConst& mc) {
  const bool two = c.nl * EW > WAVE;  // uniform (a constant in the specialized kernels)
  MItem it0 = mc.it[0], it1 = mc.it[1];
  const bool f0 = m0_active_c<EW>(a, c, t, env0, lane, mc.cm[0]);
  const bool f1 = two && m0_active_c<EW>(a, c, t, env0, lane + WAVE, mc.cm[1]);
  uint64_t pend0 = ballot(f0), pend1 = two ? ballot(f1) : 0ull;
#ifdef COTIX_STATS
  {
    // the valid candidates of the active items (tools/collider_stats.py)
    uint64_t nv = 0;
    for (int s = 0; s < 2; ++s) {
      const MItem& it = s ? it1 : it0;
      if (!(s ? f1 : f0)) continue;
      for (int idx = it.cb; idx < it.ce; ++idx) {
        const int cid = (t.tb[c.sh.o_cand + idx] >> 18) & 511u;
        if (!(cx::isn(t.f(c.L.con + 4 * cid + 2, it.e)) || cx::isn(t.f(c.L.con + 4 * cid + 3, it.e)))) ++nv;
      }
    }
    static uint64_t wsum = 0;
    if (lane == 0) wsum = 0;
    wsum += nv;
    if (lane == WAVE - 1) {
      CXK_STAT(valid_cands, wsum);
      CXK_STAT(fit64, wsum <= 64 ? 1 : 0);
      CXK_STAT(wave_steps, 1);
      CXK_STAT(active_items, popc64(pend0) + popc64(pend1));
    }
  }
#endif
  for (int round = 0; (pend0 | pend1) != 0ull; ++round) {
#ifdef COTIX_STATS
    if (lane == 0) {
      CXK_STAT(rounds, 1);
      if (round == 1) CXK_STAT(r1_left, popc64(pend0) + popc64(pend1));
    }
#endif
    const int n0 = popc64(pend0), n = n0 + popc64(pend1);
    const int ns = n < COTIX_SCAN_RANKS ? n : COTIX_SCAN_RANKS, G = lanes_per_item(ns);  // items that draw, lanes each
    const bool m0 = ((pend0 >> lane) & 1ull) != 0ull, m1 = ((pend1 >> lane) & 1ull) != 0ull;
    const int r0 = popc64(pend0 & lanes_below(lane)), r1 = n0 + popc64(pend1 & lanes_below(lane));  // ranks
    const bool d0 = m0 && r0 < ns, d1 = m1 && r1 < ns;
    if (d0) t.ws[WS_FLAG + r0] = (uint32_t)(it0.cb + it0.pos) | ((uint32_t)it0.ce << 12) | ((uint32_t)lane << 25);
    if (d1)
      t.ws[WS_FLAG + r1] =
          (uint32_t)(it1.cb + it1.pos) | ((uint32_t)it1.ce << 12) | ((uint32_t)(lane + WAVE) << 25);
    lockstep();  // every rank's slot word before the drawers read them
    const int slot = rank_of_lane(lane, G), q = lane - slot * G;
    bool pass = false;
    uint32_t cd = 0xFFFFFFFFu;
    if (slot < ns) cd = m_draw<EW>(c, t, t.ws[WS_FLAG + slot], q, kso, pass);
    const uint64_t pm = ballot(pass);
    // an owner's item: the first passing draw among its drawers r*G .. r*G+G-1
    const uint64_t gm = G == WAVE ? ~0ull : ((1ull << G) - 1ull);
    const uint64_t b0 = d0 ? (pm >> (r0 * G)) & gm : 0ull;
    const uint32_t w0 = bpermute(b0 != 0ull ? r0 * G + __builtin_ctzll(b0) : lane, cd);
    const bool k0 = m0 && m_settle<EW>(t, it0, d0, b0, w0, G);
    pend0 = ballot(k0);  // (after every lane's slot read: the next round's slot writes may follow)
    if (two) {
      const uint64_t b1 = d1 ? (pm >> (r1 * G)) & gm : 0ull;
      const uint32_t w1 = bpermute(b1 != 0ull ? r1 * G + __builtin_ctzll(b1) : lane, cd);
      const bool k1 = m1 && m_settle<EW>(t, it1, d1, b1, w1, G);
      pend1 = ballot(k1);
    }
  }
}

// phase D: choose_random_contact (cotix/_colliders.py:274-295)
CX_DEV cx::Params load_par(const uint32_t* tb, int o) {
  return cx::Params{__uint_as_float(tb[o]), __uint_as_float(tb[o + 1]), __uint_as_float(tb[o + 2]),
                    __uint_as_float(tb[o + 3])};
}
// body i's parameters for env e: the scene table, or the env's own words
// (epar: a vmapped pytree whose mass / inertia / elasticity / friction vary
// over the batch, cotix/_bodies.py:140-154)
template <int EW>
CX_DEV cx::Params body_par(const Ctx& c, Tile<EW> t, int i, int e) {
  if (c.sh.epar == 0) return load_par(t.tb, c.sh.o_par + 4 * i);
  const int o = c.L.geo + (int)c.sh.epar - 1 + 4 * i;
  return cx::Params{t.f(o, e), t.f(o + 1, e), t.f(o + 2, e), t.f(o + 3, e)};
}
CX_DEV cx::Rcp load_rcp(const uint32_t* tb, int o) {
  return cx::Rcp{__uint_as_float(tb[o]), __uint_as_float(tb[o + 1])};
}

// resolution i's velocity-independent operands (phase E0 of the design:
// computed by the phase-D item (body i, env e) right after its choice j)
// the rollout forward's per-env staging of a step's tape words, in the
// layout of the tape (tape_words): 5 words per body [partner | contact id,
// pen, cp], directly followed by the resolution records (REC_W per body,
// L.rec) -- the last 5 nb words of the adjoint region, which only the
// backward uses
CX_HD int tape_stage(const Ctx& c) { return c.L.rec - 5 * c.nb; }
template <int EW, bool RCP>
CX_DEV void e0_item(const Ctx& c, Tile<EW> t, int e, int i, int j, int cid, bool stage = false, uint32_t* tp = nullptr) {
  // branch-free: the operands are computed from clamped indices for every
  // item and the partner is set only for a real resolution (the inactive
  // items' operands are never read: E1 skips RP_NONE)
  using namespace cx;
  const SceneHdr& sc = c.sh;
  const Lay& L = c.L;
  const int ro = L.rp + RP_W * i;
  const bool pair = !(j == i || j < 0 || j >= c.nb) && cid >= 0;
  const int jc = pair ? j : i, co = L.con + 4 * (pair ? cid : 0);
  const v2 cp = v2{t.f(co + 2, e), t.f(co + 3, e)};
  const int oi = L.dyn + 6 * i, oj = L.dyn + 6 * jc;
  const Dyn bi = Dyn{t.f(oi, e), t.f(oi + 1, e), 0.0f, 0.0f, 0.0f, 0.0f};
  const Dyn bj = Dyn{t.f(oj, e), t.f(oj + 1, e), 0.0f, 0.0f, 0.0f, 0.0f};
  const Params pj = body_par<EW>(c, t, jc, e);
  const Rcp qj = load_rcp(t.tb, sc.o_rcp + 2 * jc);
  const ResPre p = resolve_pre<RCP>(bi, body_par<EW>(c, t, i, e), load_rcp(t.tb, sc.o_rcp + 2 * i), bj, pj, qj,
                                    v2{t.f(co, e), t.f(co + 1, e)}, cp, baum_of(sc));
  t.f(ro + RP_NX, e) = p.n.x;
  t.f(ro + RP_NY, e) = p.n.y;
  t.f(ro + RP_R1X, e) = p.r1.x;
  t.f(ro + RP_R1Y, e) = p.r1.y;
  t.f(ro + RP_R2X, e) = p.r2.x;
  t.f(ro + RP_R2Y, e) = p.r2.y;
  t.f(ro + RP_PX, e) = p.pen.x;
  t.f(ro + RP_PY, e) = p.pen.y;
  t.f(ro + RP_DEN, e) = p.den;
  t.f(ro + RP_PT, e) = p.pterm;
  t.f(ro + RP_NE, e) = p.ne;
  t.f(ro + RP_MU, e) = p.mu;
  t.f(ro + RP_MJ, e) = pj.mass;
  t.f(ro + RP_IJ, e) = pj.inertia;
  t.f(ro + RP_QMJ, e) = qj.m;
  t.f(ro + RP_QIJ, e) = qj.i;
  // resolve_collision returns unchanged bodies on a NaN contact point
  const bool res = pair && !vnan(cp);
  if (res) CXK_STAT(resolutions, 1);
  t.w(ro + RP_J, e) = res ? (uint32_t)j : RP_NONE;
  // the rollout forward's tape words of body i, from the operands in hand:
  // staged next to the records (analytic scenes, tape_stage), or stored
  // (polygon scenes: their broadphase pseudo-angles overlay that region)
  const uint32_t w0 = res ? (uint32_t)j | ((uint32_t)cid << 8) : RP_NONE;
  if (stage) {
    const int o = tape_stage(c) + 5 * i;
    t.w(o, e) = w0;
    t.f(o + 1, e) = t.f(co, e);
    t.f(o + 2, e) = t.f(co + 1, e);
    t.f(o + 3, e) = cp.x;
    t.f(o + 4, e) = cp.y;
  } else if (tp != nullptr) {
    tp[0] = w0;
    if (res) {
      tp[4] = __builtin_bit_cast(uint32_t, t.f(co, e));  // (rows 4 words apart, row_at)
      tp[8] = __builtin_bit_cast(uint32_t, t.f(co + 1, e));
      tp[12] = __builtin_bit_cast(uint32_t, cp.x);
      tp[16] = __builtin_bit_cast(uint32_t, cp.y);
    }
  }
}

// one (body i, env) item of phase D; NB > 0: the body count at compile time
// (unrolled loads and selects), NB == 0: any count up to MAXB
template <int EW, bool PRE, int NB, bool RCP>
CX_DEV void d_item(const Ctx& c, Tile<EW> t, int e, int i, int kso, bool stage = false, uint32_t* tp = nullptr) {
  using namespace cx;
  constexpr int MB = NB > 0 ? NB : MAXB;
  const int nb = NB > 0 ? NB : c.nb, nt = c.nt;
  const Lay& L = c.L;
  int cnt = 0;
  uint32_t good = 0u;
  int mm[MB];
#pragma unroll
  for (int j = 0; j < MB; ++j) {
    mm[j] = j < nb ? (int)t.w(L.m + i * nb + j, e) : -1;
    if (mm[j] >= 0) {
      good |= 1u << j;
      ++cnt;
    }
  }
  int ch = i;
  {  // evaluated for every item (branch-free); kept only when cnt > 0
    float p[MB], cs[MB];
    // p = notnan / count (:280-283): 1/count or 0/count == +0 (count > 0)
    const float inv = 1.0f / (float)(cnt > 0 ? cnt : 1);
#pragma unroll
    for (int j = 0; j < MB; ++j) p[j] = ((good >> j) & 1u) ? inv : 0.0f;
    if (NB > 0)
      cumsum_fixed<MB>(p, cs);
    else
      cumsum_n(p, nb, cs);
    float u;
    if (PRE) {
      u = t.f(kso + 2 + 2 * nt + i, e);  // the window slot's choice uniforms
    } else {
      const int so = nt > 0 ? L.skt + 2 * (nt - 1) : L.sk0;
      const bool part = c.sh.prng != 0;
      key2 ck = split_at_l(key2{t.w(so, e), t.w(so + 1, e)}, (uint32_t)nb, (uint32_t)i, part);
      u = unit_float(bits1_l(ck, part));
    }
    float last = cs[0];
#pragma unroll
    for (int j = 1; j < MB; ++j)
      if (j < nb) last = cs[j];
    float r = last * (1.0f - u);
    int cj = nb;
#pragma unroll
    for (int j = MB - 1; j >= 0; --j) cj = (j < nb && !(cs[j] < r)) ? j : cj;  // first j with r <= cumsum[j]
    ch = cnt > 0 ? cj : i;
  }
  t.w(L.ch + i, e) = (uint32_t)ch;
  int cid = -1;  // all_contacts[i, ch], picked from the loaded row (candidate word -> distinct contact)
#pragma unroll
  for (int j = 0; j < MB; ++j) cid = j == ch ? mm[j] : cid;
  cid = cid < 0 ? -1 : (cid >> 18) & 511;
  e0_item<EW, RCP>(c, t, e, i, ch, cid, stage, tp);
}
// TAPE: the rollout forward stages each body's tape words (partner, contact
// id, contact) here, from the operands phase D has in hand, next to phase
// E1's resolution records (tape_stage), so that the save phase copies them
// out as whole rows instead of chasing partner -> cell -> contact
template <int EW, bool PRE = false, bool TAPE = false>
CX_DEV void ph_D(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane, int kso = 0, int step = 0) {
  const int nb = c.nb;
  for (int w = lane; w < nb * EW; w += WAVE) {
    const int e = w % EW, i = w / EW;
    if (env0 + e >= a.B) continue;
    const bool stage = TAPE && a.tape != nullptr && tape_rec(c.sh);
    uint32_t* tp = TAPE && a.tape != nullptr && !stage ? a.tape + row_at(a.B, a.tw, step, 5 * i, env0 + e) : nullptr;
    if (c.sh.rcp_all) {
      if (nb == 5) d_item<EW, PRE, 5, true>(c, t, e, i, kso, stage, tp);
      else if (nb == 4) d_item<EW, PRE, 4, true>(c, t, e, i, kso, stage, tp);
      else d_item<EW, PRE, 0, true>(c, t, e, i, kso, stage, tp);
    } else {
      if (nb == 5) d_item<EW, PRE, 5, false>(c, t, e, i, kso, stage, tp);
      else if (nb == 4) d_item<EW, PRE, 4, false>(c, t, e, i, kso, stage, tp);
      else d_item<EW, PRE, 0, false>(c, t, e, i, kso, stage, tp);
    }
  }
}

// The tape backward's restore of an analytic scene as 16-byte rows (4 envs per
// wave, whole waves): row r < 6 nb is state word r (save_dyn), row 6 nb + k
// tape word k (5 per body, then the records), one 16-byte read per row and
// lane -- at most 2 rows a lane, 8 registers, so the reads can run two steps
// ahead (restore_rows_fetch into one of two register sets); the tape rows land
// in the key-window words, which the analytic backward does not use
// (rows_tape), and phase D reads them there (ph_D_tape STAGED)
CX_HD int rows_tape(const Ctx& c) { return c.L.kw; }
template <int EW>
CX_HD bool rows_restore(const KArgs& a, const Ctx& c) {
  return EW == 4 && (a.B & 3) == 0 && tape_rec(c.sh) && (a.stages & COTIX_STAGE_COLLIDER) && 18 * c.nb <= 2 * WAVE &&
         (5 + REC_W) * c.nb <= KWIN * c.L.kww;
}
struct RowRegs {
  U4 d[2];
  uint32_t k0 = 0u, k1 = 0u;
};
template <int EW>
CX_DEV void restore_rows_fetch(const KArgs& a, const Ctx& c, int env0, int lane, int step, RowRegs& r) {
  const int nd = 6 * c.nb, nr = nd + (5 + REC_W) * c.nb;
  // the row's source as a select of two byte addresses, not of the two
  // pointer arguments: a per-lane select of kernel arguments compiles into a
  // vector load of the argument itself, and the s_waitcnt vmcnt(0) it needs
  // waits for every store in flight (the previous step's grad_action).
  // The wave's rows are contiguous (row_at): 16 bytes per row from two bases
  const uintptr_t sd = reinterpret_cast<uintptr_t>(a.save_dyn) + row_at(a.B, nd, step, 0, env0) * 4u;
  const uintptr_t st = reinterpret_cast<uintptr_t>(a.tape) + row_at(a.B, a.tw, step, 0, env0) * 4u - (size_t)nd * 16u;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int row = q * WAVE + lane;
    const uintptr_t src = (row < nd ? sd : st) + (size_t)row * 16u;
    if (row < nr) r.d[q] = *reinterpret_cast<const U4*>(src);
  }
  const int g = env0 + lane;
  const bool le = lane < EW && g < a.B;
  r.k0 = le ? a.save_keys[2 * ((size_t)step * a.B + g)] : 0u;
  r.k1 = le ? a.save_keys[2 * ((size_t)step * a.B + g) + 1] : 0u;
}
template <int EW>
CX_DEV void restore_rows_apply(const Ctx& c, Tile<EW> t, int lane, const RowRegs& r) {
  const int nd = 6 * c.nb, nr = nd + (5 + REC_W) * c.nb;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int row = q * WAVE + lane;
    const int o = row < nd ? c.L.dyn + row : rows_tape(c) + (row - nd);
    if (row < nr)
#pragma unroll
      for (int e = 0; e < 4; ++e) t.w(o, e) = r.d[q].v[e];
  }
  if (lane < EW) {
    t.w(c.L.key, lane) = r.k0;
    t.w(c.L.key + 1, lane) = r.k1;
    t.w(c.L.err, lane) = 0u;
  }
}

// phase D of the backward with a tape (MODE 4): the forward's resolution of
// body i -- partner, cell, contact, and for a GJK/EPA contact EPA's final
// edge (into ge_edge's words, read by phase GE) -- from the tape registers,
// then the resolution operands as phase D computes them (e0_item); the tile
// words written are exactly those the re-play's phases B-D leave for E, GE
// and G (the chosen cell's candidate word carries only its contact id, the
// one field they read)
CX_HD bool ge_edges_fit(const Ctx& c) { return 28 * c.nb <= KWIN * c.L.kww; }
CX_DEV int ge_edge_word(const Ctx& c, int i) { return c.L.kw + 24 * c.nb + 4 * i; }
// STAGED: the step's tape words are rows of the tile (restore_rows, analytic
// scenes) instead of this lane's registers
template <int EW, bool TR, bool STAGED = false>
CX_DEV void ph_D_tape(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane, const TapeRegs& r) {
  const Lay& L = c.L;
  const int nb = c.nb, ni = nb * EW;
  const bool edges = c.sh.poly && ge_edges_fit(c);
#pragma unroll
  for (int q = 0; q < TQ; ++q) {
    if (q * WAVE >= ni) break;  // uniform
    const int w = q * WAVE + lane, e = w % EW, i = w / EW;
    if (w >= ni || env0 + e >= a.B) continue;
    auto dw = [&](int k) { return STAGED ? t.w(rows_tape(c) + 5 * (i < nb ? i : 0) + k, e) : r.d[q][k]; };
    auto xw = [&](int k) { return STAGED ? t.w(rows_tape(c) + 5 * nb + REC_W * (i < nb ? i : 0) + k, e) : r.x[q][k]; };
    const uint32_t dec = dw(0);
    const bool res = dec != RP_NONE;
    const int j = res ? (int)(dec & 255u) : i, cid = res ? (int)((dec >> 8) & 511u) : -1;
    t.w(L.ch + i, e) = (uint32_t)j;
    if (TR && tape_rec(c.sh)) {  // the forward's record of the resolution (phase E does not run)
      t.w(L.rec + REC_W * i, e) = res ? xw(0) : 0u;
      if (res)
#pragma unroll
        for (int k = 1; k < REC_W; ++k) t.w(L.rec + REC_W * i + k, e) = xw(k);
    }
    if (res) {
      t.w(L.m + i * nb + j, e) = (uint32_t)cid << 18;
      const int co = L.con + 4 * cid;
#pragma unroll
      for (int k = 0; k < 4; ++k) t.w(co + k, e) = dw(k + 1);
      if (edges) {
        const int eo = ge_edge_word(c, i);
#pragma unroll
        for (int k = 0; k < 4; ++k) t.w(eo + k, e) = r.x[q][k];
      }
    }
    if (TR && tape_rec(c.sh)) continue;  // (the resolution operands are phase E's)
    if (c.sh.rcp_all)
      e0_item<EW, true>(c, t, e, i, j, cid);
    else
      e0_item<EW, false>(c, t, e, i, j, cid);
  }
}

// phase E: sequential resolution (:310-336), joints, key update, restarts.
// E0 (item = (body i, env), all lanes): everything of resolution i that does
// not depend on velocities -- partner j = choice[i], the contact, the
// positions (a resolution changes velocities only) and the parameters --
// folded into cx::ResPre.  E1 (one lane per env): the sequential pass over
// the bodies carrying only the velocity-dependent part, velocities held in
// registers for the common body counts.

template <int EW>
CX_DEV cx::ResPre load_rp(Tile<EW> t, int ro, int e) {
  cx::ResPre p;
  p.n = cx::v2{t.f(ro + RP_NX, e), t.f(ro + RP_NY, e)};
  p.r1 = cx::v2{t.f(ro + RP_R1X, e), t.f(ro + RP_R1Y, e)};
  p.r2 = cx::v2{t.f(ro + RP_R2X, e), t.f(ro + RP_R2Y, e)};
  p.pen = cx::v2{t.f(ro + RP_PX, e), t.f(ro + RP_PY, e)};
  p.den = t.f(ro + RP_DEN, e);
  p.pterm = t.f(ro + RP_PT, e);
  p.ne = t.f(ro + RP_NE, e);
  p.mu = t.f(ro + RP_MU, e);
  return p;
}

// E1 sequential pass, NB (== nb) bodies' velocities in registers; body j is
// picked and written back by unrolled selects (no scratch)
// (TREC: the rollout forward's records for the tape -- only the resolutions'
// own words, which tape_save reads; no pass when nothing resolves)
template <int EW, bool REC, int NB, bool RCP, bool TREC = false>
CX_DEV void e1_regs(const Ctx& c, Tile<EW> t, int e) {
  using namespace cx;
  const SceneHdr& sc = c.sh;
  const Lay& L = c.L;
  uint32_t jv[NB];
  bool any = false;
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    jv[i] = t.w(L.rp + RP_W * i + RP_J, e);
    any = any | (jv[i] != RP_NONE);
  }
  if (!REC && !any) return;  // no resolution this step: the velocities stay as they are
  float vx[NB], vy[NB], vw[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    vx[b] = t.f(L.dyn + 6 * b + 2, e);
    vy[b] = t.f(L.dyn + 6 * b + 3, e);
    vw[b] = t.f(L.dyn + 6 * b + 5, e);
  }
  // every resolution's operands up front: one LDS latency for the pass
  ResPre pr[NB];
  Params pj[NB], pi[NB];
  Rcp qj[NB], qi[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int ro = L.rp + RP_W * i;
    pr[i] = load_rp<EW>(t, ro, e);
    pj[i] = Params{t.f(ro + RP_MJ, e), t.f(ro + RP_IJ, e), 0.0f, 0.0f};
    qj[i] = Rcp{t.f(ro + RP_QMJ, e), t.f(ro + RP_QIJ, e)};
    pi[i] = body_par<EW>(c, t, i, e);
    qi[i] = load_rcp(t.tb, sc.o_rcp + 2 * i);
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const uint32_t j = jv[i];
    if (REC) t.w(L.rec + REC_W * i, e) = 0u;
    if (j == RP_NONE) continue;
    constexpr bool RW = REC || TREC;  // the resolution's record words
    float jx = 0.0f, jy = 0.0f, jw = 0.0f;
#pragma unroll
    for (int b = 0; b < NB; ++b)
      if ((uint32_t)b == j) {
        jx = vx[b];
        jy = vy[b];
        jw = vw[b];
      }
    if (RW) {
      const int rc = L.rec + REC_W * i;
      t.f(rc + 1, e) = vx[i];
      t.f(rc + 2, e) = vy[i];
      t.f(rc + 3, e) = vw[i];
      t.f(rc + 4, e) = jx;
      t.f(rc + 5, e) = jy;
      t.f(rc + 6, e) = jw;
    }
    const bool applied = resolve_seq<RCP>(vx[i], vy[i], vw[i], pi[i], qi[i], jx, jy, jw, pj[i], qj[i], pr[i]);
    if (RW) t.w(L.rec + REC_W * i, e) = applied ? 1u : 0u;
#pragma unroll
    for (int b = 0; b < NB; ++b)
      if ((uint32_t)b == j) {
        vx[b] = jx;
        vy[b] = jy;
        vw[b] = jw;
      }
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    t.f(L.dyn + 6 * b + 2, e) = vx[b];
    t.f(L.dyn + 6 * b + 3, e) = vy[b];
    t.f(L.dyn + 6 * b + 5, e) = vw[b];
  }
}
// E1 for any body count: the same pass on the LDS tile
template <int EW, bool REC, bool RCP>
CX_DEV void e1_tile(const Ctx& c, Tile<EW> t, int e) {
  using namespace cx;
  const SceneHdr& sc = c.sh;
  const Lay& L = c.L;
  for (int i = 0; i < c.nb; ++i) {
    const int ro = L.rp + RP_W * i;
    const uint32_t j = t.w(ro + RP_J, e);
    if (REC) t.w(L.rec + REC_W * i, e) = 0u;
    if (j == RP_NONE) continue;
    const int oi = L.dyn + 6 * i, oj = L.dyn + 6 * (int)j;
    float ix = t.f(oi + 2, e), iy = t.f(oi + 3, e), iw = t.f(oi + 5, e);
    float jx = t.f(oj + 2, e), jy = t.f(oj + 3, e), jw = t.f(oj + 5, e);
    if (REC) {
      const int rc = L.rec + REC_W * i;
      t.f(rc + 1, e) = ix;
      t.f(rc + 2, e) = iy;
      t.f(rc + 3, e) = iw;
      t.f(rc + 4, e) = jx;
      t.f(rc + 5, e) = jy;
      t.f(rc + 6, e) = jw;
    }
    const Params pi = body_par<EW>(c, t, i, e);
    const Params pj = Params{t.f(ro + RP_MJ, e), t.f(ro + RP_IJ, e), 0.0f, 0.0f};
    const Rcp qj = Rcp{t.f(ro + RP_QMJ, e), t.f(ro + RP_QIJ, e)};
    const bool applied = resolve_seq<RCP>(ix, iy, iw, pi, load_rcp(t.tb, sc.o_rcp + 2 * i), jx, jy, jw, pj, qj,
                                     load_rp<EW>(t, ro, e));
    if (REC) t.w(L.rec + REC_W * i, e) = applied ? 1u : 0u;
    t.f(oi + 2, e) = ix;
    t.f(oi + 3, e) = iy;
    t.f(oi + 5, e) = iw;
    t.f(oj + 2, e) = jx;
    t.f(oj + 3, e) = jy;
    t.f(oj + 5, e) = jw;
  }
}

#ifdef COTIX_STATS
CX_DEV int L_rp_(const Ctx& c) { return c.L.rp; }
#endif
// the rollout's return terms (stage_ret_terms' compact list, launch
// constants) in the registers of the env's lane, read once per launch
constexpr int RT = 8;
CX_DEV int ret_terms_cap(const Ctx& c) {
  const int cap = (c.nb * 6 - 1) / 2;
  return cap < RT ? cap : RT;
}
struct RetRegs {
  int n = 0;
  int k[RT];
  float w[RT];
};
template <int EW>
CX_DEV void ret_fetch(const Ctx& c, Tile<EW> t, int lane, RetRegs& r) {
  const int e = lane < EW ? lane : 0;
  r.n = (int)t.w(c.L.rst, e);
#pragma unroll
  for (int j = 0; j < RT; ++j) {
    r.k[j] = j < r.n ? (int)t.w(c.L.rst + 1 + 2 * j, e) : 0;
    r.w[j] = j < r.n ? t.f(c.L.rst + 2 + 2 * j, e) : 0.0f;
  }
}
// return accumulation after a step (env e's lane): ret += sum_k w_k * state_k
// (w_k != 0), k ascending
template <int EW>
CX_DEV void ret_accum(const KArgs& a, const Ctx& c, Tile<EW> t, int e, const RetRegs& r) {
  float acc = t.f(c.L.ret, e);
  if (r.n <= ret_terms_cap(c)) {
    float sv[RT];
#pragma unroll
    for (int j = 0; j < RT; ++j) sv[j] = t.f(c.L.dyn + r.k[j], e);
#pragma unroll
    for (int j = 0; j < RT; ++j) acc = j < r.n ? acc + r.w[j] * sv[j] : acc;
  } else {  // more terms than the list holds: every weight from the kernel arguments
    for (int k = 0; k < c.nb * 6; ++k)
      if (a.ret_w[k] != 0.0f) acc = acc + a.ret_w[k] * t.f(c.L.dyn + k, e);
  }
  t.f(c.L.ret, e) = acc;
}

// tile rows [o, o + n) of the wave's envs (row r: EW words, env fastest) to
// rows [0, n) of step `step` of a saved-rows array of `rows` rows (row_at):
// with 4 envs per wave and a whole block, one 16-byte store per row (a lane
// each, the wave's n rows one contiguous run); else one word per (row, env)
// lane
// (dbg, tooling builds only -- the save-phase experiments of tools/gpu_fwd_exp.sh:
// 1 stores zeros without the LDS reads, 2 reads without storing, 3 non-temporal stores)
template <int EW>
CX_DEV void rows_out(Tile<EW> t, int o, int n, uint32_t* dst, int rows, int step, int B, int env0, int lane,
                     int dbg = 0) {
  if (EW == 4 && env0 + 4 <= B) {
    U4* blk = reinterpret_cast<U4*>(dst + row_at(B, rows, step, 0, env0));
    for (int r = lane; r < n; r += WAVE) {
      if (dbg == 1) {
        blk[r] = U4{{0u, 0u, 0u, 0u}};
        continue;
      }
      const U4 w = U4{{t.w(o + r, 0), t.w(o + r, 1), t.w(o + r, 2), t.w(o + r, 3)}};
#if defined(__HIP__)
      if (dbg == 2) {
        asm volatile("" ::"v"(w.v[0]), "v"(w.v[1]), "v"(w.v[2]), "v"(w.v[3]));
        continue;
      }
      if (dbg == 3) {  // non-temporal (streaming) store
        typedef uint32_t v4u __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(v4u{w.v[0], w.v[1], w.v[2], w.v[3]}, reinterpret_cast<v4u*>(blk + r));
        continue;
      }
#endif
      blk[r] = w;
    }
  } else {
    for (int w = lane; w < n * EW; w += WAVE) {
      const int e = w % EW, r = w / EW;
      if (env0 + e < B) dst[row_at(B, rows, step, r, env0 + e)] = t.w(o + r, e);
    }
  }
}

// REC (backward re-play only): record, per resolution, whether the impulses
// were applied and the pre-resolution velocities of the two bodies.
// RET (rollout forward): the return accumulation after the step, on the
// env's lane (ret_accum), in the same phase.
// the rollout forward's tape words of step `step` (tape_words): per (body i,
// env) item, from the tile's phase-D words of that step -- they live until
// the next step's phase A resets the collider scratch, so the save runs in
// the next step's save phase (ph_save) or, for the last step, after the loop
template <int EW, bool TR>
CX_DEV void tape_save(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane, int step, int dbg = 0) {
  // (polygon scenes: phase D stores their resolution words, phase B EPA's edges)
  if (TR && tape_rec(c.sh))
    rows_out<EW>(t, tape_stage(c), (5 + REC_W) * c.nb, a.tape, a.tw, step, a.B, env0, lane, dbg);
}

// TREC: the rollout forward with a tape records the resolutions (as REC) for
// tape_save, and is otherwise the forward's phase E
template <int EW, bool REC = false, bool RET = false, bool TREC = false>
CX_DEV void ph_E(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane, int kso, const RetRegs* rr = nullptr) {
  constexpr bool RC = REC || TREC;
  using namespace cx;
  const SceneHdr& sc = c.sh;
  const int nb = c.nb;
  const Lay& L = c.L;
  for (int e = lane; e < EW; e += WAVE) {
    int g = env0 + e;
    if (g >= a.B) continue;
#ifdef COTIX_STATS
    if (a.stages & COTIX_STAGE_COLLIDER) {  // dependency levels of the sequential pass (tools/collider_stats.py)
      int last[MAXB] = {0}, L = 0;
      for (int i = 0; i < nb; ++i) {
        const uint32_t j = t.w(L_rp_(c) + RP_W * i + RP_J, e);
        if (j == RP_NONE) continue;
        const int lv = (last[i] > last[j] ? last[i] : last[j]) + 1;
        last[i] = last[j] = lv;
        L = lv > L ? lv : L;
      }
      static int wmax = 0, wslots = 0;
      static uint32_t wmask = 0;
      if (e == 0) { wmax = 0; wmask = 0; }
      wmax = L > wmax ? L : wmax;
      for (int i = 0; i < nb; ++i) if (t.w(L_rp_(c) + RP_W * i + RP_J, e) != RP_NONE) wmask |= 1u << i;
      CXK_STAT(lvl_env, L);
      if (e == EW - 1) { CXK_STAT(lvl_wave, wmax); CXK_STAT(e1_slots, __builtin_popcount(wmask)); }
      (void)wslots;
    }
#endif
    if (a.stages & COTIX_STAGE_COLLIDER) {
      if (sc.rcp_all) {
        switch (nb) {
          case 4: e1_regs<EW, REC, 4, true, TREC>(c, t, e); break;
          case 5: e1_regs<EW, REC, 5, true, TREC>(c, t, e); break;
          default: e1_tile<EW, RC, true>(c, t, e); break;
        }
      } else {
        switch (nb) {
          case 4: e1_regs<EW, REC, 4, false, TREC>(c, t, e); break;
          case 5: e1_regs<EW, REC, 5, false, TREC>(c, t, e); break;
          default: e1_tile<EW, RC, false>(c, t, e); break;
        }
      }
    }
    if (!REC && (a.stages & COTIX_STAGE_LUNAR) && nb >= 3) {  // (the re-play: phase G reverses them)
      Dyn d[3];
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        const int o = L.dyn + 6 * b;
        d[b] = Dyn{t.f(o, e), t.f(o + 1, e), t.f(o + 2, e), t.f(o + 3, e), t.f(o + 4, e), t.f(o + 5, e)};
      }
      const Params p0 = body_par<EW>(c, t, 0, e), p1 = body_par<EW>(c, t, 1, e), p2 = body_par<EW>(c, t, 2, e);
      const Rcp q0 = load_rcp(t.tb, sc.o_rcp), q1 = load_rcp(t.tb, sc.o_rcp + 2), q2 = load_rcp(t.tb, sc.o_rcp + 4);
      const int rm = sc.rcp_mask;  // scene constant: uniform branch
      if ((rm & 7) == 7)
        lunar_constraints<true, true>(d[0], d[1], d[2], p0, p1, p2, q0, q1, q2);
      else if ((rm & 6) == 6)
        lunar_constraints<false, true>(d[0], d[1], d[2], p0, p1, p2, q0, q1, q2);
      else
        lunar_constraints<false, false>(d[0], d[1], d[2], p0, p1, p2, q0, q1, q2);
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        const int o = L.dyn + 6 * b;
        t.f(o + 2, e) = d[b].vx;
        t.f(o + 3, e) = d[b].vy;
        t.f(o + 5, e) = d[b].w;
      }
    }
    if (a.stages & COTIX_STAGE_ADVANCE_KEY) {  // examples/test_viz.py:39,66
      t.w(L.key, e) = t.w(kso, e);
      t.w(L.key + 1, e) = t.w(kso + 1, e);
    }
    if (a.dyn_reset != nullptr && a.reset_mode == 1) {
      // episode end on an error_if trip (the reference raises here): the env
      // restarts from its reset state (phase R, spread over the lanes); the
      // key chain continues.
      const uint32_t r = t.w(L.err, e) != 0u ? 1u : 0u;
      t.w(L.rflag, e) = r;
      t.w(L.err, e) = 0u;
      t.w(L.nres, e) = t.w(L.nres, e) + r;
    }
    if (RET) ret_accum<EW>(a, c, t, e, *rr);  // (the rollout never restarts: after phase R's place)
  }
}

// collider trace of step `step` (cotix_step_ex): chosen partner per body and
// the winning candidate per cell, item = (word, env); -1 where the collider
// stage is off or the cell is empty
template <int EW>
CX_DEV void ph_trace(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane, int step) {
  const Lay& L = c.L;
  const int nb = c.nb;
  const bool col = (a.stages & COTIX_STAGE_COLLIDER) != 0;
  if (a.trace_chosen != nullptr)
    for (int w = lane; w < nb * EW; w += WAVE) {
      const int e = w % EW, i = w / EW, g = env0 + e;
      if (g < a.B) a.trace_chosen[((size_t)step * nb + i) * a.B + g] = col ? (int32_t)t.w(L.ch + i, e) : -1;
    }
  if (a.trace_cells != nullptr)
    for (int w = lane; w < nb * nb * EW; w += WAVE) {
      const int e = w % EW, k = w / EW, g = env0 + e;
      const uint32_t cd = t.w(L.m + k, e);
      const int32_t code = (!col || cd == 0xFFFFFFFFu) ? -1 : (int32_t)((cd & 0x3FFFFu) | ((cd >> 27) << 18));
      if (g < a.B) a.trace_cells[((size_t)step * nb * nb + k) * a.B + g] = code;
    }
}

// phase R (autoreset launches): restore the restarting envs' state,
// item = (state word, env)
template <int EW>
CX_DEV void ph_R(const Ctx& c, Tile<EW> t, int lane) {
  const Lay& L = c.L;
  for (int w = lane; w < c.nb * 6 * EW; w += WAVE) {
    const int e = w % EW, off = w / EW;
    if (t.w(L.rflag, e) != 0u) t.f(L.dyn + off, e) = t.f(L.rst + off, e);
  }
}

// ---------------------------------------------------------------------------
// cotix_eval: the reference's NFE loop (cotix/_envs.py:37-117) per env, with
// the device judge.  The carry (finished, reward) lives in the tile; the
// premature-out state in rst, its key / err / reward in jk, je, jpr.
// ---------------------------------------------------------------------------
template <int EW>
CX_DEV float judge_lin(Tile<EW> t, int o, int e, int n, const uint8_t* k, const float* w) {
  float acc = 0.0f;
  for (int q = 0; q < n; ++q) {
    const float term = w[q] * t.f(o + k[q], e);
    acc = q == 0 ? term : acc + term;
  }
  return acc;
}
// the first of n boxes holding the env's state (strictly inside every bound), or -1
template <int EW>
CX_DEV int first_box(Tile<EW> t, int o, int e, int n, const int* body, const float (*lo)[6], const float (*hi)[6]) {
  for (int r = 0; r < n; ++r) {
    bool in = true;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const float v = t.f(o + 6 * body[r] + q, e);
      in = in & (lo[r][q] < v) & (v < hi[r][q]);
    }
    if (in) return r;
  }
  return -1;
}
// the first (done) region holding the env's state, or -1
template <int EW>
CX_DEV int judge_region(const JudgeArgs& j, Tile<EW> t, int o, int e) {
  return first_box<EW>(t, o, e, j.nreg, j.rbody, j.lo, j.hi);
}
// the reward rate: the base sum, plus the piece of the first rate region
// holding the state -- piecewise linear over the rate regions
template <int EW>
CX_DEV float judge_rate(const JudgeArgs& j, Tile<EW> t, int o, int e) {
  const float base = judge_lin<EW>(t, o, e, j.nrate, j.rate_k, j.rate_w);
  const int r = j.nrr > 0 ? first_box<EW>(t, o, e, j.nrr, j.prbody, j.prlo, j.prhi) : -1;
  float pc = 0.0f;  // the piece: its own sum from its first term, then base + piece
  bool has = false;
  for (int q = 0; q < JR; ++q) {
    if (q != r) continue;
    for (int m = 0; m < j.npr[q]; ++m) {
      const float term = j.pr_w[q][m] * t.f(o + j.pr_k[q][m], e);
      pc = has ? pc + term : term;
      has = true;
    }
    if (j.hasb[q]) pc = has ? pc + j.pr_b[q] : j.pr_b[q];
    has = has || j.hasb[q] != 0;
  }
  if (!has) return base;
  return j.nrate > 0 ? base + pc : pc;
}
template <int EW>
CX_DEV float judge_end(const JudgeArgs& j, Tile<EW> t, int o, int e, int r) {
  float acc = judge_lin<EW>(t, o, e, j.nend, j.end_k, j.end_w);
  if (r >= 0) acc = j.nend > 0 ? acc + j.rrew[r] : j.rrew[r];
  return acc;
}
template <int EW>
CX_DEV bool judge_done(const JudgeArgs& j, Tile<EW> t, int e, int r, int err_off) {
  return r >= 0 || (j.doe && t.w(err_off, e) != 0u);
}
// NFE start (:43-65), one lane per env: end_reward = finished ? reward :
// reward + end_reward(s); premature_out = (s, end_reward);
// already = is_done(s).  The state words are snapshot by ph_JS.
template <int EW>
CX_DEV void ph_JB(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane) {
  const Lay& L = c.L;
  for (int e = lane; e < EW; e += WAVE) {
    if (env0 + e >= a.B) continue;
    const int r = judge_region<EW>(a.judge, t, L.dyn, e);
    const float R = t.f(L.jr, e);
    t.f(L.jpr, e) = t.w(L.jfin, e) != 0u ? R : R + judge_end<EW>(a.judge, t, L.dyn, e, r);
    t.w(L.jal, e) = judge_done<EW>(a.judge, t, e, r, L.err) ? 1u : 0u;
    t.w(L.jk, e) = t.w(L.key, e);
    t.w(L.jk + 1, e) = t.w(L.key + 1, e);
    t.w(L.je, e) = t.w(L.err, e);
    t.w(L.jsn, e) = 1u;
  }
}
// after each env-step (:77-108): ending = reward + end_reward(s); the first
// step that is done becomes the premature out; reward += rate(s) * dt
template <int EW>
CX_DEV void ph_J(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane) {
  const Lay& L = c.L;
  for (int e = lane; e < EW; e += WAVE) {
    if (env0 + e >= a.B) continue;
    const int r = judge_region<EW>(a.judge, t, L.dyn, e);
    const float R = t.f(L.jr, e);
    const bool now = judge_done<EW>(a.judge, t, e, r, L.err) && t.w(L.jal, e) == 0u;
    if (now) {
      t.f(L.jpr, e) = R + judge_end<EW>(a.judge, t, L.dyn, e, r);
      t.w(L.jal, e) = 1u;
      t.w(L.jk, e) = t.w(L.key, e);
      t.w(L.jk + 1, e) = t.w(L.key + 1, e);
      t.w(L.je, e) = t.w(L.err, e);
    }
    t.w(L.jsn, e) = now ? 1u : 0u;
    t.f(L.jr, e) = R + judge_rate<EW>(a.judge, t, L.dyn, e) * a.dt;
  }
}
// the premature-out state words of the envs flagged by ph_JB / ph_J, item = (word, env)
template <int EW>
CX_DEV void ph_JS(const Ctx& c, Tile<EW> t, int lane) {
  const Lay& L = c.L;
  for (int w = lane; w < c.nb * 6 * EW; w += WAVE) {
    const int e = w % EW, off = w / EW;
    if (t.w(L.jsn, e) != 0u) t.f(L.rst + off, e) = t.f(L.dyn + off, e);
  }
}
// NFE end (:110-117): an env that is done takes its premature out; finished = already
template <int EW>
CX_DEV void ph_JE(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane) {
  const Lay& L = c.L;
  for (int w = lane; w < c.nb * 6 * EW; w += WAVE) {
    const int e = w % EW, off = w / EW;
    if (t.w(L.jal, e) != 0u) t.f(L.dyn + off, e) = t.f(L.rst + off, e);
  }
  for (int e = lane; e < EW; e += WAVE) {
    if (env0 + e >= a.B) continue;
    const bool al = t.w(L.jal, e) != 0u;
    if (al) {
      t.w(L.key, e) = t.w(L.jk, e);
      t.w(L.key + 1, e) = t.w(L.jk + 1, e);
      t.w(L.err, e) = t.w(L.je, e);
      t.f(L.jr, e) = t.f(L.jpr, e);
    }
    t.w(L.jfin, e) = al ? 1u : 0u;
  }
}

// all ones where env e's restart is taken at the store (rs and its flag),
// else 0: a mask on the word offset, not a select between the layout's
// fields (which LLVM turns into an indexed read of a private copy)
template <int EW>
CX_DEV int rsel(const Ctx& c, Tile<EW> t, int e, bool rs) {
  return -(int)(rs & (t.w(c.L.rflag, e) != 0u));
}
template <int EW, bool ROLL = false, bool EVAL = false>
CX_DEV void ph_store(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane, bool rs = false) {
  // rs: the last step's restarts are taken here (run_wave's `rstore`): a
  // flagged env's state is its restart state
  for (int w = lane; w < c.nb * 6 * EW; w += WAVE) {
    int e = w % EW, off = w / EW, g = env0 + e;
    const int src = c.L.dyn + ((c.L.rst - c.L.dyn) & rsel<EW>(c, t, e, rs));
    if (g < a.B) a.dyn[(size_t)off * a.B + g] = t.f(src + off, e);
  }
  for (int e = lane; e < EW; e += WAVE) {
    int g = env0 + e;
    if (g < a.B) {
      a.keys[2 * (size_t)g] = t.w(c.L.key, e);
      a.keys[2 * (size_t)g + 1] = t.w(c.L.key + 1, e);
      a.err[g] = t.w(c.L.err, e);
      if (a.resets && !ROLL) a.resets[g] = t.w(c.L.nres, e);
      if (ROLL) a.ret[g] = t.f(c.L.nres, e) + t.f(c.L.ret, e);  // (the incoming return, ph_load_fwd)
      if (EVAL && a.judge.on) {
        if (a.reward) a.reward[g] = t.f(c.L.jr, e);
        if (a.finished) a.finished[g] = t.w(c.L.jfin, e);
      }
    }
  }
  // the observation [B][nb][6]: the wave's EW envs are one contiguous block,
  // item = (env, word) with the word fastest -> coalesced stores
  if (!ROLL && a.obs != nullptr) {
    const int nw = c.nb * 6;
    for (int w = lane; w < nw * EW; w += WAVE) {
      const int e = w / nw, off = w % nw, g = env0 + e;
      const int src = c.L.dyn + ((c.L.rst - c.L.dyn) & rsel<EW>(c, t, e, rs));
      if (g < a.B) a.obs[(size_t)g * nw + off] = t.f(src + off, e);
    }
  }
}

// ---------------------------------------------------------------------------
// differentiable rollout: forward saves, return, backward re-play
// ---------------------------------------------------------------------------
constexpr int RQ = (MAXB * 6 * 8 + 63) / 64;  // words per lane: nb * 6 * EW over 64 lanes (EW <= 8)
// state before step `step` -> save_dyn[step], save_keys[step]
// (+ the tape words of the step before it, tape_save)
template <int EW, bool TR>
CX_DEV void ph_save(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane, int step) {
  if (CXK_SKIP(a, 8192)) step = step > 0 ? 1 : 0;  // (tooling, timing only: every step's saves to one slot)
  const int dbg = CXK_SKIP(a, 512) ? 1 : CXK_SKIP(a, 1024) ? 2 : CXK_SKIP(a, 2048) ? 3 : 0;  // tooling only (rows_out)
  if (a.tape != nullptr && step > 0 && (a.stages & COTIX_STAGE_COLLIDER) && !CXK_SKIP(a, 128))
    tape_save<EW, TR>(a, c, t, env0, lane, step - 1, dbg);
  if (CXK_SKIP(a, 256)) return;
  rows_out<EW>(t, c.L.dyn, c.nb * 6, reinterpret_cast<uint32_t*>(a.save_dyn), c.nb * 6, step, a.B, env0, lane,
               dbg);
  if (CXK_SKIP(a, 4096)) return;  // (tooling: the save phase without the key pair)
  for (int e = lane; e < EW; e += WAVE) {
    int g = env0 + e;
    if (g < a.B) {
      a.save_keys[2 * ((size_t)step * a.B + g)] = t.w(c.L.key, e);
      a.save_keys[2 * ((size_t)step * a.B + g) + 1] = t.w(c.L.key + 1, e);
    }
  }
}

// The return weights, staged once per launch into the tile's restart-state
// words (the rollout programs never restart), so that no step reads them from
// the kernel arguments (a dynamic index there is a memory load per term and
// step).  The backward (G3) reads them dense: word k of body-state word k.
// The forward's return sums only the nonzero terms, compacted in k order
// (ballots): word 0 the count n, then (k, w) pairs -- two LDS round trips per
// step for up to RT terms (the return of config 5 has one).
template <int EW>
CX_DEV void stage_ret_w(const KArgs& a, const Ctx& c, Tile<EW> t, int lane) {
  for (int w = lane; w < c.nb * 6 * EW; w += WAVE) t.f(c.L.rst + w / EW, w % EW) = a.ret_w[w / EW];
}
template <int EW>
CX_DEV void stage_ret_terms(const KArgs& a, const Ctx& c, Tile<EW> t, int lane) {
  const int nk = c.nb * 6;  // <= MAXB * 6 = 96
  const float w0 = lane < nk ? a.ret_w[lane] : 0.0f, w1 = lane + WAVE < nk ? a.ret_w[lane + WAVE] : 0.0f;
  const uint64_t m0 = ballot(w0 != 0.0f), m1 = ballot(w1 != 0.0f);
  const int n0 = popc64(m0), n = n0 + popc64(m1), cap = ret_terms_cap(c);
  const int r0 = popc64(m0 & lanes_below(lane)), r1 = n0 + popc64(m1 & lanes_below(lane));
  if (n <= cap) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float w = h ? w1 : w0;
      const int r = h ? r1 : r0;
      if (w != 0.0f)
        for (int e = 0; e < EW; ++e) {
          t.w(c.L.rst + 1 + 2 * r, e) = (uint32_t)(lane + h * WAVE);
          t.f(c.L.rst + 2 + 2 * r, e) = w;
        }
    }
  }
  if (lane < EW) t.w(c.L.rst, lane) = (uint32_t)n;
}
// backward: the saved state of step `step`, read into registers one step
// ahead (restore_fetch in the previous step's restore phase), so the global
// reads are in flight while that step re-plays and differentiates
struct RestoreRegs {
  float d[RQ];
  uint32_t k0 = 0u, k1 = 0u;
};
template <int EW>
CX_DEV void restore_fetch(const KArgs& a, const Ctx& c, int env0, int lane, int step, RestoreRegs& r) {
  const int nd = c.nb * 6 * EW;
#pragma unroll
  for (int q = 0; q < RQ; ++q) {
    const int w = q * WAVE + lane, e = w % EW, off = w / EW, g = env0 + e;
    if (q * WAVE >= nd) break;  // uniform
    const bool ok = w < nd && g < a.B;
    r.d[q] = ok ? a.save_dyn[row_at(a.B, c.nb * 6, step, ok ? off : 0, ok ? g : 0)] : 0.0f;
  }
  const int g = env0 + lane;
  const bool le = lane < EW && g < a.B;
  r.k0 = le ? a.save_keys[2 * ((size_t)step * a.B + g)] : 0u;
  r.k1 = le ? a.save_keys[2 * ((size_t)step * a.B + g) + 1] : 0u;
}
template <int EW>
CX_DEV void restore_apply(const Ctx& c, Tile<EW> t, int lane, const RestoreRegs& r) {
  const int nd = c.nb * 6 * EW;
#pragma unroll
  for (int q = 0; q < RQ; ++q) {
    const int w = q * WAVE + lane;
    if (q * WAVE >= nd) break;  // uniform
    if (w < nd) t.f(c.L.dyn + w / EW, w % EW) = r.d[q];
  }
  if (lane < EW) {
    t.w(c.L.key, lane) = r.k0;
    t.w(c.L.key + 1, lane) = r.k1;
    t.w(c.L.err, lane) = 0u;
  }
}

// the backward's tape words of step `step` (MODE 4), read into registers one
// step ahead like the saved state: per (body i, env) item (lane mapping of
// phase D), the resolution word and its contact; the recorded EPA edge of the
// resolution's contact (polygon scenes) is read once the step's resolution
// words are current (tape_edge_fetch)
// (TR: the program can meet an analytic scene -- FNSET analytic; the polygon
// programs' scenes are never analytic, launch_fnset)
template <int EW, bool TR>
CX_DEV void tape_fetch(const KArgs& a, const Ctx& c, int env0, int lane, int step, TapeRegs& r) {
  const int ni = c.nb * EW;
#pragma unroll
  for (int q = 0; q < TQ; ++q) {
    if (q * WAVE >= ni) break;  // uniform
    const int w = q * WAVE + lane, e = w % EW, i = w / EW, g = env0 + e;
    const bool ok = w < ni && g < a.B;
    const uint32_t* p = a.tape + row_at(a.B, a.tw, step, 5 * (ok ? i : 0), ok ? g : 0);  // (rows 4 words apart)
#pragma unroll
    for (int k = 0; k < 5; ++k) r.d[q][k] = ok ? p[4 * k] : RP_NONE;
    if (TR && tape_rec(c.sh)) {  // the resolution's record (read whether or not it resolved: no dependent round trip)
      const uint32_t* pr = a.tape + row_at(a.B, a.tw, step, 5 * c.nb + REC_W * (ok ? i : 0), ok ? g : 0);
#pragma unroll
      for (int k = 0; k < REC_W; ++k) r.x[q][k] = ok ? pr[4 * k] : 0u;
    }
  }
}
template <int EW>
CX_DEV void tape_edge_fetch(const KArgs& a, const Ctx& c, int env0, int lane, int step, TapeRegs& r) {
  const int ni = c.nb * EW;
#pragma unroll
  for (int q = 0; q < TQ; ++q) {
    if (q * WAVE >= ni) break;  // uniform
    const int w = q * WAVE + lane, g = env0 + w % EW;
    const bool ok = w < ni && g < a.B && r.d[q][0] != RP_NONE;
    const int cid = ok ? (int)((r.d[q][0] >> 8) & 511u) : 0;
    const uint32_t* p = a.tape + row_at(a.B, a.tw, step, 5 * c.nb + 4 * cid, ok ? g : 0);
#pragma unroll
    for (int k = 0; k < 4; ++k) r.x[q][k] = ok ? p[4 * k] : 0u;
  }
}

template <int EW>
CX_DEV void ph_adj_init(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane) {
  for (int w = lane; w < c.nb * 6 * EW; w += WAVE) {
    int e = w % EW, off = w / EW;
    t.f(c.L.adj + off, e) = a.ret_w[off];  // d ret / d state_T
  }
}

// d ret / d action[step] of env g: stored now (go == nullptr), or held in the
// env lane's registers (go) and stored by the next step's restore phase --
// before that phase issues its prefetch reads, so no later wait for the
// prefetched data (s_waitcnt vmcnt, which counts stores) also waits for a
// store issued after it (MODE 4, run_wave_backward_tape)
struct GradOut {
  float x = 0.0f, y = 0.0f;
  int step = -1;
};
CX_DEV void grad_action_out(const KArgs& a, int g, int step, float gx, float gy, GradOut* go) {
  if (go == nullptr) {
    a.grad_action[2 * ((size_t)step * a.B + g)] = gx;
    a.grad_action[2 * ((size_t)step * a.B + g) + 1] = gy;
  } else {
    go->x = gx;
    go->y = gy;
    go->step = step;
  }
}
CX_DEV void grad_action_flush(const KArgs& a, int env0, int lane, int EWn, GradOut& go) {
  const int g = env0 + lane;
  if (lane < EWn && go.step >= 0 && g < a.B) {
    a.grad_action[2 * ((size_t)go.step * a.B + g)] = go.x;
    a.grad_action[2 * ((size_t)go.step * a.B + g) + 1] = go.y;
  }
  go.step = -1;
}

// phase G: reverse of one step (one lane per env).  Entry: adj = d ret /
// d state_{step+1}; the tile holds the re-played step (post-Euler positions,
// contacts, choices, recorded pre-resolution velocities).  Exit: adj = d ret
// / d state_step, grad_action[step] written.
// a part's world geometry (the tile's world words) as a Shape
template <int EW>
CX_DEV cx::Shape world_shape(const Ctx& c, Tile<EW> t, int p, int e) {
  using namespace cx;
  Shape S;
  S.kind = t.ti(c.sh.o_pkind + p);
  S.n = S.kind == KIND_POLY ? t.ti(c.sh.o_pn + p) : 0;
  const int w = c.L.world + t.ti(c.sh.o_pwoff + p);
#pragma unroll
  for (int k = 0; k < 2 * MAXV; ++k) S.w[k] = (k < 4 || k < 2 * S.n) ? t.f(w + (k < 4 || k < 2 * S.n ? k : 0), e) : 0.0f;
  return S;
}
// the cotangent of part p's world vertices -> its body's (px, py, angle).
// A polygon's world part is Polygon.transform's forward_vector of the local
// vertices, re-sorted: world slot k holds the local vertex whose transform
// has its bits (phase TV1's exact arithmetic).  An AABB translates only
// (corners [up, (up.x, lo.y), lo, (lo.x, up.y)]).
template <int EW>
CX_DEV void part_pose_vjp(const Ctx& c, Tile<EW> t, int p, int e, const cx::Shape& W, const cx::VGrad& gv,
                          float* out) {
  using namespace cx;
  if (W.kind == KIND_AABB) {
    out[0] = ((gv.x[0] + gv.x[1]) + gv.x[2]) + gv.x[3];
    out[1] = ((gv.y[0] + gv.y[1]) + gv.y[2]) + gv.y[3];
    out[2] = 0.0f;
    return;
  }
  const Lay& L = c.L;
  const int b = t.ti(c.sh.o_pbody + p), o = L.dyn + 6 * b, lg = L.geo + t.ti(c.sh.o_pgoff + p);
  const float px = t.f(o, e), py = t.f(o + 1, e);
  float s, cs;
  sincos32(t.f(o + 4, e), &s, &cs);
  float gpx = 0.0f, gpy = 0.0f, gang = 0.0f;
  for (int j = 0; j < W.n; ++j) {
    const float x = t.f(lg + 2 * j, e), y = t.f(lg + 2 * j + 1, e);
    const float t0 = (cs * x + (-s) * y) + px * 1.0f, t1 = (s * x + cs * y) + py * 1.0f;
    v2 g = v2{0.0f, 0.0f};
    bool found = false;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {  // the slot holding this vertex (first match)
      const bool hit = k < W.n && !found && W.w[2 * k] == t0 && W.w[2 * k + 1] == t1;
      g.x = hit ? gv.x[k] : g.x;
      g.y = hit ? gv.y[k] : g.y;
      found = found || hit;
    }
    gpx += g.x;
    gpy += g.y;
    gang += drot_dot(g, v2{x, y}, s, cs);
  }
  out[0] = gpx;
  out[1] = gpy;
  out[2] = gang;
}
// the joints of LunarLander.step in reverse (cotix_grad.h fixed_vjp): the
// tile holds the post-collider, pre-joint bodies (the re-play skips them)
template <int EW>
CX_DEV void joints_vjp(const Ctx& c, Tile<EW> t, int e) {
  using namespace cx;
  const Lay& L = c.L;
  Dyn d[3], g[3];
  Params m[3];
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    const int o = L.dyn + 6 * b, q = L.adj + 6 * b;
    d[b] = Dyn{t.f(o, e), t.f(o + 1, e), t.f(o + 2, e), t.f(o + 3, e), t.f(o + 4, e), t.f(o + 5, e)};
    g[b] = Dyn{t.f(q, e), t.f(q + 1, e), t.f(q + 2, e), t.f(q + 3, e), t.f(q + 4, e), t.f(q + 5, e)};
    m[b] = body_par<EW>(c, t, b, e);
  }
  // forward (lunar_constraints, the same expressions): anchors, then the
  // bodies before each of the four impulse pairs
  const float f05 = 0.05f;
  float sn[3], cn[3];
#pragma unroll
  for (int b = 0; b < 3; ++b) sincos32(d[b].a, &sn[b], &cn[b]);
  auto rot = [](v2 v, float s_, float c_) { return v2{c_ * v.x + (-s_) * v.y, s_ * v.x + c_ * v.y}; };
  const v2 lp = v2{d[0].px, d[0].py};
  const v2 loc[4] = {v2{24.0f * f05, -8.0f * f05}, v2{24.0f * f05, 0.0f * f05}, v2{-24.0f * f05, -8.0f * f05},
                     v2{-24.0f * f05, 0.0f * f05}};
  const v2 tip = v2{0.0f, 0.4f};
  v2 c1[4], c2[4];
  int leg[4];
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    leg[f] = f < 2 ? 2 : 1;  // left leg (body 2) for the first pair, right leg (body 1) for the second
    const Dyn& L2 = d[leg[f]];
    c1[f] = add(rot(loc[f], sn[0], cn[0]), lp);
    c2[f] = (f & 1) ? add(v2{L2.px, L2.py}, rot(tip, sn[leg[f]], cn[leg[f]])) : v2{L2.px, L2.py};
  }
  Dyn pre1[4], pre2[4];
  Dyn cur[3] = {d[0], d[1], d[2]};
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    pre1[f] = cur[0];
    pre2[f] = cur[leg[f]];
    Dyn& b1 = cur[0];
    Dyn& b2 = cur[leg[f]];
    const v2 dp = sub(c1[f], c2[f]);
    const v2 dv = sub(velocity_at(b1, c1[f]), velocity_at(b2, c2[f]));
    const float k = nrm(dv) + 0.1f;
    const v2 imp = v2{dp.x * 1.0f + (dv.x * k) * f05, dp.y * 1.0f + (dv.y * k) * f05};
    auto apply = [](Dyn& b, const Params& mm, v2 im, v2 pt) {
      const v2 arm = sub(pt, v2{b.px, b.py});
      const float torque = crs(arm, im);
      b.vx = b.vx + im.x / mm.mass;
      b.vy = b.vy + im.y / mm.mass;
      b.w = b.w + torque / mm.inertia;
    };
    apply(b1, m[0], neg(imp), c1[f]);
    apply(b2, m[leg[f]], imp, c2[f]);
  }
  // reverse
  g[1].w = g[1].w * 0.95f;
  g[2].w = g[2].w * 0.95f;
  v2 gc1[4], gc2[4];
#pragma unroll
  for (int f = 3; f >= 0; --f) {
    gc1[f] = v2{0.0f, 0.0f};
    gc2[f] = v2{0.0f, 0.0f};
    fixed_vjp(pre1[f], m[0], c1[f], pre2[f], m[leg[f]], c2[f], g[0], g[leg[f]], gc1[f], gc2[f]);
  }
#pragma unroll
  for (int f = 0; f < 4; ++f) {  // anchors: rotate(local, angle) + position
    g[0].px += gc1[f].x;
    g[0].py += gc1[f].y;
    g[0].a += drot_dot(gc1[f], loc[f], sn[0], cn[0]);
    Dyn& gl = g[leg[f]];
    gl.px += gc2[f].x;
    gl.py += gc2[f].y;
    if (f & 1) gl.a += drot_dot(gc2[f], tip, sn[leg[f]], cn[leg[f]]);
  }
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    const int q = L.adj + 6 * b;
    t.f(q, e) = g[b].px;
    t.f(q + 1, e) = g[b].py;
    t.f(q + 2, e) = g[b].vx;
    t.f(q + 3, e) = g[b].vy;
    t.f(q + 4, e) = g[b].a;
    t.f(q + 5, e) = g[b].w;
  }
}

// phase GE (polygon backward): the GJK/EPA contacts' derivatives, ahead of
// the serial adjoint chain of phase G.  A contact's VJP is linear in its
// cotangent (pen, cp), so item = (basis k, resolution i, env) computes the
// VJP of the unit cotangent k (pen.x, pen.y, cp.x, cp.y) down to the two
// bodies' (px, py, angle) (cotix_grad.h convex_contact_vjp: GJK, EPA's final
// edge -- in the lane's LDS column, as phase B -- contact_from_edges;
// part_pose_vjp): 24 words per resolution in the key-window words, which the
// backward does not use (it splits each step's keys in phase A); phase G
// contracts them with the contact's actual cotangent.  Scenes whose 24 * nb
// words exceed the key window do the VJP inside phase G instead.
CX_HD bool ge_fits(const Ctx& c) { return 24 * c.nb <= KWIN * c.L.kww; }
template <int EW>
CX_DEV int ge_word(const Ctx& c, int i, int k) {
  return c.L.kw + 24 * i + 6 * k;
}
// EDGES (MODE 4): EPA's final edge from the tape (ge_edge_word) instead of a
// GJK + EPA re-run
template <int EW, bool EDGES = false>
CX_DEV void ph_GE(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane) {
  using namespace cx;
  const SceneHdr& sc = c.sh;
  const Lay& L = c.L;
  float* col = reinterpret_cast<float*>(t.ws + c.W.epa + lane);
  for (int w = lane; w < c.nb * EW * 4; w += WAVE) {
    const int e = w % EW, q = w / EW, i = q >> 2, k = q & 3;
    if (env0 + e >= a.B || t.w(L.rec + REC_W * i, e) == 0u) continue;
    const int j = (int)t.w(L.ch + i, e);
    const int cid = (int)((t.w(L.m + i * c.nb + j, e) >> 18) & 511u);
    const int fn = t.ti(sc.o_cfn + cid);
    if (fn != FN_POLY_POLY && fn != FN_AABB_POLY) continue;
    const int pa = t.ti(sc.o_cpa + cid), pb = t.ti(sc.o_cpb + cid);
    const Shape WA = world_shape<EW>(c, t, pa, e), WB = world_shape<EW>(c, t, pb, e);
    VGrad va, vb;
    va.zero();
    vb.zero();
    const v2 gpen = v2{k == 0 ? 1.0f : 0.0f, k == 1 ? 1.0f : 0.0f}, gcp = v2{k == 2 ? 1.0f : 0.0f, k == 3 ? 1.0f : 0.0f};
    if (EDGES) {
      const int eo = ge_edge_word(c, i);
      const v2 e0 = v2{t.f(eo, e), t.f(eo + 1, e)}, e1 = v2{t.f(eo + 2, e), t.f(eo + 3, e)};
      convex_contact_vjp_edge(WA, WB, e0, e1, gpen, gcp, va, vb);
    } else {
      convex_contact_vjp(WA, WB, narrow_of(sc), gpen, gcp, va, vb, MakeCol{col, WAVE});
    }
    float o[6];
    part_pose_vjp<EW>(c, t, pa, e, WA, va, o);
    part_pose_vjp<EW>(c, t, pb, e, WB, vb, o + 3);
    const int ow = ge_word<EW>(c, i, k);
#pragma unroll
    for (int r = 0; r < 6; ++r) t.f(ow + r, e) = o[r];
  }
}

// phase G of an analytic scene with NB bodies on the env's lane: the same
// reverse chain as ph_G's tile form, with the adjoints, positions and each
// resolution's flag and partner in registers (bodies picked by unrolled
// selects, no scratch) -- the resolutions' LDS reads are then independent of
// the previous resolution's writes, and the Euler / return terms run on
// registers.  Every operation and its order are ph_G's: the same bits.
// g_chain: the step's reverse on the adjoints g held by the caller (g_regs
// reads them from and writes them to the tile's adj words; the split backward's
// consumer wave carries them in registers from step to step)
// TILE: the adjoints are read from and written to the tile's adj words inside
// the chain's own loops (g_regs: the one-wave form's schedule, the adjoints
// live only across one step); otherwise the caller's registers carry them
template <int EW, int NB, bool TILE = false>
CX_DEV void g_chain(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int e, int step, float (&g)[NB][6],
                    GradOut* go = nullptr) {
  using namespace cx;
  const SceneHdr& sc = c.sh;
  const Lay& L = c.L;
  float px[NB], py[NB], an[NB];
  uint32_t fl[NB], jj[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    if (TILE)
#pragma unroll
      for (int k = 0; k < 6; ++k) g[b][k] = t.f(L.adj + 6 * b + k, e);
    px[b] = t.f(L.dyn + 6 * b, e);
    py[b] = t.f(L.dyn + 6 * b + 1, e);
    an[b] = t.f(L.dyn + 6 * b + 4, e);
    fl[b] = t.w(L.rec + REC_W * b, e);
    jj[b] = t.w(L.ch + b, e);
  }
  if (a.stages & COTIX_STAGE_COLLIDER) {
#pragma unroll
    for (int i = NB - 1; i >= 0; --i) {  // resolutions in reverse order
      if (fl[i] == 0u) continue;
      const int j = (int)jj[i];
      const int ro = L.rec + REC_W * i;
      const int cid = (int)((t.w(L.m + i * NB + j, e) >> 18) & 511u);
      const int co = L.con + 4 * cid;
      float pxj = 0.0f, pyj = 0.0f, anj = 0.0f;
      Dyn gj = Dyn{0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int b = 0; b < NB; ++b)
        if (b == j) {
          pxj = px[b];
          pyj = py[b];
          anj = an[b];
          gj = Dyn{g[b][0], g[b][1], g[b][2], g[b][3], g[b][4], g[b][5]};
        }
      const Dyn bi = Dyn{px[i], py[i], t.f(ro + 1, e), t.f(ro + 2, e), an[i], t.f(ro + 3, e)};
      const Dyn bj = Dyn{pxj, pyj, t.f(ro + 4, e), t.f(ro + 5, e), anj, t.f(ro + 6, e)};
      Dyn gi = Dyn{g[i][0], g[i][1], g[i][2], g[i][3], g[i][4], g[i][5]};
      v2 gpen = v2{0.0f, 0.0f}, gcp = v2{0.0f, 0.0f};
      resolve_vjp(bi, body_par<EW>(c, t, i, e), bj, body_par<EW>(c, t, j, e),
                  v2{t.f(co, e), t.f(co + 1, e)}, v2{t.f(co + 2, e), t.f(co + 3, e)}, gi, gj, gpen, gcp, baum_of(sc));
      const int pa = t.ti(sc.o_cpa + cid), pb = t.ti(sc.o_cpb + cid), fn = t.ti(sc.o_cfn + cid);
      const int ka = t.ti(sc.o_pkind + pa), kb = t.ti(sc.o_pkind + pb);
      const int wa = L.world + t.ti(sc.o_pwoff + pa), wb = L.world + t.ti(sc.o_pwoff + pb);
      Shape SA, SB;
      SA.kind = ka;
      SB.kind = kb;
      SA.n = SB.n = 0;
      for (int k = 0; k < 2 * MAXV; ++k) SA.w[k] = SB.w[k] = 0.0f;
      for (int k = 0; k < 4; ++k) {
        SA.w[k] = t.f(wa + k, e);
        SB.w[k] = t.f(wb + k, e);
      }
      float ga[4] = {0.0f, 0.0f, 0.0f, 0.0f}, gb[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      contact_vjp(fn, SA, SB, gpen, gcp, ga, gb);
      const float gw[6] = {gi.px, gi.py, gi.vx, gi.vy, gi.a, gi.w}, hw[6] = {gj.px, gj.py, gj.vx, gj.vy, gj.a, gj.w};
#pragma unroll
      for (int k = 0; k < 6; ++k) g[i][k] = gw[k];
      const int qa = t.ti(sc.o_pbody + pa), qb = t.ti(sc.o_pbody + pb);
      const float ax = ka == KIND_CIRCLE ? ga[1] : ga[0] + ga[2], ay = ka == KIND_CIRCLE ? ga[2] : ga[1] + ga[3];
      const float bx = kb == KIND_CIRCLE ? gb[1] : gb[0] + gb[2], by = kb == KIND_CIRCLE ? gb[2] : gb[1] + gb[3];
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        if (b == j)
#pragma unroll
          for (int k = 0; k < 6; ++k) g[b][k] = hw[k];
      }
#pragma unroll
      for (int b = 0; b < NB; ++b)
        if (b == qa) {
          g[b][0] = g[b][0] + ax;
          g[b][1] = g[b][1] + ay;
        }
#pragma unroll
      for (int b = 0; b < NB; ++b)
        if (b == qb) {
          g[b][0] = g[b][0] + bx;
          g[b][1] = g[b][1] + by;
        }
    }
  }
  const int g_env = env0 + e;
  if (a.action != nullptr && a.grad_action != nullptr) {  // v[action_body] += action[step]
    float gx = 0.0f, gy = 0.0f;
#pragma unroll
    for (int b = 0; b < NB; ++b)
      if (b == a.action_body) {
        gx = g[b][2];
        gy = g[b][3];
      }
    grad_action_out(a, g_env, step, gx, gy, go);
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    if (a.stages & COTIX_STAGE_EULER) {  // p += v dt, angle += w dt
      g[b][2] = g[b][2] + g[b][0] * a.dt;
      g[b][3] = g[b][3] + g[b][1] * a.dt;
      g[b][5] = g[b][5] + g[b][4] * a.dt;
    }
    if (step > 0)
#pragma unroll
      for (int k = 0; k < 6; ++k) g[b][k] = g[b][k] + t.f(L.rst + 6 * b + k, e);  // ret_w (staged)
    if (TILE)
#pragma unroll
      for (int k = 0; k < 6; ++k) t.f(L.adj + 6 * b + k, e) = g[b][k];
  }
}
template <int EW, int NB>
CX_DEV void g_regs(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int e, int step, GradOut* go = nullptr) {
  float g[NB][6];
  g_chain<EW, NB, true>(a, c, t, env0, e, step, g, go);
}

template <int EW, int FNSET = FNS_ANALYTIC>
CX_DEV void ph_G(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane, int step, GradOut* go = nullptr) {
  using namespace cx;
  const SceneHdr& sc = c.sh;
  const int nb = c.nb;
  const Lay& L = c.L;
  for (int e = lane; e < EW; e += WAVE) {
    const int g = env0 + e;
    if (g >= a.B) continue;
#ifndef COTIX_NO_GREGS  // (tooling: the tile form for every scene, tests/test_grad_cpu.py checks the two agree)
    if (FNSET == FNS_ANALYTIC && nb == 5) {  // RoboCup
      g_regs<EW, 5>(a, c, t, env0, e, step, go);
      continue;
    }
    if (FNSET == FNS_ANALYTIC && nb == 7) {  // the box world
      g_regs<EW, 7>(a, c, t, env0, e, step, go);
      continue;
    }
#endif
    if (FNSET != FNS_ANALYTIC && (a.stages & COTIX_STAGE_LUNAR) && nb >= 3) joints_vjp<EW>(c, t, e);
    if (a.stages & COTIX_STAGE_COLLIDER) {
      for (int i = nb - 1; i >= 0; --i) {  // resolutions in reverse order
        const int ro = L.rec + REC_W * i;
        if (t.w(ro, e) == 0u) continue;
        const int j = (int)t.w(L.ch + i, e);
        const int cid = (int)((t.w(L.m + i * nb + j, e) >> 18) & 511u);
        const int co = L.con + 4 * cid, oi = L.dyn + 6 * i, oj = L.dyn + 6 * j;
        const Dyn bi = Dyn{t.f(oi, e), t.f(oi + 1, e), t.f(ro + 1, e), t.f(ro + 2, e), t.f(oi + 4, e), t.f(ro + 3, e)};
        const Dyn bj = Dyn{t.f(oj, e), t.f(oj + 1, e), t.f(ro + 4, e), t.f(ro + 5, e), t.f(oj + 4, e), t.f(ro + 6, e)};
        const int ai = L.adj + 6 * i, aj = L.adj + 6 * j;
        Dyn gi = Dyn{t.f(ai, e), t.f(ai + 1, e), t.f(ai + 2, e), t.f(ai + 3, e), t.f(ai + 4, e), t.f(ai + 5, e)};
        Dyn gj = Dyn{t.f(aj, e), t.f(aj + 1, e), t.f(aj + 2, e), t.f(aj + 3, e), t.f(aj + 4, e), t.f(aj + 5, e)};
        v2 gpen = v2{0.0f, 0.0f}, gcp = v2{0.0f, 0.0f};
        resolve_vjp(bi, body_par<EW>(c, t, i, e), bj, body_par<EW>(c, t, j, e),
                    v2{t.f(co, e), t.f(co + 1, e)}, v2{t.f(co + 2, e), t.f(co + 3, e)}, gi, gj, gpen, gcp,
                    baum_of(sc));
        // the contact: fn(world(part pa), world(part pb)); world = local + body position
        const int pa = t.ti(sc.o_cpa + cid), pb = t.ti(sc.o_cpb + cid), fn = t.ti(sc.o_cfn + cid);
        const int ka = t.ti(sc.o_pkind + pa), kb = t.ti(sc.o_pkind + pb);
        const int wa = L.world + t.ti(sc.o_pwoff + pa), wb = L.world + t.ti(sc.o_pwoff + pb);
        if ((FNSET & FNS_CIRCLE_POLY) != 0 && fn == FN_CIRCLE_POLY) {
          // circle x polygon: the whole GJK / EPA chain through the circle's
          // support (cx::circle_poly_vjp; a = the circle, b = the polygon)
          const float gw_[12] = {gi.px, gi.py, gi.vx, gi.vy, gi.a, gi.w, gj.px, gj.py, gj.vx, gj.vy, gj.a, gj.w};
#pragma unroll
          for (int k = 0; k < 6; ++k) {
            t.f(ai + k, e) = gw_[k];
            t.f(aj + k, e) = gw_[6 + k];
          }
          const Shape WA = world_shape<EW>(c, t, pa, e), WB = world_shape<EW>(c, t, pb, e);
          v2 gc = v2{0.0f, 0.0f};
          VGrad vb;
          vb.zero();
          circle_poly_vjp(WA, WB, narrow_of(sc), gpen, gcp, &gc, vb);
          float gp[3] = {0.0f, 0.0f, 0.0f};
          part_pose_vjp<EW>(c, t, pb, e, WB, vb, gp);
          const int qa = L.adj + 6 * t.ti(sc.o_pbody + pa), qb = L.adj + 6 * t.ti(sc.o_pbody + pb);
          t.f(qa, e) = t.f(qa, e) + gc.x;  // the circle translates with its body
          t.f(qa + 1, e) = t.f(qa + 1, e) + gc.y;
          t.f(qb, e) = t.f(qb, e) + gp[0];
          t.f(qb + 1, e) = t.f(qb + 1, e) + gp[1];
          t.f(qb + 4, e) = t.f(qb + 4, e) + gp[2];
          continue;
        }
        if (FNSET != FNS_ANALYTIC && (fn == FN_POLY_POLY || fn == FN_AABB_POLY)) {
          // (store the resolution's body cotangents first: the contact's go on top)
          const float gw_[12] = {gi.px, gi.py, gi.vx, gi.vy, gi.a, gi.w, gj.px, gj.py, gj.vx, gj.vy, gj.a, gj.w};
#pragma unroll
          for (int k = 0; k < 6; ++k) {
            t.f(ai + k, e) = gw_[k];
            t.f(aj + k, e) = gw_[6 + k];
          }
          float gp[6] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
          if (ge_fits(c)) {  // the contact's VJP from phase GE's basis responses
            const float gk[4] = {gpen.x, gpen.y, gcp.x, gcp.y};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const int m = ge_word<EW>(c, i, k);
#pragma unroll
              for (int q = 0; q < 6; ++q) gp[q] += gk[k] * t.f(m + q, e);
            }
          } else {
            const Shape WA = world_shape<EW>(c, t, pa, e), WB = world_shape<EW>(c, t, pb, e);
            VGrad va, vb;
            va.zero();
            vb.zero();
            convex_contact_vjp(WA, WB, narrow_of(sc), gpen, gcp, va, vb);
            part_pose_vjp<EW>(c, t, pa, e, WA, va, gp);
            part_pose_vjp<EW>(c, t, pb, e, WB, vb, gp + 3);
          }
          const int qa = L.adj + 6 * t.ti(sc.o_pbody + pa), qb = L.adj + 6 * t.ti(sc.o_pbody + pb);
          t.f(qa, e) = t.f(qa, e) + gp[0];
          t.f(qa + 1, e) = t.f(qa + 1, e) + gp[1];
          t.f(qa + 4, e) = t.f(qa + 4, e) + gp[2];
          t.f(qb, e) = t.f(qb, e) + gp[3];
          t.f(qb + 1, e) = t.f(qb + 1, e) + gp[4];
          t.f(qb + 4, e) = t.f(qb + 4, e) + gp[5];
          continue;
        }
        Shape SA, SB;
        SA.kind = ka;
        SB.kind = kb;
        SA.n = SB.n = 0;
        for (int k = 0; k < 2 * MAXV; ++k) SA.w[k] = SB.w[k] = 0.0f;
        for (int k = 0; k < 4; ++k) {
          SA.w[k] = t.f(wa + k, e);
          SB.w[k] = t.f(wb + k, e);
        }
        float ga[4] = {0.0f, 0.0f, 0.0f, 0.0f}, gb[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        contact_vjp(fn, SA, SB, gpen, gcp, ga, gb);
        t.f(ai, e) = gi.px;
        t.f(ai + 1, e) = gi.py;
        t.f(ai + 2, e) = gi.vx;
        t.f(ai + 3, e) = gi.vy;
        t.f(ai + 4, e) = gi.a;
        t.f(ai + 5, e) = gi.w;
        t.f(aj, e) = gj.px;
        t.f(aj + 1, e) = gj.py;
        t.f(aj + 2, e) = gj.vx;
        t.f(aj + 3, e) = gj.vy;
        t.f(aj + 4, e) = gj.a;
        t.f(aj + 5, e) = gj.w;
        const int qa = L.adj + 6 * t.ti(sc.o_pbody + pa), qb = L.adj + 6 * t.ti(sc.o_pbody + pb);
        if (ka == KIND_CIRCLE) {
          t.f(qa, e) = t.f(qa, e) + ga[1];
          t.f(qa + 1, e) = t.f(qa + 1, e) + ga[2];
        } else {
          t.f(qa, e) = t.f(qa, e) + (ga[0] + ga[2]);
          t.f(qa + 1, e) = t.f(qa + 1, e) + (ga[1] + ga[3]);
        }
        if (kb == KIND_CIRCLE) {
          t.f(qb, e) = t.f(qb, e) + gb[1];
          t.f(qb + 1, e) = t.f(qb + 1, e) + gb[2];
        } else {
          t.f(qb, e) = t.f(qb, e) + (gb[0] + gb[2]);
          t.f(qb + 1, e) = t.f(qb + 1, e) + (gb[1] + gb[3]);
        }
      }
    }
    if (a.action != nullptr && a.grad_action != nullptr) {  // v[action_body] += action[step]
      const int o = L.adj + 6 * a.action_body;
      grad_action_out(a, g, step, t.f(o + 2, e), t.f(o + 3, e), go);
    }
    for (int b = 0; b < nb; ++b) {
      const int o = L.adj + 6 * b;
      if (a.stages & COTIX_STAGE_EULER) {  // p += v dt, angle += w dt
        t.f(o + 2, e) = t.f(o + 2, e) + t.f(o + 0, e) * a.dt;
        t.f(o + 3, e) = t.f(o + 3, e) + t.f(o + 1, e) * a.dt;
        t.f(o + 5, e) = t.f(o + 5, e) + t.f(o + 4, e) * a.dt;
      }
      if (step > 0)
        for (int k = 0; k < 6; ++k) t.f(o + k, e) = t.f(o + k, e) + t.f(L.rst + 6 * b + k, e);  // ret_w (staged)
    }
  }
}

template <int EW>
CX_DEV void ph_adj_store(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int lane) {
  if (a.grad_dyn == nullptr) return;
  for (int w = lane; w < c.nb * 6 * EW; w += WAVE) {
    int e = w % EW, off = w / EW, g = env0 + e;
    if (g < a.B) a.grad_dyn[(size_t)off * a.B + g] = t.f(c.L.adj + off, e);
  }
}

// ---------------------------------------------------------------------------
// the wave programs.  R runs one phase over the wave's lanes and orders it
// before the next: on the GPU R = this lane + wave_sync(); in the CPU
// emulation of the tests R loops over the 64 lanes.  The phase id is used
// only by the phase-timing build (COTIX_PHASE_PROF, tools/phase_prof.py).
enum : int { PH_LOAD, PH_SAVE, PH_A, PH_T, PH_B, PH_C0, PH_C0B, PH_C1, PH_C2, PH_C3, PH_D, PH_E, PH_RET, PH_STORE,
             PH_RESTORE, PH_G, PH_ADJ, PH_F, PH_K, PH_E1, PH_R, PH_TRACE, PH_BP0, PH_BP1, PH_F0, PH_F1, PH_F2, PH_F3,
             PH_TV0, PH_TV1, PH_TV2, PH_TV3, PH_J, PH_GE, PH_COUNT };
// ---------------------------------------------------------------------------
// kso: tile offset of this step's sk0 (skt follows): the key window slot, or
// L.sk0 where phase A splits the keys (backward re-play)
// AB: phases A, T and B ran as one (ab_fetch / ph_A / ab_contacts, analytic forward programs)
// phase T and (polygon scenes) TV0-TV4: the world parts of the step
template <int EW, int FNSET, class R>
CX_DEV void transform_phases(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, const R& run) {
  {
    run(PH_T, [&](int l) { ph_T<EW, FNSET>(a, c, t, env0, l); });
    if (FNSET != FNS_ANALYTIC && c.sh.nvt > 0) {
      // the rebuild flags of TV0 and the chunks they make run, wave-uniform:
      // computed once for TV1-TV4.  TV0 runs in TV1's phase (the flags are
      // ballot from each lane's own word; TV1 reads none of TV0's other words)
      uint64_t redo = 0ull;
      uint32_t runs = 0u;
      run(PH_TV1, [&](int l) {
        ph_TV0<EW>(a, c, t, env0, l);
        redo = tv_redo_mask<EW>(c, t, l);
        runs = tv_chunks<EW>(c, t, redo);
        ph_TV1<EW>(a, c, t, env0, l, redo, runs);
      });
      run(PH_TV2, [&](int l) { ph_TV2<EW>(a, c, t, env0, l, redo, runs); });
      run(PH_TV3, [&](int l) { ph_TV3<EW>(a, c, t, env0, l, redo, runs); });
      if ((FNSET & FNS_CONVEX) != 0 && c.sh.poly && (a.stages & COTIX_STAGE_BROADPHASE) && !CXK_SKIP(a, 2))
        run(PH_TV3, [&](int l) { ph_TV4<EW>(a, c, t, env0, l, redo, runs); });
#ifdef COTIX_EMU_POISON
      // test instrumentation (the host emulation's build): the vertex items
      // die with phase T -- poison them so that a later step reading stale
      // ones cannot pass by luck
      run(PH_TV3, [&](int l) {
        for (int q = l; q < 3 * c.sh.nvt * EW; q += WAVE) t.ws[c.W.vt + q] = 0x7FBADBADu;
      });
#endif
    }
  }
}
// TAPE: the rollout forward with a tape (phase B records EPA's edges)
template <int EW, int FNSET, bool PRE, class R, bool AB = false, bool TAPE = false>
CX_DEV void collider_phases(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, const R& run, int slot, int kso,
                            const MConst& mc, int step = 0) {
  if (!AB && !CXK_SKIP(a, 1)) transform_phases<EW, FNSET>(a, c, t, env0, run);
  if ((FNSET & FNS_CONVEX) != 0 && c.sh.poly && (a.stages & COTIX_STAGE_BROADPHASE) && !CXK_SKIP(a, 2)) {
    run(PH_BP0, [&](int l) { ph_BP0<EW>(a, c, t, env0, l); });
    const int n = (int)t.ws[c.W.bl_n];  // uniform: read after the phase barrier
    CXK_STAT(b_items, 0);
    const bool pairs = b_pairs<FNSET>() && t.ws[c.W.bl_mode] != 0u;  // uniform: read after the barrier
    const int per_round = pairs ? WAVE / 2 : WAVE;
    for (int r = 0; r * per_round < n; ++r)
      run(PH_B, [&](int l) { ph_BP2<EW, FNSET, TAPE>(a, c, t, env0, l, r, pairs, step); });
  } else if (!AB && !CXK_SKIP(a, 2)) {
    run(PH_B, [&](int l) { ph_B<EW, FNSET, TAPE>(a, c, t, env0, l, step); });
  }
  if ((FNSET & FNS_CONVEX) != 0 && c.sh.poly && !CXK_SKIP(a, 2)) {
    for (int ch = 0; ch * WAVE < c.nc * EW; ++ch) run(PH_F0, [&](int l) { ph_F0<EW>(c, t, l, ch); });
    const int n = (int)t.ws[c.W.cf_n];
    CXK_STAT(f_items, n);
    for (int b = 0; b < n; b += CFB) {
      run(PH_F1, [&](int l) { ph_F1<EW>(c, t, l, b); });
      int TC = 0, TE = 0;
      for (int i = 0; i < CFB; ++i) {
        TC += (int)t.ws[c.W.cf_c + i];
        TE += (int)t.ws[c.W.cf_s + i] - (int)t.ws[c.W.cf_c + i];
      }
      for (int r = 0; r * WAVE < TC; ++r) run(PH_F2, [&](int l) { ph_F2<EW, false>(c, t, l, b, r); });
      for (int r = 0; r * WAVE < TE; ++r) run(PH_F2, [&](int l) { ph_F2<EW, true>(c, t, l, b, r); });
      run(PH_F3, [&](int l) { ph_F3<EW>(c, t, l, b); });
    }
  }
  if (!CXK_SKIP(a, 4) && c.nl > 0 && scan_fused<EW>(c)) {
    run(PH_C1, [&](int l) { ph_M_fused<EW>(a, c, t, env0, l, kso, mc); });
  } else if (!CXK_SKIP(a, 4) && c.nl > 0) {
    for (int ch = 0; ch * WAVE < c.nl * EW; ++ch) {
      run(PH_C0, [&](int l) { ph_C0<EW>(a, c, t, env0, l, ch); });
      run(PH_C0B, [&](int l) { ph_C0b<EW>(c, t, l, ch); });
    }
    CXK_STAT(wave_steps, 1);
    CXK_STAT(active_items, t.ws[WS_N]);
    for (int par = 0; t.ws[WS_N] != 0u; par ^= 1) {  // uniform: read after the phase barrier
      CXK_STAT(rounds, 1);
      run(PH_C1, [&](int l) { ph_C1<EW>(a, c, t, l, par, kso); });
      run(PH_C2, [&](int l) { ph_C2<EW>(c, t, l, par); });
      run(PH_C3, [&](int l) { ph_C3<EW>(c, t, l, par); });
    }
  }
  if (!CXK_SKIP(a, 8)) run(PH_D, [&](int l) { ph_D<EW, PRE, TAPE>(a, c, t, env0, l, kso, step); });
}

// forward: n_steps fused steps; ROLL adds the trajectory save and the return
// (cotix_rollout), EVAL the device judge and control (cotix_eval with either
// on), both compiled out of the plain step kernel
// the forward programs' load phase (the kernel may run it before its
// workgroup barrier: it touches only the wave's own tile)
// ROLL: the incoming return is read with the state (ph_store adds the launch's
// sum to it without a read: a read at the end waited behind every store in
// flight, ~15 us per launch); it lives in the restart-counter word, which the
// rollout programs (no restarts, no counter) do not use
template <int EW, bool ROLL, bool EVAL = false>
CX_DEV void ph_load_fwd(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, int l) {
  const float r0 = (ROLL && l < EW && env0 + l < a.B) ? a.ret[env0 + l] : 0.0f;
  ph_load<EW, EVAL>(a, c, t, env0, l);
  if (ROLL) {
    for (int e = l; e < EW; e += WAVE) {
      t.f(c.L.ret, e) = 0.0f;
      t.f(c.L.nres, e) = r0;
    }
    stage_ret_terms<EW>(a, c, t, l);
  }
}
// ---------------------------------------------------------------------------
// The key-window helper (the step program at two waves per env group).  Phase
// K's window -- the driver key chain, the per-type keys and every body's
// choice uniform for 16 steps -- depends on the env's launch key only, never
// on the physics (the chain k_{s+1} = split(k_s)[0] is what phase E stores as
// the key; restarts keep it).  So a helper wave can compute window w + 1 while
// the env group's step wave runs the steps of window w: the step wave computes
// window 0 itself, then at each later window start waits at one workgroup
// barrier and reads the window from one of two buffers -- its own tile's key
// window (even windows) or the helper's (odd), `kwalt` words from it in the
// tile's [word][env] addressing.  The same K0 / K1 / K2 code writes the same
// words (K0 with the chain key carried in the helper lane's registers): the
// same bits (tests/test_emu_cpu.py runs it on the host emulation, the
// helper's window computed at the step wave's barrier).
// ---------------------------------------------------------------------------
struct NoKeyHelp {
  static constexpr bool on = false;
  int kwalt = 0;
  CX_MF void bar() const {}
};
template <int EW>
struct KeyHelper {
  Tile<EW> tm;  // the step wave's tile: window buffer 0 is its key window
  Tile<EW> th;  // a view whose key window is buffer 1 (th.u = buffer 1 - L.kw * EW)
  int env0 = 0;
  int w = 0;  // windows produced (window 0 is the step wave's)
  cx::key2 k = cx::key2{0u, 0u};  // this lane's (env, half) chain key at the next window
};
// K0 on the key in the lane's registers: items (env, half) on lanes < 2 EW,
// split_at_pair as ph_K0; write: the window's sk0 words (else only advance)
template <int EW>
CX_DEV void k0_regs(const KArgs& a, const Ctx& c, Tile<EW> t, int lane, int n, cx::key2& k, bool write) {
  using namespace cx;
  const Lay& L = c.L;
  for (int w = lane; w < 2 * EW; w += WAVE) {
    const int e = w >> 1, h = w & 1;
    for (int s = 0; s < n; ++s) {
      const key2 s0 = split_at_pair(k, 2u, 0u, h, c.sh.prng != 0);
      if (write && h == 0) {
        t.w(L.kw + s * L.kww, e) = s0.a;
        t.w(L.kw + s * L.kww + 1, e) = s0.b;
      }
      if (a.stages & COTIX_STAGE_ADVANCE_KEY) k = s0;
    }
  }
}
// the helper's start: the env's launch key (the input keys, as ph_load reads
// them), advanced past window 0
template <int EW, class R>
CX_DEV void key_helper_init(const KArgs& a, const Ctx& c, KeyHelper<EW>& h, const R& run) {
  run(PH_K, [&](int l) {
    const int e = l >> 1, g = h.env0 + e;
    if (l < 2 * EW && g < a.B) h.k = cx::key2{a.keys[2 * (size_t)g], a.keys[2 * (size_t)g + 1]};
    k0_regs<EW>(a, c, h.tm, l, a.n_steps < KWIN ? a.n_steps : KWIN, h.k, false);
  });
}
// window h.w + 1 (steps 16 (w + 1) ..) into buffer (w + 1) & 1
template <int EW, class R>
CX_DEV void key_helper_next(const KArgs& a, const Ctx& c, KeyHelper<EW>& h, const R& run) {
  const int w = ++h.w, step0 = w * KWIN, n = a.n_steps - step0 < KWIN ? a.n_steps - step0 : KWIN;
  const Tile<EW> t = (w & 1) ? h.th : h.tm;
  run(PH_K, [&](int l) { k0_regs<EW>(a, c, t, l, n, h.k, true); });
  run(PH_K, [&](int l) { ph_K1<EW>(c, t, l, n); });
  if (a.stages & COTIX_STAGE_COLLIDER) run(PH_K, [&](int l) { ph_K2<EW>(c, t, l, n); });
}
// the barriers of a launch with a helper: one per window after the first
CX_HD int key_helper_windows(const KArgs& a) { return a.n_steps > KWIN ? (a.n_steps - 1) / KWIN : 0; }
// a step wave's LDS region with a helper (tile + scratch, a multiple of EW
// words: the buffer offset kwalt is whole tile words) and the workgroup's LDS
// bytes (tables, wpb regions, wpb helper window buffers)
template <int EW>
CX_HD int help_region_words(const Ctx& c) { return (c.L.S * EW + c.W.words + EW - 1) / EW * EW; }
template <int EW>
CX_HD size_t help_lds_bytes(const SceneHdr& s, int wpb) {
  const Ctx c = make_ctx<EW>(s);
  return 4 * ((size_t)s.nhot + (size_t)wpb * (help_region_words<EW>(c) + KWIN * c.L.kww * EW));
}

template <int EW, int FNSET, bool ROLL, bool EVAL = false, bool SDEFER = false, class R = void, class H = NoKeyHelp>
CX_DEV void run_wave(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, const R& run, bool loaded = false,
                     const H& help = H{}) {
  static_assert(!(ROLL && EVAL), "the rollout has no judge");
  static_assert(!(H::on && (ROLL || EVAL)), "the key helper runs the step program only");
  if (!loaded) run(PH_LOAD, [&](int l) { ph_load_fwd<EW, ROLL, EVAL>(a, c, t, env0, l); });
  const bool keys = keys_on(a);
  if (EVAL && a.judge.on) {  // the first NFE's start
    run(PH_J, [&](int l) { ph_JB<EW>(a, c, t, env0, l); });
    run(PH_J, [&](int l) { ph_JS<EW>(c, t, l); });
  }

  // analytic scenes beyond the fused form's chunks: phase B's launch-constant
  // item words in registers for the whole launch (ph_B_const)
  const bool bconst = FNSET == FNS_ANALYTIC && c.nc * EW > ABQ * WAVE && c.nc * EW <= HQ * WAVE &&
                      (a.stages & COTIX_STAGE_COLLIDER) != 0 && !CXK_SKIP(a, 2) &&
                      a.n_steps >= COTIX_BCONST_MIN_STEPS;
  BConst bc;
  if (bconst) run(PH_B, [&](int l) { bc_fetch<EW>(c, t, l, bc); });
  MConst mc;  // the fused scan's launch-constant owner words
  if ((a.stages & COTIX_STAGE_COLLIDER) && c.nl > 0 && scan_fused<EW>(c))
    run(PH_C1, [&](int l) { mc_fetch<EW>(c, t, l, mc); });
  RetRegs rr;  // the rollout's return terms
  if (ROLL) run(PH_RET, [&](int l) { ret_fetch<EW>(c, t, l, rr); });
  // the actions one step ahead (act_fetch): an the next step's, ac this step's
  // (the rollout forward: from the action window instead, act_window_fill)
  // The rollout programs never hold an action in flight across the step
  // loop: its stores (the save phase) count in vmcnt too, and any read of a
  // register with a possibly pending load -- even a select that discards it
  // -- makes the compiler wait for every store before it (s_waitcnt vmcnt(0)
  // in phase A, ~1.2 k cycles per step).  ROLL: the window or, without one
  // (nb < 3 or no actions), the direct read in euler_item.
  const bool awin = ROLL && act_window<EW>(a, c);
  const bool apf = ROLL ? awin : act_prefetch<EW>(a, c);
  ActRegs an, ac;
  if (!ROLL && apf) run(PH_A, [&](int l) { act_fetch<EW>(a, c, env0, l, 0, an); });
  auto act_next = [&](int l, int step) {  // (in phase A, before its use: the read overlaps the step)
    if (ROLL) {  // (awin: the lane's item's env, act_fetch's lane mapping)
      if (awin) {
        const int o = c.L.rst + 2 * (step % AWIN);
        ac.x = t.f(o, l % EW);
        ac.y = t.f(o + 1, l % EW);
      }
    } else {
      ac = an;
      if (apf && !a.action_held && step + 1 < a.n_steps) act_fetch<EW>(a, c, env0, l, step + 1, an);
    }
  };
  // restarts deferred into phase A (restart_deferred)
  const bool staged = !bconst && FNSET == FNS_ANALYTIC && c.nc * EW <= ABQ * WAVE;
  const bool defer = restart_deferred(a) && (!staged || SDEFER);
  // the last step's restarts taken by the store (ph_store's rs; nothing reads
  // the state after the last phase E but the judge)
  const bool rstore = a.dyn_reset != nullptr && a.reset_mode == 1 && !(EVAL && a.judge.on);
  for (int step = 0; step < a.n_steps; ++step) {
    // (the window's reads before this step's save stores: they wait only for
    // the previous step's, long complete)
    if (awin && step % AWIN == 0) run(PH_K, [&](int l) { act_window_fill<EW>(a, c, t, env0, l, step); });
    if (ROLL) run(PH_SAVE, [&](int l) { ph_save<EW, FNSET == FNS_ANALYTIC>(a, c, t, env0, l, step); });
    const int slot = step % KWIN;
    if (H::on && keys && slot == 0 && step > 0) {
      help.bar();  // the helper's window (key_helper_next)
    } else if (keys && slot == 0 && !(step == 0 && k_in_prologue(a))) {
      const int n = a.n_steps - step < KWIN ? a.n_steps - step : KWIN;
      if (n == 1) {  // (a launch's last window: the keys from the tile)
        run(PH_K, [&](int l) {
          const uint32_t k0 = l < EW ? t.w(c.L.key, l) : 0u, k1 = l < EW ? t.w(c.L.key + 1, l) : 0u;
          k_one_regs<EW>(a, c, t, l, k0, k1);
        });
      } else {
        run(PH_K, [&](int l) { ph_K0<EW>(a, c, t, l, n); });
        run(PH_K, [&](int l) { ph_K1<EW>(c, t, l, n); });
        if (a.stages & COTIX_STAGE_COLLIDER) run(PH_K, [&](int l) { ph_K2<EW>(c, t, l, n); });
      }
    }
    // this step's sk0, skt in the key window (with a helper: odd windows in its buffer)
    const int kso = c.L.kw + (H::on && ((step / KWIN) & 1) ? help.kwalt : 0) + slot * c.L.kww;
    // phases A, T, B as one (circle / AABB scenes whose contact items fit the
    // phase's ABQ prefetched chunks; uniform)
    if (bconst) {  // phase A, then B from the launch-constant item words (no phase T)
      run(PH_A, [&](int l) {
        act_next(l, step);
        ph_A<EW, true, EVAL, true>(a, c, t, env0, l, step, slot, apf, ac);
      });
      if (a.stages & COTIX_STAGE_COLLIDER) {
        run(PH_B, [&](int l) { ph_B_const<EW>(a, c, t, env0, l, bc); });
        collider_phases<EW, FNSET, true, R, true, ROLL>(a, c, t, env0, run, slot, kso, mc, step);
      }
    } else if (FNSET == FNS_ANALYTIC && c.nc * EW <= ABQ * WAVE) {
      // stage 1 reads the pre-Euler state: every read is issued before phase
      // A's writes (stage 2); stage 3 computes the contacts
      run.template staged<ABRegs>(
          PH_B, [&](int l, ABRegs& r) { ab_fetch<EW, SDEFER>(a, c, t, l, r); },
          [&](int l) {
            act_next(l, step);
            ph_A<EW, true, EVAL, SDEFER>(a, c, t, env0, l, step, slot, apf, ac);
          },
          [&](int l, const ABRegs& r) { ab_contacts<EW>(a, c, t, env0, l, r); });
      if (a.stages & COTIX_STAGE_COLLIDER) collider_phases<EW, FNSET, true, R, FNSET == FNS_ANALYTIC, ROLL>(
          a, c, t, env0, run, slot, kso, mc, step);
    } else {
      run(PH_A, [&](int l) {
        act_next(l, step);
        ph_A<EW, true, EVAL, true>(a, c, t, env0, l, step, slot, apf, ac);
      });
      if (a.stages & COTIX_STAGE_COLLIDER)
        collider_phases<EW, FNSET, true, R, false, ROLL>(a, c, t, env0, run, slot, kso, mc, step);
    }
    if (a.trace_chosen != nullptr || a.trace_cells != nullptr)
      run(PH_TRACE, [&](int l) { ph_trace<EW>(a, c, t, env0, l, step); });
    if (!CXK_SKIP(a, 32)) {
      if (ROLL && FNSET == FNS_ANALYTIC && a.tape != nullptr && tape_rec(c.sh) && (a.stages & COTIX_STAGE_COLLIDER))
        run(PH_E1, [&](int l) { ph_E<EW, false, ROLL, true>(a, c, t, env0, l, kso, &rr); });
      else
        run(PH_E1, [&](int l) { ph_E<EW, false, ROLL>(a, c, t, env0, l, kso, &rr); });
      if (a.dyn_reset != nullptr && a.reset_mode == 1 && !defer && !(rstore && step == a.n_steps - 1))
        run(PH_R, [&](int l) { ph_R<EW>(c, t, l); });
    } else if (ROLL) {
      run(PH_RET, [&](int l) {
        for (int e = l; e < EW; e += WAVE)
          if (env0 + e < a.B) ret_accum<EW>(a, c, t, e, rr);
      });
    }
    if (EVAL && a.judge.on) {  // cotix_eval: NFE bookkeeping (cotix/_envs.py:77-117)
      run(PH_J, [&](int l) { ph_J<EW>(a, c, t, env0, l); });
      run(PH_J, [&](int l) { ph_JS<EW>(c, t, l); });
      if ((step + 1) % a.nfe_len == 0) {
        run(PH_J, [&](int l) { ph_JE<EW>(a, c, t, env0, l); });
        if (step + 1 < a.n_steps) {
          run(PH_J, [&](int l) { ph_JB<EW>(a, c, t, env0, l); });
          run(PH_J, [&](int l) { ph_JS<EW>(c, t, l); });
        }
      }
    }
  }
  if (ROLL && a.tape != nullptr && (a.stages & COTIX_STAGE_COLLIDER) && a.n_steps > 0)
    run(PH_SAVE, [&](int l) { tape_save<EW, FNSET == FNS_ANALYTIC>(a, c, t, env0, l, a.n_steps - 1); });  // the last step's
  if (defer && a.n_steps > 0 && !rstore) run(PH_R, [&](int l) { ph_R<EW>(c, t, l); });  // the last step's
  run(PH_STORE, [&](int l) { ph_store<EW, ROLL, EVAL>(a, c, t, env0, l, rstore); });
}

// backward with the forward's tape (MODE 4): steps n_steps-1 .. 0, each
// restored from the saved state and the tape -- Euler (+ action), the world
// parts, the recorded resolutions (ph_D_tape) -- and reversed by phases E
// (recording the pre-resolution velocities), GE and G as in the re-play.
// No key split, narrowphase, RNG scan or choice runs: the tape holds their
// outcome, and every value the VJPs read is bit-identical to the re-play's
template <int EW, int FNSET, class R>
CX_DEV void run_wave_backward_tape(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, const R& run) {
  run(PH_ADJ, [&](int l) {
    ws_poly_init<EW>(c, t, l);
    ph_geo<EW>(a, c, t, env0, l);
    ph_adj_init<EW>(a, c, t, env0, l);
    stage_ret_w<EW>(a, c, t, l);
    for (int e = l; e < EW; e += WAVE) t.w(c.L.pcv, e) = 0u;  // phase T's pose entries
  });
  const bool col = (a.stages & COTIX_STAGE_COLLIDER) != 0;
  const bool edges = FNSET != FNS_ANALYTIC && c.sh.poly && ge_fits(c) && ge_edges_fit(c);
  constexpr bool TR = FNSET == FNS_ANALYTIC;  // the tape's resolution records (tape_rec)
  GradOut go;  // the previous (later) step's d ret / d action, stored by the restore phase
  const bool apf = act_prefetch<EW>(a, c);
  ActRegs ac;
  // the step after its restore: Euler, world parts, the tape's resolutions,
  // the reverse chain (the same for both restore forms)
  auto reverse_step = [&](int step, auto dphase) CXK_INLINE_LAMBDA {
    run(PH_A, [&](int l) {  // Euler (+ gravity, + action); no key split, no collider scratch
      if (a.stages & (COTIX_STAGE_EULER | COTIX_STAGE_GRAVITY))
        for (int w = l; w < c.nb * EW; w += WAVE) {
          const int e = w % EW, b = w / EW;
          if (env0 + e < a.B) euler_item<EW>(a, c, t, env0, e, b, step, apf, ac);
        }
    });
    if (col) {
      transform_phases<EW, FNSET>(a, c, t, env0, run);
      run(PH_D, dphase);
    }
    // phase E re-runs the sequential pass for its records -- unless the tape has them
    if (!(TR && col && tape_rec(c.sh))) run(PH_E, [&](int l) { ph_E<EW, true>(a, c, t, env0, l, c.L.sk0); });
    if (FNSET != FNS_ANALYTIC && col && ge_fits(c)) {
      if (edges)
        run(PH_GE, [&](int l) { ph_GE<EW, true>(a, c, t, env0, l); });
      else
        run(PH_GE, [&](int l) { ph_GE<EW>(a, c, t, env0, l); });
    }
    run(PH_G, [&](int l) { ph_G<EW, FNSET>(a, c, t, env0, l, step, &go); });
  };
  if (TR && rows_restore<EW>(a, c)) {  // rows, two steps ahead (two register sets: the loop unrolled by two)
    struct Pre {
      RowRegs rw;
      ActRegs an;
    };
    Pre p0, p1;
    const TapeRegs none{};
    auto prefetch = [&](int l, int s, Pre& p) CXK_INLINE_LAMBDA {
      restore_rows_fetch<EW>(a, c, env0, l, s, p.rw);
      if (apf) act_fetch<EW>(a, c, env0, l, s, p.an);
    };
    if (a.n_steps > 0)
      run(PH_RESTORE, [&](int l) {
        prefetch(l, a.n_steps - 1, p0);
        if (a.n_steps > 1) prefetch(l, a.n_steps - 2, p1);
      });
    auto one = [&](int step, Pre& cur) CXK_INLINE_LAMBDA {
      run(PH_RESTORE, [&](int l) {
        restore_rows_apply<EW>(c, t, l, cur.rw);
        ac = cur.an;
        if (a.grad_action != nullptr) grad_action_flush(a, env0, l, EW, go);  // (stores, then the prefetch reads)
        if (step > 1) prefetch(l, step - 2, cur);
      });
      reverse_step(step, [&](int l) { ph_D_tape<EW, TR, true>(a, c, t, env0, l, none); });
    };
    for (int step = a.n_steps - 1; step >= 0; step -= 2) {
      one(step, p0);
      if (step >= 1) one(step - 1, p1);
    }
    run(PH_ADJ, [&](int l) {
      if (a.grad_action != nullptr) grad_action_flush(a, env0, l, EW, go);  // step 0's
      ph_adj_store<EW>(a, c, t, env0, l);
    });
    return;
  }
  RestoreRegs rr;
  TapeRegs tn, tr;  // the next (earlier) step's tape words, the current step's
  ActRegs an;       // the actions, one step ahead as the state
  if (a.n_steps > 0)
    run(PH_RESTORE, [&](int l) {
      restore_fetch<EW>(a, c, env0, l, a.n_steps - 1, rr);
      if (col) tape_fetch<EW, TR>(a, c, env0, l, a.n_steps - 1, tn);
      if (apf) act_fetch<EW>(a, c, env0, l, a.n_steps - 1, an);
    });
  for (int step = a.n_steps - 1; step >= 0; --step) {
    run(PH_RESTORE, [&](int l) {
      restore_apply<EW>(c, t, l, rr);
      if (col) {
        tr = tn;
        if (edges) tape_edge_fetch<EW>(a, c, env0, l, step, tr);
      }
      ac = an;
      if (a.grad_action != nullptr) grad_action_flush(a, env0, l, EW, go);  // (stores, then the prefetch reads)
      if (step > 0) {  // the next (earlier) step, in flight
        restore_fetch<EW>(a, c, env0, l, step - 1, rr);
        if (col) tape_fetch<EW, TR>(a, c, env0, l, step - 1, tn);
        if (apf && !a.action_held) act_fetch<EW>(a, c, env0, l, step - 1, an);
      }
    });
    reverse_step(step, [&](int l) { ph_D_tape<EW, TR>(a, c, t, env0, l, tr); });
  }
  run(PH_ADJ, [&](int l) {
    if (a.grad_action != nullptr) grad_action_flush(a, env0, l, EW, go);  // step 0's
    ph_adj_store<EW>(a, c, t, env0, l);
  });
}

// ---------------------------------------------------------------------------
// The tape backward at two waves per env group (split backward).  MODE 4's
// step is an adjoint-independent part -- the restore of the saved state and
// tape rows, Euler, the world parts, phase D from the tape -- and the reverse
// chain G, which reads only the tile that part leaves and the adjoints.  G is
// a chain of dependent LDS reads and IEEE divisions on 4 of 64 lanes (VALU
// active ~27 % of the backward's wave cycles at one wave per SIMD), so here a
// producer wave runs the first part of step s into one tile of the group while
// its consumer wave runs G of step s + 1 on the other tile; the two share a
// SIMD (waves w and w + WPB of the workgroup) and G's latency overlaps the
// producer's phases instead of following them.  One workgroup barrier per step
// hands the filled tile to the consumer and the read one back to the
// producer; the consumer carries the adjoints in registers (g_chain).  Every
// phase is MODE 4's own code on the same tile words -- the same bits
// (tests/test_grad_cpu.py runs this program on the host emulation, producer
// then consumer per step, against run_wave_backward_tape).
// Scenes: analytic, the row restore (rows_restore), G in registers (5 or 7
// bodies: RoboCup, the box world); the launcher also needs the two tiles per
// group to fit the LDS (cotix_step.hip).
template <int EW>
CX_HD bool split_bwd_ok(const KArgs& a, const Ctx& c) {
#ifdef COTIX_NO_GREGS
  (void)a;
  (void)c;
  return false;
#else
  return rows_restore<EW>(a, c) && (c.nb == 5 || c.nb == 7) && c.sh.poly == 0;
#endif
}
// the producer's prefetch registers of one step (two sets: the loop is
// unrolled by two, as run_wave_backward_tape's)
struct SplitPre {
  RowRegs rw;
  ActRegs an;
};
template <int EW>
CX_DEV void split_prefetch(const KArgs& a, const Ctx& c, int env0, int l, int s, bool apf, SplitPre& p) {
  restore_rows_fetch<EW>(a, c, env0, l, s, p.rw);
  if (apf) act_fetch<EW>(a, c, env0, l, s, p.an);
}
// the producer's part of step `step` on tile t: restore, Euler, world parts, D
template <int EW, class R>
CX_DEV void split_produce(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, const R& run, int step, SplitPre& cur,
                          bool apf) {
  ActRegs ac;
  run(PH_RESTORE, [&](int l) {
    restore_rows_apply<EW>(c, t, l, cur.rw);
    ac = cur.an;
    if (step > 1) split_prefetch<EW>(a, c, env0, l, step - 2, apf, cur);
  });
  run(PH_A, [&](int l) {  // Euler (+ gravity, + action)
    if (a.stages & (COTIX_STAGE_EULER | COTIX_STAGE_GRAVITY))
      for (int w = l; w < c.nb * EW; w += WAVE) {
        const int e = w % EW, b = w / EW;
        if (env0 + e < a.B) euler_item<EW>(a, c, t, env0, e, b, step, apf, ac);
      }
  });
  transform_phases<EW, FNS_ANALYTIC>(a, c, t, env0, run);
  const TapeRegs none{};
  run(PH_D, [&](int l) { ph_D_tape<EW, true, true>(a, c, t, env0, l, none); });
}
// role: 1 producer, 2 consumer (the GPU's two waves of a group), 3 both in
// turn (the host emulation: a step's producer part, then the consumer's);
// bar(): the workgroup barrier (nothing on the host)
template <int EW, int NB, class R, class BAR>
CX_DEV void run_backward_split(const KArgs& a, const Ctx& c, Tile<EW> t0, Tile<EW> t1, int env0, const R& run,
                               int role, const BAR& bar) {
  const bool prod = (role & 1) != 0, cons = (role & 2) != 0, live = env0 < a.B;
  const int n = a.n_steps;
  const bool apf = act_prefetch<EW>(a, c);
  SplitPre p0, p1;
  float g[NB][6];
  if (prod && live)
    run(PH_ADJ, [&](int l) {
      for (int q = 0; q < 2; ++q) {
        const Tile<EW> t = q ? t1 : t0;
        ph_geo<EW>(a, c, t, env0, l);
        stage_ret_w<EW>(a, c, t, l);
        for (int e = l; e < EW; e += WAVE) t.w(c.L.pcv, e) = 0u;  // phase T's pose entries
      }
      if (n > 0) split_prefetch<EW>(a, c, env0, l, n - 1, apf, p0);
      if (n > 1) split_prefetch<EW>(a, c, env0, l, n - 2, apf, p1);
    });
  if (cons)  // d ret / d state_T (ph_adj_init's words)
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int k = 0; k < 6; ++k) g[b][k] = a.ret_w[6 * b + k];
  bar();
  // iteration k: the producer fills tile k & 1 with step n-1-k, the consumer
  // reverses step n-k on tile (k-1) & 1, which the producer filled at k-1
  auto iter = [&](int k, Tile<EW> tp, Tile<EW> tc, SplitPre& pre) CXK_INLINE_LAMBDA {
    if (prod && live && k < n) split_produce<EW>(a, c, tp, env0, run, n - 1 - k, pre, apf);
    if (cons && live && k >= 1)
      run(PH_G, [&](int l) CXK_INLINE_LAMBDA {
        if (l < EW && env0 + l < a.B) g_chain<EW, NB>(a, c, tc, env0, l, n - k, g);
      });
    if (k < n) bar();
  };
  for (int k = 0; k <= n; k += 2) {
    iter(k, t0, t1, p0);
    if (k + 1 <= n) iter(k + 1, t1, t0, p1);
  }
  if (cons && live)
    run(PH_ADJ, [&](int l) {
      if (l < EW)
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
          for (int k = 0; k < 6; ++k) t0.f(c.L.adj + 6 * b + k, l) = g[b][k];
      cxk::lockstep();
      ph_adj_store<EW>(a, c, t0, env0, l);
    });
}

// backward: steps n_steps-1 .. 0, each re-played from the saved state (so
// every discrete choice is the forward's) and then reversed by phase G
template <int EW, int FNSET, class R>
CX_DEV void run_wave_backward(const KArgs& a, const Ctx& c, Tile<EW> t, int env0, const R& run) {
  run(PH_ADJ, [&](int l) {
    ws_poly_init<EW>(c, t, l);
    ph_geo<EW>(a, c, t, env0, l);
    ph_adj_init<EW>(a, c, t, env0, l);
    stage_ret_w<EW>(a, c, t, l);
    for (int e = l; e < EW; e += WAVE) t.w(c.L.pcv, e) = 0u;  // phase T's pose entries
  });
  RestoreRegs rr;
  if (a.n_steps > 0) run(PH_RESTORE, [&](int l) { restore_fetch<EW>(a, c, env0, l, a.n_steps - 1, rr); });
  MConst mc;  // the fused scan's launch-constant owner words
  if ((a.stages & COTIX_STAGE_COLLIDER) && c.nl > 0 && scan_fused<EW>(c))
    run(PH_C1, [&](int l) { mc_fetch<EW>(c, t, l, mc); });
  for (int step = a.n_steps - 1; step >= 0; --step) {
    run(PH_RESTORE, [&](int l) {
      restore_apply<EW>(c, t, l, rr);
      if (step > 0) restore_fetch<EW>(a, c, env0, l, step - 1, rr);  // the next (earlier) step, in flight
    });
    run(PH_A, [&](int l) { ph_A<EW, false>(a, c, t, env0, l, step); });
    if (a.stages & COTIX_STAGE_COLLIDER) collider_phases<EW, FNSET, false>(a, c, t, env0, run, 0, c.L.sk0, mc);
    run(PH_E, [&](int l) { ph_E<EW, true>(a, c, t, env0, l, c.L.sk0); });
    if (FNSET != FNS_ANALYTIC && (a.stages & COTIX_STAGE_COLLIDER) && ge_fits(c))
      run(PH_GE, [&](int l) { ph_GE<EW>(a, c, t, env0, l); });
    run(PH_G, [&](int l) { ph_G<EW, FNSET>(a, c, t, env0, l, step); });
  }
  run(PH_ADJ, [&](int l) { ph_adj_store<EW>(a, c, t, env0, l); });
}

}  // namespace cxk
