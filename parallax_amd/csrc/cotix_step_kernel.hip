// cotix_step_kernel.hip -- the fused step kernel (gfx950) for ONE envs-per-wave
// tiling: compiled once per EW with -DCOTIX_EW=N (see cotix_launch.h); the
// phase programs live in cotix_kernel.h, design notes there and in DESIGN.md.
#include <hip/hip_runtime.h>

#include "../../include/cotix_amd.h"
#include "cotix_device.h"
#include "cotix_kernel.h"
#include "cotix_launch.h"

#ifndef COTIX_EW
#error "compile with -DCOTIX_EW=1|2|4|8"
#endif

using cxk::FNS_ANALYTIC;
using cxk::FNS_CIRCLE_POLY;
using cxk::FNS_CONVEX;
using cxk::SceneDev;

namespace {

// ---------------------------------------------------------------------------
// the fused step kernel: WPB independent waves per workgroup, EW envs per wave
// ---------------------------------------------------------------------------
using cxl::WPB;
#ifdef COTIX_PHASE_PROF
__device__ unsigned long long g_phase_cycles[cxk::PH_COUNT];
// per-wave timeline of the last launch (s_memrealtime, 100 MHz, chip-wide):
// entry, state loaded (before the workgroup barrier), after the barrier, end
// (after the stores completed) -- tools/k1_stamps.py
constexpr int STAMP_WAVES = 4096;
__device__ unsigned long long g_stamps[STAMP_WAVES * 4];
#define CXK_STAMP(v) const unsigned long long v = __builtin_amdgcn_s_memrealtime()
#else
#define CXK_STAMP(v) ((void)0)
#endif
// one phase on this lane, then wave-local ordering before the next phase.
// staged(ph, fetch, mid, finish): a phase of three stages whose per-lane
// state S passes from the first to the last in registers, every lane's
// stage before every lane's next (lockstep: nothing on the GPU, an order
// point of the host emulation's fibers); the emulation's HostRun is this
struct WaveRun {
  int lane;
  template <class S, class F1, class F2, class F3>
  __device__ __forceinline__ void staged(int ph, F1 fetch, F2 mid, F3 finish) const {
    (*this)(ph, [&](int l) {
      S s;
      fetch(l, s);
      cxk::lockstep();
      mid(l);
      cxk::lockstep();
      finish(l, s);
    });
  }
#ifdef COTIX_PHASE_PROF
  unsigned long long* acc;  // per-phase cycle accumulators (registers after inlining)
  template <class F>
  __device__ __forceinline__ void operator()(int ph, F f) const {
    const unsigned long long t0 = clock64();
    f(lane);
    cxk::wave_sync();
    acc[ph] += clock64() - t0;
  }
#elif defined(COTIX_ASM_MARKERS)  // tooling: phase markers in the ISA (tools/isa_phases.py)
  template <class F>
  __device__ __forceinline__ void operator()(int ph, F f) const {
    asm volatile(";#PHASE_BEGIN %0" ::"s"(ph));
    f(lane);
    cxk::wave_sync();
    asm volatile(";#PHASE_END %0" ::"s"(ph));
  }
#else
  // lockstep: the wave-uniform reads between phases precede the phase (a
  // no-op on the GPU, an order point of the host emulation's fibers)
  template <class F>
  __device__ __forceinline__ void operator()(int, F f) const {
    cxk::lockstep();
    f(lane);
    cxk::wave_sync();
  }
#endif
};
// MODE 0: step, 1: rollout forward (saves + return, + tape), 2: rollout
// backward re-playing the forward, 3: eval with the device judge / control
// (cotix_eval), 4: rollout backward from the forward's tape;
// SPEC: scene specialization (cxk::SPEC_*, compile-time dimensions)
template <int EW, int FNSET, int MODE, int SPEC = cxk::SPEC_GENERIC>
__global__ __launch_bounds__(WPB * 64) void step_kernel(cxk::KArgs a) {
  extern __shared__ uint32_t lds[];
  CXK_STAMP(st0);
  const SceneDev* sc = a.sc;
  const cxk::SceneHdr sh = cxk::spec_hdr<SPEC>(a.sh);  // a constant for SPEC > 0
  const int nhot = sh.nhot;
  // the scene tables into LDS: HC reads per thread issued before any store
  // (one global round trip per HC * 256 words, not one per 256)
  constexpr int HC = 16;
  // waves in this workgroup: WPB, or 2 / 1 for scenes whose tiles do not fit
  // four at a time (generic kernel only: the specializations are the
  // reference scenes, which fit, and keep their folded constants)
  const int nw = SPEC != cxk::SPEC_GENERIC ? WPB : (int)blockDim.x >> 6;
  const int nt = nw * 64;
  for (int base = 0; base < nhot; base += HC * nt) {
    uint32_t r[HC];
#pragma unroll
    for (int k = 0; k < HC; ++k) {
      const int i = base + k * nt + (int)threadIdx.x;
      r[k] = i < nhot ? sc->hot[i] : 0u;
    }
#pragma unroll
    for (int k = 0; k < HC; ++k) {
      const int i = base + k * nt + (int)threadIdx.x;
      if (i < nhot) lds[i] = r[k];
    }
  }
  const cxk::Ctx c = cxk::make_ctx<EW>(sh);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int env0 = (blockIdx.x * nw + wave) * EW;
  uint32_t* wbase = lds + nhot + wave * (c.L.S * EW + c.W.words);
  const cxk::Tile<EW> t{wbase, lds, wbase + c.L.S * EW};
  // the forward programs load the wave's state before the barrier: it writes
  // only the wave's own tile (disjoint from the tables), so its global reads
  // overlap the table copy's (a launch's fixed cost, K = 1 RL loops)
  if (MODE != 2 && MODE != 4 && env0 < a.B) {
    if (MODE == 3)
      cxk::ph_load_fwd<EW, false, true>(a, c, t, env0, lane);
    else
      cxk::ph_load_fwd<EW, MODE == 1>(a, c, t, env0, lane);
  }
#ifdef COTIX_PHASE_PROF
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#endif
  CXK_STAMP(st1);
  __syncthreads();
  CXK_STAMP(st2);
  if (env0 >= a.B) return;  // whole wave idle (after the only workgroup barrier)
#ifdef COTIX_PHASE_PROF
  unsigned long long acc[cxk::PH_COUNT];
  for (int q = 0; q < cxk::PH_COUNT; ++q) acc[q] = 0ull;
  const WaveRun run{lane, acc};
#else
  const WaveRun run{lane};
#endif
  if (MODE == 4)
    cxk::run_wave_backward_tape<EW, FNSET>(a, c, t, env0, run);
  else if (MODE == 2)
    cxk::run_wave_backward<EW, FNSET>(a, c, t, env0, run);
  else if (MODE == 3)
    cxk::run_wave<EW, FNSET, false, true>(a, c, t, env0, run, true);
  else
    cxk::run_wave<EW, FNSET, MODE == 1, false,
                  MODE == 0 && (SPEC == cxk::SPEC_ROBOCUP || SPEC == cxk::SPEC_ROBOCUP_PART)>(a, c, t, env0, run, true);
#ifdef COTIX_PHASE_PROF
  if (lane == 0)
    for (int q = 0; q < cxk::PH_COUNT; ++q) atomicAdd(&g_phase_cycles[q], acc[q]);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  CXK_STAMP(st3);
  const int gw = (int)blockIdx.x * nw + wave;
  if (lane == 0 && gw < STAMP_WAVES) {
    g_stamps[4 * gw] = st0;
    g_stamps[4 * gw + 1] = st1;
    g_stamps[4 * gw + 2] = st2;
    g_stamps[4 * gw + 3] = st3;
  }
#endif
}

#if COTIX_EW == 4
// the tape backward at two waves per env group (cxk::run_backward_split):
// waves g and g + WPB of the workgroup are env group g's producer and
// consumer (one SIMD each pair), the group's two tiles are the LDS regions of
// those two waves.  The workgroup barrier waits for LDS only: the producer's
// prefetch reads (two steps ahead) and the consumer's gradient stores stay in
// flight across it.
CX_DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
template <int NB, int SPEC>
__global__ __launch_bounds__(2 * WPB * 64) void bwd_split_kernel(cxk::KArgs a) {
  constexpr int EW = 4;
  extern __shared__ uint32_t lds[];
  const SceneDev* sc = a.sc;
  const cxk::SceneHdr sh = cxk::spec_hdr<SPEC>(a.sh);
  const int nhot = sh.nhot;
  constexpr int HC = 8, NT = 2 * WPB * 64;
  for (int base = 0; base < nhot; base += HC * NT) {
    uint32_t r[HC];
#pragma unroll
    for (int k = 0; k < HC; ++k) {
      const int i = base + k * NT + (int)threadIdx.x;
      r[k] = i < nhot ? sc->hot[i] : 0u;
    }
#pragma unroll
    for (int k = 0; k < HC; ++k) {
      const int i = base + k * NT + (int)threadIdx.x;
      if (i < nhot) lds[i] = r[k];
    }
  }
  const cxk::Ctx c = cxk::make_ctx<EW>(sh);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int grp = wave % WPB, role = wave < WPB ? 1 : 2;
  const int env0 = (blockIdx.x * WPB + grp) * EW;
  const int rw = c.L.S * EW + c.W.words;  // one wave's region: tile + scratch
  uint32_t* r0 = lds + nhot + grp * rw;
  uint32_t* r1 = lds + nhot + (grp + WPB) * rw;
  uint32_t* ws = (role == 1 ? r0 : r1) + c.L.S * EW;
  const cxk::Tile<EW> t0{r0, lds, ws}, t1{r1, lds, ws};
  __syncthreads();
#ifdef COTIX_PHASE_PROF
  unsigned long long acc[cxk::PH_COUNT];
  for (int q = 0; q < cxk::PH_COUNT; ++q) acc[q] = 0ull;
  const WaveRun run{lane, acc};
#else
  const WaveRun run{lane};
#endif
  cxk::run_backward_split<EW, NB>(a, c, t0, t1, env0, run, role, [] { lds_barrier(); });
#ifdef COTIX_PHASE_PROF
  if (lane == 0 && env0 < a.B)
    for (int q = 0; q < cxk::PH_COUNT; ++q) atomicAdd(&g_phase_cycles[q], acc[q]);
#endif
}
// the step program with a key-window helper wave per env group
// (cxk::KeyHelper): waves g < WPB step env group g, wave g + WPB computes its
// key windows; LDS: the tables, WPB wave regions (tile + scratch, stride rounded
// to a multiple of EW words), then WPB helper window buffers
struct GpuKeyHelp {
  static constexpr bool on = true;
  int kwalt;
  __device__ __forceinline__ void bar() const { lds_barrier(); }
};
template <int FNSET, int SPEC, bool SDEFER>
__global__ __launch_bounds__(2 * WPB * 64) void step_help_kernel(cxk::KArgs a) {
  constexpr int EW = 4;
  extern __shared__ uint32_t lds[];
  const SceneDev* sc = a.sc;
  const cxk::SceneHdr sh = cxk::spec_hdr<SPEC>(a.sh);
  const int nhot = sh.nhot;
  constexpr int HC = 8, NT = 2 * WPB * 64;
  for (int base = 0; base < nhot; base += HC * NT) {
    uint32_t r[HC];
#pragma unroll
    for (int k = 0; k < HC; ++k) {
      const int i = base + k * NT + (int)threadIdx.x;
      r[k] = i < nhot ? sc->hot[i] : 0u;
    }
#pragma unroll
    for (int k = 0; k < HC; ++k) {
      const int i = base + k * NT + (int)threadIdx.x;
      if (i < nhot) lds[i] = r[k];
    }
  }
  const cxk::Ctx c = cxk::make_ctx<EW>(sh);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int grp = wave % WPB;
  const bool stepper = wave < WPB;
  const int env0 = (blockIdx.x * WPB + grp) * EW;
  const int rw = cxk::help_region_words<EW>(c), hw = cxk::KWIN * c.L.kww * EW;
  uint32_t* um = lds + nhot + grp * rw;
  uint32_t* hb = lds + nhot + WPB * rw + grp * hw;
  const cxk::Tile<EW> tm{um, lds, um + c.L.S * EW};
  if (stepper && env0 < a.B) cxk::ph_load_fwd<EW, false>(a, c, tm, env0, lane);
  __syncthreads();
  const WaveRun run{lane};
  const int nbar = cxk::keys_on(a) ? cxk::key_helper_windows(a) : 0;
  if (env0 >= a.B) {  // an idle wave keeps the barrier count
    for (int q = 0; q < nbar; ++q) lds_barrier();
    return;
  }
  if (stepper) {
    const GpuKeyHelp help{(int)(hb - um) / EW - c.L.kw};
    cxk::run_wave<EW, FNSET, false, false, SDEFER>(a, c, tm, env0, run, true, help);
  } else {
    cxk::KeyHelper<EW> h;
    h.tm = tm;
    h.th = cxk::Tile<EW>{hb - c.L.kw * EW, lds, nullptr};
    h.env0 = env0;
    if (nbar > 0) cxk::key_helper_init<EW>(a, c, h, run);
    for (int q = 0; q < nbar; ++q) {
      cxk::key_helper_next<EW>(a, c, h, run);
      lds_barrier();
    }
  }
}
#endif

}  // namespace

#if COTIX_EW == 4
// 0: launched; 1: not compiled for this scene / launch (the caller launches step_kernel)
int cxl::launch_step_help(const cxk::KArgs& ka, int spec, size_t lds, hipStream_t st) {
  const dim3 grid((ka.B + WPB * 4 - 1) / (WPB * 4)), block(2 * WPB * 64);
  if (spec == cxk::SPEC_ROBOCUP)
    hipLaunchKernelGGL((step_help_kernel<FNS_ANALYTIC, cxk::SPEC_ROBOCUP, true>), grid, block, lds, st, ka);
  else
    return 1;
  return 0;
}
// 0: launched; 1: not this scene / launch (the caller runs MODE 4)
int cxl::launch_bwd_split(const cxk::KArgs& ka, int spec, size_t lds, hipStream_t st) {
  const dim3 grid((ka.B + WPB * 4 - 1) / (WPB * 4)), block(2 * WPB * 64);
  const int nb = ka.sh.nb;
#define COTIX_LAUNCH_SPLIT(NB, SP) hipLaunchKernelGGL((bwd_split_kernel<NB, SP>), grid, block, lds, st, ka)
  // the specializations only: with the header's dimensions as run-time
  // values the two roles' registers exceed 256 VGPRs and spill (the generic
  // scenes keep MODE 4)
  if (spec == cxk::SPEC_ROBOCUP && nb == 5)
    COTIX_LAUNCH_SPLIT(5, cxk::SPEC_ROBOCUP);
  // (the box world's split form is compiled and emulation-tested but not
  // launched: measured slower than its one-wave MODE 4, 0.55 against 0.42 ms
  // per 64-step backward)
  else
    return 1;
#undef COTIX_LAUNCH_SPLIT
  return 0;
}
#endif

#define CXL_NAME2(n) launch_step_ew##n
#define CXL_NAME(n) CXL_NAME2(n)
hipError_t cxl::CXL_NAME(COTIX_EW)(const cxk::KArgs& ka, int fs, int mode, size_t lds, hipStream_t st, int spec,
                                   int wpb) {
  constexpr int EW = COTIX_EW;
  if ((wpb != 1 && wpb != 2 && wpb != WPB) || (wpb != WPB && spec != cxk::SPEC_GENERIC)) return hipErrorInvalidValue;
  const dim3 grid((ka.B + wpb * EW - 1) / (wpb * EW)), block(wpb * 64);
#define COTIX_LAUNCH(FS, BW) hipLaunchKernelGGL((step_kernel<EW, FS, BW>), grid, block, lds, st, ka)
#define COTIX_LAUNCH_SPEC(FS, BW, SP) hipLaunchKernelGGL((step_kernel<EW, FS, BW, SP>), grid, block, lds, st, ka)
  constexpr int F_AN = FNS_ANALYTIC, F_PP = FNS_ANALYTIC | FNS_CONVEX, F_AP = F_PP | cxk::FNS_AABB_POLY,
                F_ALL = F_AP | FNS_CIRCLE_POLY;
  const int F = cxk::launch_fnset(fs, mode);  // the contact-function program for this scene
#if COTIX_EW == 4 || COTIX_EW == 2
  // the reference-scene specializations: every program of RoboCup at the
  // default tiling, the step programs (mode 0) at 4 and 2 envs per wave
  // (the re-play backward, mode 2, is the tape backward's check: generic only)
  if (spec == cxk::SPEC_ROBOCUP && F == F_AN && mode != 2 && (mode == 0 || COTIX_EW == 4)) {
    if (mode == 3)
      COTIX_LAUNCH_SPEC(F_AN, 3, cxk::SPEC_ROBOCUP);
    else if (mode == 4)
      COTIX_LAUNCH_SPEC(F_AN, 4, cxk::SPEC_ROBOCUP);
    else if (mode == 1)
      COTIX_LAUNCH_SPEC(F_AN, 1, cxk::SPEC_ROBOCUP);
    else
      COTIX_LAUNCH_SPEC(F_AN, 0, cxk::SPEC_ROBOCUP);
    return hipGetLastError();
  }
  if (spec == cxk::SPEC_LUNAR && mode == 0 && F == F_PP) {
    COTIX_LAUNCH_SPEC(F_PP, 0, cxk::SPEC_LUNAR);
    return hipGetLastError();
  }
#if COTIX_EW == 4
  // the box world's structure: the step and rollout programs (finite_scene, grad_box)
  if (spec == cxk::SPEC_BOX && F == F_AN && (mode <= 1 || mode == 4)) {
    if (mode == 4)
      COTIX_LAUNCH_SPEC(F_AN, 4, cxk::SPEC_BOX);
    else if (mode == 1)
      COTIX_LAUNCH_SPEC(F_AN, 1, cxk::SPEC_BOX);
    else
      COTIX_LAUNCH_SPEC(F_AN, 0, cxk::SPEC_BOX);
    return hipGetLastError();
  }
#endif
  // the partitionable layout's specializations: the step program only
  if (spec == cxk::SPEC_ROBOCUP_PART && mode == 0 && F == F_AN) {
    COTIX_LAUNCH_SPEC(F_AN, 0, cxk::SPEC_ROBOCUP_PART);
    return hipGetLastError();
  }
  if (spec == cxk::SPEC_LUNAR_PART && mode == 0 && F == F_PP) {
    COTIX_LAUNCH_SPEC(F_PP, 0, cxk::SPEC_LUNAR_PART);
    return hipGetLastError();
  }
#else
  (void)spec;
#endif
#undef COTIX_LAUNCH_SPEC
  if (mode == 2) {
    if (F == F_AN)
      COTIX_LAUNCH(F_AN, 2);
    else
      COTIX_LAUNCH(F_ALL, 2);  // polygon scenes (the host rejects circle x polygon contacts)
  } else if (mode == 4) {
    if (F == F_AN)
      COTIX_LAUNCH(F_AN, 4);
    else
      COTIX_LAUNCH(F_ALL, 4);
  } else if (mode == 3) {
    if (F == F_AN)
      COTIX_LAUNCH(F_AN, 3);
    else
      COTIX_LAUNCH(F_ALL, 3);
  } else if (mode == 1) {
    if (F == F_AN)
      COTIX_LAUNCH(F_AN, 1);
    else
      COTIX_LAUNCH(F_ALL, 1);
  } else if (F == F_AN) {
    COTIX_LAUNCH(F_AN, 0);
  } else if (F == F_PP) {
    COTIX_LAUNCH(F_PP, 0);
  } else if (F == F_AP) {
    COTIX_LAUNCH(F_AP, 0);
  } else {
    COTIX_LAUNCH(F_ALL, 0);
  }
#undef COTIX_LAUNCH
  return hipGetLastError();
}

#ifdef COTIX_PHASE_PROF
// profiling build only: per-phase cycles summed over waves since the last call (then reset)
extern "C" int cotix_phase_cycles(unsigned long long* out, int n) {
  unsigned long long h[cxk::PH_COUNT] = {};
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_phase_cycles), sizeof(h)) != hipSuccess) return -1;
  unsigned long long z[cxk::PH_COUNT] = {};
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_phase_cycles), z, sizeof(z)) != hipSuccess) return -1;
  for (int q = 0; q < n && q < cxk::PH_COUNT; ++q) out[q] = h[q];
  // then the 8 sub-phase timers (CXK_SUB_T1)
  unsigned long long sub[8] = {};
  if (hipMemcpyFromSymbol(sub, HIP_SYMBOL(cxk::g_sub_cycles), sizeof(sub)) != hipSuccess) return -1;
  unsigned long long z8[8] = {};
  if (hipMemcpyToSymbol(HIP_SYMBOL(cxk::g_sub_cycles), z8, sizeof(z8)) != hipSuccess) return -1;
  unsigned long long dsub[4] = {};  // GJK timer of cotix_device.h in slot 4
  if (hipMemcpyFromSymbol(dsub, HIP_SYMBOL(cx::g_dev_sub), sizeof(dsub)) != hipSuccess) return -1;
  if (hipMemcpyToSymbol(HIP_SYMBOL(cx::g_dev_sub), z8, sizeof(dsub)) != hipSuccess) return -1;
  sub[4] = dsub[0];  // GJK
  sub[5] = dsub[1];  // EPA
  for (int q = 0; q < 8 && cxk::PH_COUNT + q < n; ++q) out[cxk::PH_COUNT + q] = sub[q];
  return cxk::PH_COUNT + 8 < n ? cxk::PH_COUNT + 8 : n;
}
// profiling build only: the last launch's per-wave timeline (g_stamps), n words
extern "C" int cotix_phase_stamps(unsigned long long* out, int n) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  const int m = n < STAMP_WAVES * 4 ? n : STAMP_WAVES * 4;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * m) != hipSuccess) return -1;
  return m;
}
#endif
