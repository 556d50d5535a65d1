// TEST INFRASTRUCTURE ONLY -- the host emulation's SIMT runtime: the 64 lanes
// of a wave run the kernel's own wave program (cxk::run_wave, the GPU's code
// path, cross-lane operations included) as 64 fibers on one thread.  A lane
// runs until it reaches a collective point -- a phase barrier (wave_sync), an
// order point inside a phase (lockstep), a ballot, a lane permute or a pair
// exchange -- and waits there; the scheduler resolves a collective once every
// lane it involves waits at it, then resumes them.  Between collective points
// lanes run one after another in lane order (the GPU runs them in lockstep;
// the kernel orders every cross-lane LDS dependency by a collective point).
//
// Resolution rules (cxk_simt:: primitives, cotix_kernel.h):
//  * pair operations (pair_swap: quad_perm(1,0,3,2)) resolve per lane pair,
//    as soon as both lanes wait at one -- their n-th each (the two lanes of
//    a pair run their exchanges in lockstep; a count mismatch aborts);
//  * wave operations (sync, lockstep, ballot, bpermute) are convergent: they
//    resolve when every live lane waits at its n-th wave operation, the same
//    operation on every lane (anything else aborts as a divergent collective
//    -- the kernel calls them with the whole wave).
// Call sites are not an identity (the compiler may duplicate a call into
// branches); the per-lane operation counts are.  A lane that leaves the
// program takes no further part.

// Fibers switch by a few instructions of x86-64 assembly (callee-saved
// registers and the stack pointer), with AddressSanitizer's fiber
// annotations in the sanitizer builds.
#pragma once
#include <sys/mman.h>

#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>

#if defined(__SANITIZE_ADDRESS__)
extern "C" void __sanitizer_start_switch_fiber(void** fake_stack_save, const void* bottom, size_t size);
extern "C" void __sanitizer_finish_switch_fiber(void* fake_stack_save, const void** bottom_old, size_t* size_old);
#define CXS_ASAN 1
#else
#define CXS_ASAN 0
#endif

// cxs_switch(save, load): store this context's stack pointer at *save, resume
// the context whose stack pointer is `load`
extern "C" void cxs_switch(void** save, void* load);
asm(R"(
  .text
  .globl cxs_switch
  .type cxs_switch, @function
cxs_switch:
  pushq %rbp
  pushq %rbx
  pushq %r12
  pushq %r13
  pushq %r14
  pushq %r15
  movq %rsp, (%rdi)
  movq %rsi, %rsp
  popq %r15
  popq %r14
  popq %r13
  popq %r12
  popq %rbx
  popq %rbp
  ret
  .size cxs_switch, .-cxs_switch
  .section .note.GNU-stack,"",@progbits
  .text
)");

namespace cxk_simt {

constexpr int NL = 64;
#if CXS_ASAN
constexpr size_t STACK = 4u << 20;
#else
constexpr size_t STACK = 1u << 20;
#endif

enum Op : int { OP_NONE = 0, OP_SYNC, OP_LOCKSTEP, OP_BALLOT, OP_BPERMUTE, OP_PAIR_SWAP };
enum State : int { RUN = 0, WAIT, DONE };

struct Fiber {
  void* sp = nullptr;
  char* stack = nullptr;
  int state = DONE;
  int op = OP_NONE;
  const void* site = nullptr;
  uint64_t in = 0, out = 0;
  uint64_t npair = 0, nwave = 0;  // pair / wave operations resolved so far
#if CXS_ASAN
  void* fake = nullptr;
#endif
};

struct Wave {
  Fiber f[NL];
  void* sched_sp = nullptr;
  int cur = -1;
  const std::function<void(int)>* body = nullptr;
#if CXS_ASAN
  const void* sched_bottom = nullptr;
  size_t sched_size = 0;
#endif
};

// static, not inline: an inline variable is a GNU_UNIQUE symbol, bound once per
// process across every emulation build a test loads (plain, ASan with 4 MiB
// stacks, mutation builds) -- one build's stride over another's mapping.
static thread_local Wave* g_wave = nullptr;
static thread_local char* g_stacks = nullptr;  // NL stacks, mapped once per thread (never unmapped)

[[noreturn]] inline void fail(const char* what, int lane) {
  std::fprintf(stderr, "cotix_simt: %s (lane %d)\n", what, lane);
  std::abort();
}

// the running fiber hands control back to the scheduler
inline void to_sched(Fiber& f, bool dying) {
  Wave& w = *g_wave;
#if CXS_ASAN
  __sanitizer_start_switch_fiber(dying ? nullptr : &f.fake, w.sched_bottom, w.sched_size);
#else
  (void)dying;
#endif
  cxs_switch(&f.sp, w.sched_sp);
#if CXS_ASAN
  __sanitizer_finish_switch_fiber(f.fake, nullptr, nullptr);
#endif
}

inline void entry() {
  Wave& w = *g_wave;
  const int lane = w.cur;
#if CXS_ASAN
  __sanitizer_finish_switch_fiber(nullptr, &w.sched_bottom, &w.sched_size);
#endif
  (*w.body)(lane);
  w.f[lane].state = DONE;
  to_sched(w.f[lane], true);
  fail("resumed after leaving the program", lane);
}

// one collective point of the running lane: wait, then the resolved value
inline uint64_t wait(int op, const void* site, uint64_t in) {
  Wave* w = g_wave;
  if (w == nullptr || w->cur < 0) {  // outside a wave program (single-lane entry points)
    if (op == OP_SYNC || op == OP_LOCKSTEP) return 0;
    fail("cross-lane operation outside a wave program", -1);
  }
  Fiber& f = w->f[w->cur];
  f.state = WAIT;
  f.op = op;
  f.site = site;
  f.in = in;
  to_sched(f, false);
  return f.out;
}

inline void resume(Wave& w, int l) {
  Fiber& f = w.f[l];
  w.cur = l;
#if CXS_ASAN
  void* fake = nullptr;
  __sanitizer_start_switch_fiber(&fake, f.stack, STACK);
#endif
  cxs_switch(&w.sched_sp, f.sp);
#if CXS_ASAN
  __sanitizer_finish_switch_fiber(fake, nullptr, nullptr);
#endif
  w.cur = -1;
}

// run body(lane) for the 64 lanes of one wave as SIMT fibers
inline void run(const std::function<void(int)>& body) {
  if (g_wave != nullptr) fail("nested wave program", -1);
  if (g_stacks == nullptr) {
    void* p = mmap(nullptr, STACK * NL, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (p == MAP_FAILED) fail("fiber stacks: mmap failed", -1);
    g_stacks = static_cast<char*>(p);
  }
  Wave w;
  w.body = &body;
  for (int l = 0; l < NL; ++l) {
    Fiber& f = w.f[l];
    f.stack = g_stacks + STACK * l;
    // initial frame: six callee-saved registers (zero), then cxs_switch's
    // return into entry() with the stack aligned as after a call
    uintptr_t top = (reinterpret_cast<uintptr_t>(f.stack) + STACK) & ~uintptr_t(15);
    uint64_t* sp = reinterpret_cast<uint64_t*>(top);
    *--sp = 0;                                     // entry()'s return address (never used)
    *--sp = reinterpret_cast<uint64_t>(&entry);  // cxs_switch's ret target
    for (int r = 0; r < 6; ++r) *--sp = 0;
    f.sp = sp;
    f.state = RUN;
  }
  g_wave = &w;
  for (;;) {
    for (int l = 0; l < NL; ++l)
      if (w.f[l].state == RUN) resume(w, l);
    // every lane waits or has left: resolve pair operations first
    bool resolved = false;
    for (int l = 0; l < NL; l += 2) {
      Fiber &a = w.f[l], &b = w.f[l + 1];
      const bool pa = a.state == WAIT && a.op == OP_PAIR_SWAP, pb = b.state == WAIT && b.op == OP_PAIR_SWAP;
      if (pa && pb) {
        if (a.npair != b.npair) fail("pair exchange out of step (the lanes' exchange counts differ)", l);
        ++a.npair;
        ++b.npair;
        a.out = b.in;
        b.out = a.in;
        a.state = b.state = RUN;
        resolved = true;
      }
    }
    if (resolved) continue;
    // then one wave operation, with every live lane
    int lead = -1;
    uint64_t act = 0, bal = 0;
    for (int l = 0; l < NL; ++l) {
      const Fiber& f = w.f[l];
      if (f.state == DONE) continue;
      if (f.op == OP_PAIR_SWAP) fail("pair exchange whose partner waits elsewhere or has left", l);
      if (lead < 0) lead = l;
      const Fiber& g = w.f[lead];
      if (f.op != g.op || f.nwave != g.nwave) {
        std::fprintf(stderr, "cotix_simt: lane %d op %d #%llu at %p, lane %d op %d #%llu at %p\n", lead, g.op,
                     (unsigned long long)g.nwave, g.site, l, f.op, (unsigned long long)f.nwave, f.site);
        fail("divergent wave operation", l);
      }
      act |= 1ull << l;
      if (f.in != 0) bal |= 1ull << l;
    }
    if (lead < 0) break;  // every lane has left
    const int op = w.f[lead].op;
    for (int l = 0; l < NL; ++l) {
      if (!((act >> l) & 1ull)) continue;
      Fiber& f = w.f[l];
      if (op == OP_BALLOT) {
        f.out = bal;
      } else if (op == OP_BPERMUTE) {
        const int src = (int)(f.in >> 32) & (NL - 1);
        f.out = ((act >> src) & 1ull) ? (w.f[src].in & 0xFFFFFFFFull) : 0ull;
      } else {
        f.out = 0;
      }
      ++f.nwave;
      f.state = RUN;
    }
  }
  g_wave = nullptr;
}

// the collective points (declared in cotix_kernel.h; the call site keys the
// resolution, so they are never inlined)
__attribute__((noinline)) void sync() { wait(OP_SYNC, __builtin_return_address(0), 0); }
__attribute__((noinline)) void lockstep() { wait(OP_LOCKSTEP, __builtin_return_address(0), 0); }
__attribute__((noinline)) uint64_t ballot(bool p) { return wait(OP_BALLOT, __builtin_return_address(0), p ? 1 : 0); }
__attribute__((noinline)) uint32_t bpermute(int src, uint32_t v) {
  return (uint32_t)wait(OP_BPERMUTE, __builtin_return_address(0), ((uint64_t)(uint32_t)src << 32) | v);
}
__attribute__((noinline)) uint32_t pair_swap(uint32_t v) {
  return (uint32_t)wait(OP_PAIR_SWAP, __builtin_return_address(0), v);
}

}  // namespace cxk_simt
