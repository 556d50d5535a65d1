// TEST INFRASTRUCTURE ONLY -- host emulation of the fused HIP step kernel.
//
// Compiles parallax_amd/csrc/cotix_kernel.h (the kernel's phase functions)
// for the host and runs every phase for all BLK lanes of every workgroup in
// turn, which is what the __syncthreads() between phases guarantees on the
// GPU.  Used to (a) check the kernel logic against the oracle on CPU and
// (b) run it under AddressSanitizer/UBSan (GPU sanitizers are unavailable).
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../parallax_amd/csrc/cotix_kernel.h"
#include "../../parallax_amd/csrc/cotix_scene.h"

namespace {
std::string g_err;
struct EmuScene {
  cxk::SceneDev s;
  int n_cand = 0, fnset = 0;
};

template <int E>
void run_blocks(const cxk::KArgs& a) {
  const cxk::SceneDev& sc = *a.sc;
  const cxk::Lay L = cxk::layout(sc);
  const int nblk = (a.B + E - 1) / E;
  std::vector<uint32_t> lds((size_t)cxk::lds_words(sc) * E);
  const int BLK = cxk::BLK;
  for (int b = 0; b < nblk; ++b) {
    std::fill(lds.begin(), lds.end(), 0x7FBADBADu);  // poison (a NaN pattern)
    const cxk::Tile<E> t{lds.data()};
    const int env0 = b * E;
    for (int tid = 0; tid < BLK; ++tid) cxk::ph_load<E>(a, sc, L, t, env0, tid);
    for (int step = 0; step < a.n_steps; ++step) {
      for (int tid = 0; tid < BLK; ++tid) cxk::ph_A<E>(a, sc, L, t, env0, tid, step);
      if (a.stages & COTIX_STAGE_COLLIDER) {
        for (int tid = 0; tid < BLK; ++tid) cxk::ph_T<E>(a, sc, L, t, env0, tid);
        for (int tid = 0; tid < BLK; ++tid) cxk::ph_B<E, 7>(a, sc, L, t, env0, tid);
        for (int tid = 0; tid < BLK; ++tid) cxk::ph_C<E>(a, sc, L, t, env0, tid);
        for (int tid = 0; tid < BLK; ++tid) cxk::ph_D<E>(a, sc, L, t, env0, tid);
      }
      for (int tid = 0; tid < BLK; ++tid) cxk::ph_E<E>(a, sc, L, t, env0, tid);
    }
    for (int tid = 0; tid < BLK; ++tid) cxk::ph_store<E>(a, sc, L, t, env0, tid);
  }
}
}  // namespace

extern "C" {
const char* emu_last_error(void) { return g_err.c_str(); }

int emu_scene_create(int n_bodies, const float* body_params, int n_parts, const int* part_body, const int* part_type,
                     const int* part_nverts, void** out) {
  EmuScene* s = new EmuScene();
  if (cxk::compile_scene(n_bodies, body_params, n_parts, part_body, part_type, part_nverts, s->s, s->n_cand,
                         s->fnset, g_err)) {
    delete s;
    return -1;
  }
  *out = s;
  return 0;
}

int emu_scene_destroy(void* s) {
  delete static_cast<EmuScene*>(s);
  return 0;
}

int emu_step(void* scene, float* dyn, uint32_t* keys, uint32_t* err, const float* geom, int gstride, int B,
             int n_steps, float dt, int stages, const float* action, int action_body, const float* dyn_reset,
             uint32_t* resets, int E) {
  EmuScene* s = static_cast<EmuScene*>(scene);
  cxk::KArgs a{&s->s, dyn, keys, err, geom, gstride, B, n_steps, dt, stages, action, action_body, dyn_reset, resets, 0};
  if (E == 8) run_blocks<8>(a);
  else if (E == 32) run_blocks<32>(a);
  else run_blocks<16>(a);
  return 0;
}

int emu_contacts(int fn, int n, const float* a, const float* b, float* out, uint32_t* err) {
  const cx::v2 d0{-0.05243401f, 0.9986244f};
  uint32_t bx = 0xbd56c50bu, by = 0x3f7fa5d9u;
  cx::v2 dd;
  std::memcpy(&dd.x, &bx, 4);
  std::memcpy(&dd.y, &by, 4);
  (void)d0;
  for (int i = 0; i < n; ++i) {
    cx::Shape A, Bs;
    A.kind = (int)a[18 * i];
    A.n = (int)a[18 * i + 1];
    Bs.kind = (int)b[18 * i];
    Bs.n = (int)b[18 * i + 1];
    for (int k = 0; k < 16; ++k) {
      A.d[k] = a[18 * i + 2 + k];
      Bs.d[k] = b[18 * i + 2 + k];
    }
    uint32_t er = 0;
    cx::Contact c = cx::run_contact(fn, A, Bs, dd, &er);
    out[4 * i] = c.pen.x;
    out[4 * i + 1] = c.pen.y;
    out[4 * i + 2] = c.cp.x;
    out[4 * i + 3] = c.cp.y;
    if (err) err[i] = er;
  }
  return 0;
}
}
