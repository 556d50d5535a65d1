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

// one wave at a time (waves are independent); within a wave every phase
// runs for all 64 lanes before the next (what wave_sync() guarantees)
template <int EW>
void run_blocks(const cxk::KArgs& a) {
  const cxk::SceneDev& sc = *a.sc;
  const cxk::Ctx c{sc.nb, sc.np, sc.nc, sc.nl, sc.nt, &sc, cxk::layout(sc.nb, sc.W, sc.nc, sc.nt)};
  const int nwaves = (a.B + EW - 1) / EW;
  std::vector<uint32_t> lds((size_t)sc.nhot + (size_t)c.L.S * EW);
  for (int q = 0; q < sc.nhot; ++q) lds[q] = sc.hot[q];
  const int W = cxk::WAVE;
  for (int wv = 0; wv < nwaves; ++wv) {
    std::fill(lds.begin() + sc.nhot, lds.end(), 0x7FBADBADu);  // poison (a NaN pattern)
    const cxk::Tile<EW> t{lds.data() + sc.nhot, lds.data()};
    const int env0 = wv * EW;
    for (int l = 0; l < W; ++l) cxk::ph_load<EW>(a, c, t, env0, l);
    for (int step = 0; step < a.n_steps; ++step) {
      for (int l = 0; l < W; ++l) cxk::ph_A<EW>(a, c, t, env0, l, step);
      if (a.stages & COTIX_STAGE_COLLIDER) {
        for (int l = 0; l < W; ++l) cxk::ph_T<EW, 7>(a, c, t, env0, l);
        for (int l = 0; l < W; ++l) cxk::ph_B<EW, 7>(a, c, t, env0, l);
        for (int l = 0; l < W; ++l) cxk::ph_C<EW>(a, c, t, env0, l);
        for (int l = 0; l < W; ++l) cxk::ph_D<EW>(a, c, t, env0, l);
      }
      for (int l = 0; l < W; ++l) cxk::ph_E<EW>(a, c, t, env0, l);
    }
    for (int l = 0; l < W; ++l) cxk::ph_store<EW>(a, c, t, env0, l);
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
  if (E == 1) run_blocks<1>(a);
  else if (E == 4) run_blocks<4>(a);
  else if (E == 8) run_blocks<8>(a);
  else run_blocks<2>(a);
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
