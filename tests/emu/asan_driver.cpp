// TEST INFRASTRUCTURE ONLY -- standalone AddressSanitizer/UBSan driver of the
// kernel's host emulation (GPU sanitizers are unavailable on this pool).
// usage: asan_driver IN OUT.  IN (little-endian): int32 header
//   nb np B T stages G gstride mode E action_body
// then f32 body_params[nb*4], int32 part_body[np], part_type[np],
// part_nverts[np], f32 geom[gstride ? B*gstride : G], f32 dyn[nb*6*B],
// u32 keys[B*2]; mode 1 adds f32 actions[T*B*2], f32 ret_w[nb*6].
// OUT: mode 0: dyn, keys, err; mode 1: dyn, keys, err, ret, grad_action, grad_dyn0
// (the backward from the forward's tape; the re-play backward must give the
// same bits, else exit 6).
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

extern "C" {
int emu_scene_create(int, const float*, int, const int*, const int*, const int*, void**);
int emu_step(void*, float*, uint32_t*, uint32_t*, const float*, int, int, int, float, int, const float*, int,
             const float*, uint32_t*, int);
int emu_rollout_tape_words(void*);
int emu_rollout(void*, float*, uint32_t*, uint32_t*, const float*, int, int, int, float, int, const float*, int,
                const float*, float*, float*, uint32_t*, uint32_t*, int);
int emu_rollout_backward(void*, const float*, const uint32_t*, const uint32_t*, const float*, int, int, int, float, int,
                         const float*, int, const float*, float*, float*, int);
const char* emu_last_error(void);
int emu_scene_destroy(void*);
}

template <class T>
static bool rd(FILE* f, std::vector<T>& v, size_t n) {
  v.resize(n);
  return fread(v.data(), sizeof(T), n, f) == n;
}
template <class T>
static void wr(FILE* f, const std::vector<T>& v) {
  fwrite(v.data(), sizeof(T), v.size(), f);
}

int main(int argc, char** argv) {
  if (argc != 3) return 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<int32_t> h;
  if (!rd(f, h, 10)) return 3;
  const int nb = h[0], np = h[1], B = h[2], T = h[3], stages = h[4], G = h[5], gs = h[6], mode = h[7], E = h[8],
            ab = h[9];
  std::vector<float> par, geom, dyn, act, rw;
  std::vector<int32_t> pb, pt, pn;
  std::vector<uint32_t> keys;
  if (!rd(f, par, nb * 4) || !rd(f, pb, np) || !rd(f, pt, np) || !rd(f, pn, np)) return 3;
  if (!rd(f, geom, gs ? (size_t)B * gs : (size_t)G) || !rd(f, dyn, (size_t)nb * 6 * B) || !rd(f, keys, 2 * (size_t)B))
    return 3;
  if (mode == 1 && (!rd(f, act, (size_t)T * B * 2) || !rd(f, rw, nb * 6))) return 3;
  fclose(f);
  void* sc = nullptr;
  if (emu_scene_create(nb, par.data(), np, pb.data(), pt.data(), pn.data(), &sc)) {
    fprintf(stderr, "%s\n", emu_last_error());
    return 4;
  }
  std::vector<uint32_t> err(B, 0u);
  FILE* o = fopen(argv[2], "wb");
  if (mode == 0) {
    emu_step(sc, dyn.data(), keys.data(), err.data(), geom.data(), gs, B, T, 1e-2f, stages, nullptr, 0, nullptr,
             nullptr, E);
    wr(o, dyn);
    wr(o, keys);
    wr(o, err);
  } else {
    const size_t B4 = (size_t)(B + 3) / 4 * 4;  // saved rows in env blocks of 4 (cxk::row_at)
    std::vector<float> ret(B, 0.0f), sd((size_t)T * nb * 6 * B4), ga((size_t)T * B * 2), gd((size_t)nb * 6 * B);
    std::vector<uint32_t> sk((size_t)T * B * 2), tape((size_t)T * emu_rollout_tape_words(sc) * B4, 0x7FBADBADu);
    emu_rollout(sc, dyn.data(), keys.data(), err.data(), geom.data(), gs, B, T, 1e-2f, stages, act.data(), ab,
                rw.data(), ret.data(), sd.data(), sk.data(), tape.data(), E);
    std::vector<float> ra(ga.size()), rd_(gd.size());
    if (emu_rollout_backward(sc, sd.data(), sk.data(), tape.data(), geom.data(), gs, B, T, 1e-2f, stages, act.data(),
                             ab, rw.data(), ga.data(), gd.data(), E) ||
        emu_rollout_backward(sc, sd.data(), sk.data(), nullptr, geom.data(), gs, B, T, 1e-2f, stages, act.data(), ab,
                             rw.data(), ra.data(), rd_.data(), E)) {
      fprintf(stderr, "%s\n", emu_last_error());
      return 5;
    }
    if (memcmp(ga.data(), ra.data(), ga.size() * 4) != 0 || memcmp(gd.data(), rd_.data(), gd.size() * 4) != 0) {
      fprintf(stderr, "tape backward != re-play backward\n");
      return 6;
    }
    wr(o, dyn);
    wr(o, keys);
    wr(o, err);
    wr(o, ret);
    wr(o, ga);
    wr(o, gd);
  }
  fclose(o);
  emu_scene_destroy(sc);
  return 0;
}
