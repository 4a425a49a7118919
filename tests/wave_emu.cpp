// wave_emu.cpp — test-only host build of the production wavefront pipeline
// (go-raytracing_amd/csrc/wavefront.hip kernels: camera, extend, shade,
// shadow, NEE apply, accumulate, finalize) with one lane per workgroup and
// one workgroup per launch, driven like run_batches() over a librtscene scene
// flattened by flatten.cpp.  Runs under AddressSanitizer + UBSan in the CPU
// suite (tests/test_flatten_host.py): every stream / queue / job index the
// kernels compute is checked against exactly-sized host buffers.  The
// traversal stack ring is 4 entries so deep traversals take the spill path.
// Not a product path: the product is the gfx950 build in librtgpu.so.
//
// usage: wave_emu <scene> <width> <spp> <seed> <asset_dir> <out.f32> [batch_spp]
// writes H*W*3 float sums (the accumulation buffer rt_render returns).
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../go-raytracing_amd/csrc/wavefront.hip"
#include "emu_scene.h"

using namespace rtg;

namespace {

constexpr int kRing = 4;

template <bool kVol, bool kEnvIS, int kShade, bool kQuant, bool kWide = false>
void run(const DScene& sc, const DCamera& cam, WaveArgs a, uint32_t spp, uint32_t spb, int max_depth, float* out) {
  uint32_t* cnt_stream[2] = {a.counts + CNT_STREAM0, a.counts + CNT_STREAM1};
  uint32_t* fetch_ext = a.counts + CNT_FETCH_EXT;
  for (double* p = a.acc; p < a.acc + size_t(a.npix) * 3; ++p) *p = 0.0;
  const int tail_after = getenv("RTG_EMU_TAIL") ? atoi(getenv("RTG_EMU_TAIL")) : -1;
  // RTG_EMU_OVERLAP=1: the bounce overlap's order (run_batches, WavePlan::
  // overlap): bounce b's k_shadow / k_nee_apply only after bounce b + 1's
  // k_extend has run to its end, the most any interleaving of the two streams
  // can separate them
  const bool ovl = getenv("RTG_EMU_OVERLAP") && atoi(getenv("RTG_EMU_OVERLAP")) > 0;
  auto nee = [&](int b) {   // as run_batches: no lights, no NEE launches
    if (sc.num_lights == 0) return;
    uint32_t* const cnt_sh = a.counts + cnt_shadow(b & 1);
    k_shadow<kRing, false, kVol, kEnvIS, kQuant, kWide>(sc, a, cnt_sh, a.counts + cnt_fetch_sh(b & 1),
                                                        a.counts + cnt_fetch_sh((b + 1) & 1));
    k_nee_apply<kEnvIS>(a, cnt_sh);
  };
  for (uint32_t s0 = 0; s0 < spp; s0 += spb) {
    const uint32_t sb = spp - s0 < spb ? spp - s0 : spb;
    const uint32_t nslots = sb * a.npix;
    k_set_counts(a.counts, nslots);
    int pending = -1;   // the bounce whose NEE kernels have not run yet (ovl)
    for (int b = 0; b < max_depth; ++b) {
      const int c = b & 1, nx = c ^ 1;
      uint32_t* const cnt_sh = a.counts + cnt_shadow(c);
      uint32_t* const fetch_sh = a.counts + cnt_fetch_sh(c);
      if (b == 0)
        k_extend<kRing, false, kVol, true, kQuant, kWide>(sc, cam, a, a.s[c], cnt_stream[c], cnt_stream[nx], cnt_sh, fetch_sh,
                                                          fetch_ext, s0);
      else
        k_extend<kRing, false, kVol, false, kQuant, kWide>(sc, cam, a, a.s[c], cnt_stream[c], cnt_stream[nx], cnt_sh, fetch_sh,
                                                           fetch_ext, s0);
      if (pending >= 0) { nee(pending); pending = -1; }
      if (b == 0) k_shade<false, kEnvIS, kShade, true>(sc, cam, a, a.s[c], cnt_stream[c], a.s[nx], cnt_stream[nx], cnt_sh, s0, 0u);
      else k_shade<false, kEnvIS, kShade, false>(sc, cam, a, a.s[c], cnt_stream[c], a.s[nx], cnt_stream[nx], cnt_sh, s0,
                                                  uint32_t(b));
      if (ovl) pending = b;
      else nee(b);
      // RTG_EMU_TAIL=b: after bounce b the long-tail kernel carries every
      // path left to its end (run_batches' hand-off, scenes without lights)
      if (sc.num_lights == 0 && tail_after >= 0 && b == tail_after && b + 1 < max_depth) {
        k_tail<kRing, kVol, kShade, kQuant, kWide>(sc, cam, a, a.s[nx], cnt_stream[nx], fetch_ext);
        break;
      }
    }
    if (pending >= 0) nee(pending);
    k_accum(a, sb);
  }
  k_finalize(a, out, 0);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 7) return 2;
  const uint32_t spp = uint32_t(atoi(argv[3]));
  const uint32_t seed = uint32_t(strtoul(argv[4], nullptr, 10));
  const uint32_t spb = argc > 7 ? uint32_t(atoi(argv[7])) : spp;
  emu::EmuScene E;
  if (int rc = emu::load(argv[1], atoi(argv[2]), argv[5], E)) return rc;
  const DScene& d = E.d;
  const DCamera& cam = E.cam;
  const uint32_t npix = uint32_t(cam.width) * uint32_t(cam.height);
  const size_t S = size_t(spb) * npix;

  // exactly-sized buffers, one allocation per array (render_wave in api.cpp
  // carves the same arrays out of one buffer; separate ones let ASan see a
  // store that leaves its array)
  std::vector<std::vector<float4>> f4(kSlotF4, std::vector<float4>(S, float4{0.0f, 0.0f, 0.0f, 0.0f}));
  std::vector<uint32_t> q(CNT_WORDS_Q, 0u), sj_info(S, 0u), sj_vis(S, 0u);
  std::vector<uint32_t> pixels(npix);
  // bucket-like pixel list: reversed, so slot -> pixel is not the identity
  for (uint32_t i = 0; i < npix; ++i) pixels[i] = npix - 1u - i;
  std::vector<uint32_t> spill(size_t(kStackMax - kRing), 0u), spill_sh(size_t(kStackMax - kRing), 0u);
  std::vector<double> acc(size_t(npix) * 3, 0.0);
  std::vector<unsigned long long> counters(3 * CNT_BLOCK, 0ull);
  int err = 0;

  WaveArgs a{};
  auto arr = [&](int k) { return f4[size_t(k)].data(); };
  for (int k = 0; k < 2; ++k) a.s[k] = PathStream{arr(3 * k), arr(3 * k + 1), arr(3 * k + 2)};
  a.hit = arr(6); a.Lout = arr(7);
  a.sj_p = arr(8); a.sj_a = arr(9); a.sj_h = arr(10);
  a.ne_a = arr(11); a.ne_h = arr(12); a.ne_beta = arr(13);
  a.counts = q.data();
  a.sj_info = sj_info.data();
  a.sj_vis = sj_vis.data();
  a.pixels = pixels.data();
  a.npix = npix;
  a.acc = acc.data();
  a.seed = seed;
  a.max_depth = E.max_depth;
  a.counters = counters.data();
  a.err = &err;
  a.refill = 1;                      // one lane per wave: claim whenever idle
  a.spill = spill.data();
  a.spill_sh = spill_sh.data();
  a.spill_lanes = 1;
  a.spill_cap = kStackMax - kRing;
  a.slots = uint32_t(S);
  a.out_pixels = uint32_t(npix);

  std::vector<float> out(size_t(npix) * 3, 0.0f);
  const bool vol = d.has_volumes != 0 || d.n_circles > 0 || d.dfs_order != 0, envis = d.env.valid && d.env.use_is;
#define RUNQ(V, H, F)                                                  \
  do {                                                                 \
    if constexpr (!(V)) {                                              \
      if (d.wide_nodes) { run<V, H, F, false, true>(d, cam, a, spp, spb, E.max_depth, out.data()); break; } \
    }                                                                  \
    if (d.quant_nodes) run<V, H, F, true>(d, cam, a, spp, spb, E.max_depth, out.data()); \
    else run<V, H, F, false>(d, cam, a, spp, spb, E.max_depth, out.data()); \
  } while (0)
#define RUN(V, H)                                                      \
  do {                                                                 \
    if (d.shade_kind == SHADE_FULL) RUNQ(V, H, SHADE_FULL);            \
    else if (d.shade_kind == SHADE_VOL) RUNQ(V, H, SHADE_VOL);         \
    else if (d.shade_kind == SHADE_MAT) RUNQ(V, H, SHADE_MAT);         \
    else RUNQ(V, H, SHADE_LEAN);                                       \
  } while (0)
  if (vol) {
    if (envis) RUN(true, true); else RUN(true, false);
  } else {
    if (envis) RUN(false, true); else RUN(false, false);
  }
#undef RUNQ
#undef RUN
  FILE* f = fopen(argv[6], "wb");
  if (!f) return 5;
  fwrite(out.data(), sizeof(float), out.size(), f);
  fclose(f);
  printf("{\"width\": %d, \"height\": %d, \"slots\": %zu, \"overflow\": %d, \"wide\": %d, \"nodes8\": %zu, \"rgbe\": %d}\n",
         cam.width, cam.height, S, err, d.wide_nodes, E.h.nodes8.size(), d.env.rgbe != nullptr ? 1 : 0);
  return err ? 6 : 0;
}
