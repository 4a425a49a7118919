// ray_emu.cpp — test-only: the production closest-hit kernel (wavefront.hip
// k_extend, a later bounce: rays read from the path stream) compiled for the
// host, one lane, over given rays.  Reads "ox oy oz dx dy dz" lines from
// stdin, prints "kind idx t(bits) inst refpos" per ray: the hit record
// k_extend stores (store_hit).  Used to replay single rays of a GPU render
// on the host (tools/format_diff.py finds them).  Not a product path.
//
// usage: ray_emu <scene> <width> <asset_dir>   (RTG_EMU_QUANT / RTG_EMU_FULL_LUCY as wave_emu)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../go-raytracing_amd/csrc/wavefront.hip"
#include "emu_scene.h"

using namespace rtg;

namespace {

constexpr int kRing = 8;

template <bool kWide, bool kQuant>
float4 trace(const DScene& sc, const DCamera& cam, WaveArgs a, float4 o, float4 d) {
  a.s[0].o[0] = o;
  a.s[0].d[0] = d;
  a.s[0].beta[0] = float4{1.0f, 1.0f, 1.0f, 0.0f};
  a.counts[CNT_STREAM0] = 1u;
  for (uint32_t k = 0; k < kSegs; ++k) a.counts[CNT_FETCH_EXT + k * kSegStride] = 0u;
  k_extend<kRing, false, false, false, kQuant, kWide>(sc, cam, a, a.s[0], a.counts + CNT_STREAM0, a.counts + CNT_STREAM1,
                                                      a.counts + CNT_SHADOW, a.counts + CNT_FETCH_SH,
                                                      a.counts + CNT_FETCH_EXT, 0u);
  return a.hit[0];
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  emu::EmuScene E;
  if (int rc = emu::load(argv[1], atoi(argv[2]), argv[3], E)) return rc;
  const DScene& d = E.d;
  if (d.has_volumes || d.n_circles > 0 || d.dfs_order) {
    fprintf(stderr, "ray_emu: rare-primitive scenes are not supported\n");
    return 3;
  }
  std::vector<float4> f4(size_t(kSlotF4), float4{0.0f, 0.0f, 0.0f, 0.0f});
  std::vector<uint32_t> q(CNT_WORDS_Q, 0u), sj(2, 0u);
  std::vector<uint32_t> pixels(1, 0u), spill(size_t(kStackMax - kRing), 0u);
  std::vector<double> acc(3, 0.0);
  std::vector<unsigned long long> counters(3 * CNT_BLOCK, 0ull);
  int err = 0;
  WaveArgs a{};
  auto arr = [&](int k) { return &f4[size_t(k)]; };
  for (int k = 0; k < 2; ++k) a.s[k] = PathStream{arr(3 * k), arr(3 * k + 1), arr(3 * k + 2)};
  a.hit = arr(6); a.Lout = arr(7);
  a.sj_p = arr(8); a.sj_a = arr(9); a.sj_h = arr(10);
  a.ne_a = arr(11); a.ne_h = arr(12); a.ne_beta = arr(13);
  a.counts = q.data();
  a.sj_info = sj.data();
  a.sj_vis = sj.data() + 1;
  a.pixels = pixels.data();
  a.npix = 1;
  a.acc = acc.data();
  a.max_depth = E.max_depth;
  a.counters = counters.data();
  a.err = &err;
  a.refill = 1;
  a.spill = spill.data();
  a.spill_lanes = 1;
  a.spill_cap = kStackMax - kRing;
  a.slots = 1;
  a.out_pixels = 1;
  float o[3], dd[3];
  while (scanf("%f %f %f %f %f %f", &o[0], &o[1], &o[2], &dd[0], &dd[1], &dd[2]) == 6) {
    const float4 ro{o[0], o[1], o[2], 0.0f}, rd{dd[0], dd[1], dd[2], 0.0f};
    const float4 h = d.wide_nodes ? trace<true, false>(d, E.cam, a, ro, rd)
                     : d.quant_nodes ? trace<false, true>(d, E.cam, a, ro, rd)
                                     : trace<false, false>(d, E.cam, a, ro, rd);
    uint32_t w[4];
    memcpy(w, &h, 16);
    printf("%u %u %.9g %d %d\n", w[1] >> 28, w[1] & 0x0FFFFFFFu, double(h.x), int(w[2]), int(w[3]));
  }
  return err ? 6 : 0;
}
