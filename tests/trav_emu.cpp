// trav_emu.cpp — test-only host build of the device path-tracing code
// (go-raytracing_amd/csrc/device_common.h: traversal, shading, NEE) with one
// lane per wave, driven over a librtscene scene flattened by flatten.cpp.
// Lets the CPU suite (tests/test_flatten_host.py) run the kernels' own source
// under AddressSanitizer and compare it with the oracle.  Not a product path:
// the product is the gfx950 build in librtgpu.so.
//
// usage: trav_emu <scene> <width> <spp> <seed> <asset_dir> <out.f32>
// writes H*W*3 float sums (the accumulation buffer rt_render returns).
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../go-raytracing_amd/csrc/device_common.h"
#include "emu_scene.h"

using namespace rtg;

int main(int argc, char** argv) {
  if (argc < 7) return 2;
  const int spp = atoi(argv[3]);
  const uint32_t seed = uint32_t(strtoul(argv[4], nullptr, 10));
  emu::EmuScene E;
  if (int rc = emu::load(argv[1], atoi(argv[2]), argv[5], E)) return rc;
  const DScene& d = E.d;
  const DCamera& cam = E.cam;

  const int W = cam.width, H = cam.height, cap = E.h.stack_needed;
  // a 4-entry LDS ring + a spill area of exactly the remaining bound: every
  // traversal deeper than 4 goes through the spill path; overflow -> err,
  // ASan sees any out-of-range slot
  const int ring = 4, spill_cap = cap > ring ? cap - ring : 0;
  std::vector<uint32_t> ring_mem(static_cast<size_t>(ring)), spill_mem(static_cast<size_t>(spill_cap > 0 ? spill_cap : 1));
  std::vector<float> world_ray(9);
  const TStack S{ring_mem.data(), 1, ring, spill_mem.data(), 1, spill_cap, world_ray.data()};
  std::vector<float> out(size_t(W) * H * 3, 0.0f);
  int e = 0;
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      double s[3] = {0, 0, 0};
      for (int k = 0; k < spp; ++k) {
        Cnt cnt{};
        const uint32_t key = path_key(seed, uint32_t(y * W + x), uint32_t(k));
        V3 L = trace_path<false>(d, cam, x, y, key, E.max_depth, S, cnt, &e);
        s[0] += L.x; s[1] += L.y; s[2] += L.z;
      }
      float* o = &out[(size_t(y) * W + x) * 3];
      o[0] = float(s[0]); o[1] = float(s[1]); o[2] = float(s[2]);
    }
  FILE* f = fopen(argv[6], "wb");
  if (!f) return 5;
  fwrite(out.data(), sizeof(float), out.size(), f);
  fclose(f);
  printf("{\"width\": %d, \"height\": %d, \"stack_needed\": %d, \"overflow\": %d}\n", W, H, cap, e);
  return e ? 6 : 0;
}
