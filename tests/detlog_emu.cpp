// detlog_emu.cpp — test-only host build of the device's libm-free logarithm
// (go-raytracing_amd/csrc/device_common.h rt_logf) over every value the RNG
// can produce, k * 2^-24 for k in [0, 2^24).  tests/test_detlog.py compares
// the output bit for bit with the oracle's fp32 restatement (o_logf).
//
// usage: detlog_emu <out.f32>
#include <cstdio>
#include <vector>

#include "../go-raytracing_amd/csrc/device_common.h"

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const uint32_t n = 1u << 24;
  std::vector<float> out(n);
  for (uint32_t k = 0; k < n; ++k) out[k] = rtg::rt_logf(float(k) * 0x1p-24f);
  FILE* f = std::fopen(argv[1], "wb");
  if (!f) return 5;
  std::fwrite(out.data(), sizeof(float), out.size(), f);
  std::fclose(f);
  return 0;
}
