// claim_perm_emu.cpp — test-only host build of the traversal kernels' claim
// order (go-raytracing_amd/csrc/device_common.h claim_perm): for every queue
// length n in the given list, every claim index in [0, n) maps to a distinct
// position in [0, n), and 64-claim blocks stay 64 consecutive positions.
// Prints "ok" or the first failure.  Built and run by tests/test_claim_perm.py.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../go-raytracing_amd/csrc/device_common.h"

int main(int argc, char** argv) {
  for (int a = 1; a < argc; ++a) {
    const uint32_t n = uint32_t(std::strtoul(argv[a], nullptr, 10));
    std::vector<unsigned char> seen(n, 0);
    for (uint32_t i = 0; i < n; ++i) {
      const uint32_t p = rtg::claim_perm(i, n);
      if (p >= n || seen[p]) { std::printf("n %u: claim %u -> %u %s\n", n, i, p, p >= n ? "out of range" : "repeated"); return 1; }
      seen[p] = 1;
      if ((i & 63u) != 0u && p != rtg::claim_perm(i - 1u, n) + 1u) {
        std::printf("n %u: claim %u not next to claim %u\n", n, i, i - 1u);
        return 1;
      }
    }
  }
  std::printf("ok\n");
  return 0;
}
