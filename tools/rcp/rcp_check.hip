// Exhaustive check (diagnostic): for every fp32 bit pattern x,
// does v_rcp_f32 + one FMA Newton step give the correctly rounded 1/x that
// IEEE division (hipcc's default fp32 divide) gives?  Counts mismatches per
// exponent class; prints the first few.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k_check(uint32_t base, unsigned long long* bad, unsigned long long* bad_normal, uint32_t* first) {
  const uint32_t bits = base + blockIdx.x * blockDim.x + threadIdx.x;
  const float x = __uint_as_float(bits);
  const float ref = 1.0f / x;
  const float r = __builtin_amdgcn_rcpf(x);
  const float e = fmaf(-x, r, 1.0f);
  const float y = fmaf(e, r, r);
  const bool same = __float_as_uint(ref) == __float_as_uint(y) || (ref != ref && y != y);
  if (!same) {
    atomicAdd(bad, 1ull);
    const uint32_t ex = (bits >> 23) & 0xFFu;
    if (ex >= 2u && ex <= 252u) {
      const unsigned long long k = atomicAdd(bad_normal, 1ull);
      if (k < 8ull) first[k] = bits;
    }
  }
}

int main() {
  unsigned long long *bad, *badn;
  uint32_t* first;
  hipMalloc(&bad, 8); hipMalloc(&badn, 8); hipMalloc(&first, 32);
  hipMemset(bad, 0, 8); hipMemset(badn, 0, 8); hipMemset(first, 0, 32);
  const uint32_t chunk = 1u << 28;
  for (uint64_t b = 0; b < (1ull << 32); b += chunk)
    hipLaunchKernelGGL(k_check, dim3(chunk / 256), dim3(256), 0, 0, uint32_t(b), bad, badn, first);
  unsigned long long h = 0, hn = 0;
  uint32_t f[8];
  hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
  hipMemcpy(&hn, badn, 8, hipMemcpyDeviceToHost);
  hipMemcpy(f, first, 32, hipMemcpyDeviceToHost);
  printf("mismatches: all %llu, exponent field 2..252: %llu\n", h, hn);
  for (int i = 0; i < 8 && i < int(hn); ++i) printf("  x bits 0x%08x = %.9g\n", f[i], __builtin_bit_cast(float, f[i]));
  return 0;
}
