// fetch_calib.hip — calibration of rocprofv3's FETCH_SIZE for the access
// patterns of the traversal kernels.  FETCH_SIZE counts
// the L2's memory-side read requests (TCC_EA0_RDREQ, tallied at 32 / 64 B;
// MI355X_MICROARCH.md: a coalesced 128-B line read is tallied at 64 B), so
// what one missed line costs in its units depends on the request the L2
// issues for that access width.  Each pattern below misses a known number of
// 128-B lines exactly once: a table of N lines, L2 cleared before every
// measured launch by streaming a 96 MB buffer (larger than the 32 MB of L2,
// small enough that the 8 MB table stays in the 256 MB Infinity Cache), every
// line touched by one lane (or one 8-lane group) in a random permutation:
//   stream   16 B per lane, coalesced (lane i reads row i): N x 128 B read
//   line8    8 lanes read the 8 rows of one line in one instruction: N x 128 B
//   row16    one lane reads one 16-B row of its line: N x 16 B requested
//   node7    one lane reads 7 of its line's 8 rows in 7 loads, near / far
//            rows picked by per-lane signs as trav_step does: N x 112 B
//            requested (k_extend's BVH4 node step, device_common.h)
// Run under rocprofv3 --pmc (tools/fetch_calib.sh); the dispatch order is
// printed so tools/fetch_calib.py can name each dispatch.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <random>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void k_flush(const float4* __restrict__ b, size_t n, float* out) {
  float s = 0.0f;
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
    const float4 v = b[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 1.2345f) out[0] = s;   // keeps the loads; never true for the fill below
}
__global__ void k_stream(const float4* __restrict__ t, uint32_t rows, float* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows) return;
  const float4 v = t[i];
  out[i] = v.x + v.y + v.z + v.w;
}
__global__ void k_line8(const float4* __restrict__ t, const uint32_t* __restrict__ perm, uint32_t lines, float* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= lines * 8u) return;
  const float4 v = t[size_t(perm[i >> 3]) * 8u + (i & 7u)];
  out[i] = v.x + v.y + v.z + v.w;
}
__global__ void k_row16(const float4* __restrict__ t, const uint32_t* __restrict__ perm, uint32_t lines, float* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= lines) return;
  const float4 v = t[size_t(perm[i]) * 8u + (i & 7u)];
  out[i] = v.x + v.y + v.z + v.w;
}
__global__ void k_node7(const float4* __restrict__ t, const uint32_t* __restrict__ perm, uint32_t lines, float* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= lines) return;
  const char* nb = reinterpret_cast<const char*>(t) + size_t(perm[i]) * 128u;
  const uint32_t h = i * 0x9E3779B9u;
  const uint32_t sx = (h >> 27) & 16u, sy = (h >> 26) & 16u, sz = (h >> 25) & 16u;
  auto ld = [&](uint32_t off) { return *reinterpret_cast<const float4*>(nb + off); };
  const float4 nx = ld(sx), fx = ld(16u - sx), ny = ld(32u + sy), fy = ld(48u - sy), nz = ld(64u + sz), fz = ld(80u - sz);
  const float4 it = ld(96u);
  out[i] = nx.x + fx.y + ny.z + fy.w + nz.x + fz.y + it.z;
}

int main(int argc, char** argv) {
  const uint32_t lines = argc > 1 ? uint32_t(atoi(argv[1])) : 65536u;   // 8 MB table
  const int reps = argc > 2 ? atoi(argv[2]) : 3;
  const size_t flush_n = (size_t(96) << 20) / sizeof(float4);
  float4 *table = nullptr, *flush = nullptr;
  uint32_t* perm = nullptr;
  float* out = nullptr;
  CK(hipMalloc(&table, size_t(lines) * 128u));
  CK(hipMalloc(&flush, flush_n * sizeof(float4)));
  CK(hipMalloc(&perm, size_t(lines) * 4u));
  CK(hipMalloc(&out, size_t(lines) * 8u * sizeof(float)));
  CK(hipMemset(table, 0x3c, size_t(lines) * 128u));
  CK(hipMemset(flush, 0x3c, flush_n * sizeof(float4)));
  std::vector<uint32_t> p(lines);
  for (uint32_t k = 0; k < lines; ++k) p[k] = k;
  std::mt19937 rng(12345);
  std::shuffle(p.begin(), p.end(), rng);
  CK(hipMemcpy(perm, p.data(), size_t(lines) * 4u, hipMemcpyHostToDevice));
  const uint32_t rows = lines * 8u;
  auto flush_l2 = [&]() { hipLaunchKernelGGL(k_flush, dim3(2048), dim3(256), 0, 0, flush, flush_n, out); };
  // warm the table into the Infinity Cache
  hipLaunchKernelGGL(k_stream, dim3((rows + 255) / 256), dim3(256), 0, 0, table, rows, out);
  int d = 0;
  printf("{\"lines\": %u, \"line_bytes\": 128, \"dispatches\": [", lines);
  for (int r = 0; r < reps; ++r) {
    const char* names[4] = {"stream", "line8", "row16", "node7"};
    for (int k = 0; k < 4; ++k) {
      flush_l2();
      d += 1;   // the flush
      if (k == 0) hipLaunchKernelGGL(k_stream, dim3((rows + 255) / 256), dim3(256), 0, 0, table, rows, out);
      if (k == 1) hipLaunchKernelGGL(k_line8, dim3((rows + 255) / 256), dim3(256), 0, 0, table, perm, lines, out);
      if (k == 2) hipLaunchKernelGGL(k_row16, dim3((lines + 255) / 256), dim3(256), 0, 0, table, perm, lines, out);
      if (k == 3) hipLaunchKernelGGL(k_node7, dim3((lines + 255) / 256), dim3(256), 0, 0, table, perm, lines, out);
      d += 1;
      printf("%s\"%s\"", (r || k) ? ", " : "", names[k]);
    }
  }
  CK(hipDeviceSynchronize());
  printf("]}\n");
  return 0;
}
