// node_quant.h — DNode4 (fp32 child boxes) -> DNodeQ (8-bit child planes in
// a per-axis node frame), shared by the device quantise kernel
// (build.hip k_quantize) and the host emulation of the traversal
// (tests/emu_scene.h), so both read the same bytes.
//
// Margin m = 2^-17 M (at least 2^-60), M = the largest |coordinate| of the
// node's used child planes on any axis: the slab test evaluates a plane's t
// in fp32 as fma(q, inv * step, (origin - o) * inv), whose rounding error is
// a few ulps of the ray's distance to the node; every dequantised plane lies
// at least m outside the fp32 plane, which covers that error (and keeps a
// thin box's slab interval several ulps long) for rays up to ~20 node
// magnitudes away, so the test is conservative.
// Per axis, over the node's used children [L, U] (fp32 values):
//   * origin = L - m rounded down to fp32; step = (U + m - origin) / 255
//     rounded up to fp32 (at least 2^-100);
//   * lo byte = the largest q with origin + q step <= lo - m,
//     hi byte = the smallest q with origin + q step >= hi + m (in [0, 255]),
//     checked in double (origin + q step is exact to far below m there).
// An axis with a non-finite or huge (|x| > 2^96) used plane gets the coarse
// frame origin -2^107, step 2^100, bytes 0 / 255: it then culls nothing.
#pragma once
#include <math.h>
#include <stdint.h>

#include "dev_layout.h"

namespace rtg {

__host__ __device__ inline float nq_round_down(double x) {
  float f = float(x);
  if (double(f) > x) f = nextafterf(f, -HUGE_VALF);
  return f;
}
__host__ __device__ inline float nq_round_up(double x) {
  float f = float(x);
  if (double(f) < x) f = nextafterf(f, HUGE_VALF);
  return f;
}

__host__ __device__ inline DNodeQ quantize_node(const DNode4& n) {
  DNodeQ q;
  const float* lo[3] = {n.xlo, n.ylo, n.zlo};
  const float* hi[3] = {n.xhi, n.yhi, n.zhi};
  bool used[4];
  for (int c = 0; c < 4; ++c) {
    used[c] = n.xlo[c] <= n.xhi[c] && n.ylo[c] <= n.yhi[c] && n.zlo[c] <= n.zhi[c];
    q.item[c] = n.item[c];
  }
  double M = 0.0;   // node magnitude over the finite used planes
  for (int a = 0; a < 3; ++a)
    for (int c = 0; c < 4; ++c)
      if (used[c] && fabs(lo[a][c]) <= 0x1p96 && fabs(hi[a][c]) <= 0x1p96)
        M = fmax(M, fmax(fabs(double(lo[a][c])), fabs(double(hi[a][c]))));
  const double m = fmax(ldexp(M, -17), 0x1p-60);
  for (int a = 0; a < 3; ++a) {
    double L = HUGE_VAL, U = -HUGE_VAL;
    bool coarse = false, any = false;
    for (int c = 0; c < 4; ++c) {
      if (!used[c]) continue;
      const double l = lo[a][c], h = hi[a][c];
      if (!(fabs(l) <= 0x1p96) || !(fabs(h) <= 0x1p96)) coarse = true;
      if (l < L) L = l;
      if (h > U) U = h;
      any = true;
    }
    float org = 0.0f, step = 1.0f;
    if (coarse) {
      org = -0x1p107f;
      step = 0x1p100f;
    } else if (any) {
      org = nq_round_down(L - m);
      step = nq_round_up(fmax((U + m - double(org)) / 255.0, 0x1p-100));
    }
    uint32_t rlo = 0, rhi = 0;
    for (int c = 0; c < 4; ++c) {
      uint32_t bl = 255u, bh = 0u;   // unused child: rejected on every axis
      if (used[c] && coarse) {
        bl = 0u;
        bh = 255u;
      } else if (used[c]) {
        const double tl = double(lo[a][c]) - m, th = double(hi[a][c]) + m;
        double ql = floor((tl - double(org)) / double(step));
        double qh = ceil((th - double(org)) / double(step));
        if (ql < 0.0) ql = 0.0;
        if (qh > 255.0) qh = 255.0;
        while (ql > 0.0 && double(org) + ql * double(step) > tl) ql -= 1.0;
        while (qh < 255.0 && double(org) + qh * double(step) < th) qh += 1.0;
        bl = uint32_t(ql);
        bh = uint32_t(qh);
      }
      rlo |= bl << (8 * c);
      rhi |= bh << (8 * c);
    }
    q.org[a] = org;
    q.step[a] = step;
    q.q[2 * a] = rlo;
    q.q[2 * a + 1] = rhi;
  }
  return q;
}

}  // namespace rtg
