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
#include <string.h>

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

// The same quantiser for the 8-wide node (DNode8, RT_NODES_WIDE8), whose
// steps are stored as bf16 (the upper half of an fp32): a step is rounded up
// to 8 significant bits, which can only widen the grid, and the bytes are
// then chosen on that grid exactly as above (the largest q with org + q step
// <= lo - m, the smallest with org + q step >= hi + m), so every child box
// holds its fp32 box plus the margin.  box[s] = {xlo, xhi, ylo, yhi, zlo,
// zhi} of slot s; used[s] false = an unused slot (lo 255, hi 0 on every
// axis).  Writes org, the three bf16 steps and the 18 plane words.
__host__ __device__ inline uint32_t nq_bf16_up(float f) {   // f >= 0: bits of the smallest bf16 >= f
  uint32_t b;
  memcpy(&b, &f, 4);
  if (b & 0xFFFFu) b = (b + 0x10000u) & 0xFFFF0000u;
  return b;
}
__host__ __device__ inline void quantize_node8(const float (*box)[6], const bool* used, float org[3], uint32_t step_bits[3],
                                               uint32_t q[18]) {
  double M = 0.0;
  for (int s = 0; s < 8; ++s)
    if (used[s])
      for (int k = 0; k < 6; ++k)
        if (fabs(double(box[s][k])) <= 0x1p96) M = fmax(M, fabs(double(box[s][k])));
  const double m = fmax(ldexp(M, -17), 0x1p-60);
  for (int a = 0; a < 3; ++a) {
    double L = HUGE_VAL, U = -HUGE_VAL;
    bool coarse = false, any = false;
    for (int s = 0; s < 8; ++s) {
      if (!used[s]) continue;
      const double l = box[s][2 * a], h = box[s][2 * a + 1];
      if (!(fabs(l) <= 0x1p96) || !(fabs(h) <= 0x1p96)) coarse = true;
      if (l < L) L = l;
      if (h > U) U = h;
      any = true;
    }
    float o = 0.0f;
    uint32_t sb = 0x3F800000u;   // 1.0
    if (coarse) {
      o = -0x1p107f;
      sb = 0x71800000u;          // 2^100 (exact in bf16)
    } else if (any) {
      o = nq_round_down(L - m);
      sb = nq_bf16_up(nq_round_up(fmax((U + m - double(o)) / 255.0, 0x1p-100)));
    }
    float st;
    memcpy(&st, &sb, 4);
    uint32_t lo[2] = {0u, 0u}, hi[2] = {0u, 0u};
    for (int s = 0; s < 8; ++s) {
      uint32_t bl = 255u, bh = 0u;   // unused slot: rejected on every axis
      if (used[s] && coarse) {
        bl = 0u;
        bh = 255u;
      } else if (used[s]) {
        const double tl = double(box[s][2 * a]) - m, th = double(box[s][2 * a + 1]) + m;
        double ql = floor((tl - double(o)) / double(st));
        double qh = ceil((th - double(o)) / double(st));
        if (ql < 0.0) ql = 0.0;
        if (qh > 255.0) qh = 255.0;
        while (ql > 0.0 && double(o) + ql * double(st) > tl) ql -= 1.0;
        while (qh < 255.0 && double(o) + qh * double(st) < th) qh += 1.0;
        bl = uint32_t(ql);
        bh = uint32_t(qh);
      }
      lo[s >> 2] |= bl << (8 * (s & 3));
      hi[s >> 2] |= bh << (8 * (s & 3));
    }
    org[a] = o;
    step_bits[a] = sb;
    uint32_t* r = q + 6 * a;   // lo, hi, lo: a 16-B window at +0 or +8 is (near, far)
    r[0] = lo[0]; r[1] = lo[1]; r[2] = hi[0]; r[3] = hi[1]; r[4] = lo[0]; r[5] = lo[1];
  }
}

}  // namespace rtg
