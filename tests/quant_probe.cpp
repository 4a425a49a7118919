// quant_probe.cpp — test-only: the RT_NODES_QUANT8 node quantiser
// (go-raytracing_amd/csrc/node_quant.h) on random BVH4 nodes.
//   1. containment: every used child's dequantised planes (origin + q step,
//      evaluated in double) lie at least the margin outside its fp32 planes;
//      unused children encode lo = 255 / hi = 0 on every axis;
//   2. conservative fp32 slab test: for rays aimed at random points on or
//      inside a child box from up to 20 node magnitudes away (grazing edges
//      and corners included), the traversal's quantised test
//      (device_common.h: fma(q, inv * step, (origin - o) * inv), fmaxf/fminf)
//      accepts the child with an interval that holds the aimed point;
//   3. outside that envelope (measured, not asserted): rays from 10^2 to
//      10^5 node magnitudes away.  There the aimed point itself is lost in
//      the rounding of o, so the reference is the fp32 format's own slab test
//      on the child's DNode4 box (device_common.h, fp32 branch): far_fail
//      counts rays that box accepts but the quantised test rejects or
//      narrows (rtgpu.h documents the envelope).
// Prints one JSON line; exit code 0 iff no violation of 1 and 2.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <random>

#include "../go-raytracing_amd/csrc/node_quant.h"

using namespace rtg;

int main(int argc, char** argv) {
  const int nodes = argc > 1 ? atoi(argv[1]) : 20000;
  std::mt19937_64 rng(12345);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  long contain_fail = 0, slab_fail = 0, rays = 0, unused_fail = 0, far_rays = 0, far_fail = 0;
  const float inf = HUGE_VALF;
  for (int it = 0; it < nodes; ++it) {
    // node magnitude and child size span many decades (world walls to mesh leaves)
    const double mag = std::pow(10.0, -3.0 + 7.0 * U(rng));
    const double size = mag * std::pow(10.0, -6.0 * U(rng));
    DNode4 n{};
    const int used = 1 + int(U(rng) * 4.0);
    for (int c = 0; c < 4; ++c) {
      float* lo[3] = {&n.xlo[c], &n.ylo[c], &n.zlo[c]};
      float* hi[3] = {&n.xhi[c], &n.yhi[c], &n.zhi[c]};
      for (int a = 0; a < 3; ++a) {
        if (c >= used) { *lo[a] = inf; *hi[a] = -inf; continue; }
        const double ctr = (U(rng) * 2.0 - 1.0) * mag;
        const double ext = U(rng) < 0.2 ? 0.0 : U(rng) * size;   // flat boxes (axis-aligned quads)
        *lo[a] = float(ctr);
        *hi[a] = std::nextafter(float(ctr + ext), inf);
        if (*hi[a] < *lo[a]) *hi[a] = *lo[a];
      }
      n.item[c] = uint32_t(c);
    }
    const DNodeQ q = quantize_node(n);
    const float* lo4[3] = {n.xlo, n.ylo, n.zlo};
    const float* hi4[3] = {n.xhi, n.yhi, n.zhi};
    for (int c = 0; c < 4; ++c)
      for (int a = 0; a < 3; ++a) {
        const uint32_t bl = (q.q[2 * a] >> (8 * c)) & 255u, bh = (q.q[2 * a + 1] >> (8 * c)) & 255u;
        if (c >= used) { unused_fail += !(bl == 255u && bh == 0u); continue; }
        double M = 0.0;
        for (int b = 0; b < 3; ++b)
          for (int k = 0; k < used; ++k) M = std::fmax(M, std::fmax(std::fabs(lo4[b][k]), std::fabs(hi4[b][k])));
        const double m = std::fmax(std::ldexp(M, -17), 0x1p-60);
        const double pl = double(q.org[a]) + double(bl) * double(q.step[a]);
        const double ph = double(q.org[a]) + double(bh) * double(q.step[a]);
        contain_fail += !(pl <= double(lo4[a][c]) - m && ph >= double(hi4[a][c]) + m);
      }
    // rays at points on / inside the used children
    for (int r = 0; r < 12; ++r) {
      const bool far = r >= 8;   // outside the documented envelope
      const int c = int(U(rng) * used);
      double P[3];
      for (int a = 0; a < 3; ++a) {
        const double l = lo4[a][c], h = hi4[a][c];
        const double u = U(rng);
        P[a] = u < 0.3 ? l : u < 0.6 ? h : l + (h - l) * U(rng);   // faces, edges, corners
      }
      const double dist = far ? mag * std::pow(10.0, 2.0 + 3.0 * U(rng))    // 10^2..10^5 magnitudes away
                              : mag * std::pow(10.0, -2.0 + 3.3 * U(rng));  // up to 20 magnitudes away
      double dir[3], len = 0.0;
      for (double& v : dir) { v = U(rng) * 2.0 - 1.0; len += v * v; }
      len = std::sqrt(len);
      float o[3], d[3], inv[3];
      for (int a = 0; a < 3; ++a) {
        d[a] = float(dir[a] / len * dist);
        o[a] = float(P[a] - double(d[a]));   // o + 1 * d ~ P
        inv[a] = 1.0f / d[a];
      }
      // the real-number ray o + t d passes P's neighbourhood at t ~ 1: the
      // quantised test must accept the child with [a, b] around t = 1
      float A[3], B[3];
      uint32_t nr[3], fr[3];
      for (int a = 0; a < 3; ++a) {
        A[a] = (q.org[a] - o[a]) * inv[a];
        B[a] = inv[a] * q.step[a];
        const bool s = std::signbit(inv[a]);
        nr[a] = s ? q.q[2 * a + 1] : q.q[2 * a];
        fr[a] = s ? q.q[2 * a] : q.q[2 * a + 1];
      }
      auto qf = [c](uint32_t row) { return float((row >> (8 * c)) & 0xFFu); };
      float ta = 0.0f, tb = inf;
      for (int a = 0; a < 3; ++a) {
        ta = std::fmax(ta, std::fma(qf(nr[a]), B[a], A[a]));
        tb = std::fmin(tb, std::fma(qf(fr[a]), B[a], A[a]));
      }
      const bool ok = tb > ta && ta <= 1.0f + 0x1p-20f && tb >= 1.0f - 0x1p-20f;
      if (far) {
        // the fp32 format's test of the same child: planes picked by the
        // direction's sign, (plane - o) * inv, fmaxf / fminf from [0, inf]
        float fa = 0.0f, fb = inf;
        for (int a = 0; a < 3; ++a) {
          const bool s = std::signbit(inv[a]);
          const float np = s ? hi4[a][c] : lo4[a][c], fp = s ? lo4[a][c] : hi4[a][c];
          fa = std::fmax(fa, (np - o[a]) * inv[a]);
          fb = std::fmin(fb, (fp - o[a]) * inv[a]);
        }
        if (fb > fa) {
          ++far_rays;
          far_fail += !(tb > ta && ta <= fa && tb >= fb);
        }
        continue;
      }
      ++rays;
      // P itself is only float-close to o + d: allow 2^-20 relative in t
      if (!ok) {
        if (getenv("QP_VERBOSE") && slab_fail < 8)
          fprintf(stderr, "fail mag %g size %g dist %g ta %.9g tb %.9g\n", mag, size, dist, ta, tb);
        ++slab_fail;
      }
    }
  }
  printf("{\"nodes\": %d, \"rays\": %ld, \"contain_fail\": %ld, \"unused_fail\": %ld, \"slab_fail\": %ld, "
         "\"far_rays\": %ld, \"far_fail\": %ld}\n", nodes, rays, contain_fail, unused_fail, slab_fail, far_rays, far_fail);
  return contain_fail || unused_fail || slab_fail ? 1 : 0;
}
