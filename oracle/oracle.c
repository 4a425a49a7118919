/*
 * oracle.c — CPU oracle (TEST INFRASTRUCTURE ONLY, see oracle.h).
 *
 * Parity status: the Go reference has no tests, golden vectors or
 * fixtures for this path and cannot be built here (no
 * Go toolchain), so this restatement is pinned by (1) hand-derived
 * known-answer tests of each Go formula (tests/test_oracle_kat.py), (2) the
 * reference's one data artifact, the HDRI asset (decode statistics,
 * totalPower), and (3) statistical agreement with /root/reference/image.png.
 * See DESIGN.md §Parity.
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------ RNG */
static inline uint32_t o_lowbias32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
static inline uint32_t o_path_key(uint32_t seed, uint32_t pixel, uint32_t sample) {
  uint32_t k = o_lowbias32(seed ^ 0xA511E9B3u);
  k = o_lowbias32(k ^ pixel);
  return o_lowbias32(k + sample * 0x9E3779B9u);
}
static inline uint32_t o_ctr(uint32_t bounce, uint32_t dom, uint32_t idx) { return (bounce << 16) | (dom << 12) | idx; }
static inline uint32_t o_draw(uint32_t key, uint32_t counter) { return o_lowbias32(key ^ o_lowbias32(counter ^ 0x632BE5ABu)); }

enum { O_DOM_CAMERA = 0, O_DOM_SCATTER = 1, O_DOM_FRESNEL = 2, O_DOM_NEE = 3, O_DOM_VOL = 4, O_DOM_VOL_SH_AREA = 5,
       O_DOM_VOL_SH_HDRI = 6 };
#define O_MAX_TRIES 64

double oracle_rng_uniform(uint32_t seed, uint32_t pixel, uint32_t sample, uint32_t counter) {
  return (double)(o_draw(o_path_key(seed, pixel, sample), counter) >> 8) * 0x1p-24;
}

/* ------------------------------------------------------------ prepared scene (fp64) */
typedef struct {
  const rt_scene_desc* d;
  unsigned char* is_top;
  int* vol_id;
  int nvol;
  int env_valid, env_use_is, env_w, env_h;
  double env_rotation, env_total_power;
  const double* env_rgb;
  double *env_pdf, *env_marg, *env_cond;
} OScene;

/* HDRIEnvironment.BuildDistribution hdri.go:145-224 */
static double build_distribution(const double* rgb, int W, int H, double* pdf, double* marg, double* cond) {
  double total = 0;
  double* rows = (double*)calloc((size_t)H, sizeof(double));
  for (int y = 0; y < H; ++y) {
    double v = ((double)y + 0.5) / (double)H;
    double theta = (0.5 - v) * M_PI;
    double st = cos(theta);
    if (cond) cond[(size_t)y * (W + 1)] = 0;
    for (int x = 0; x < W; ++x) {
      size_t idx = (size_t)y * W + x;
      const double* c = rgb + idx * 3;
      double lum = 0.2126 * c[0] + 0.7152 * c[1] + 0.0722 * c[2];
      double w = lum * st;
      if (w < 0) w = 0;
      if (pdf) pdf[idx] = w;
      rows[y] += w;
      total += w;
      if (cond) cond[(size_t)y * (W + 1) + x + 1] = cond[(size_t)y * (W + 1) + x] + w;
    }
  }
  if (cond)
    for (int y = 0; y < H; ++y)
      if (rows[y] > 0)
        for (int x = 0; x <= W; ++x) cond[(size_t)y * (W + 1) + x] /= rows[y];
  if (marg) {
    marg[0] = 0;
    for (int y = 0; y < H; ++y) marg[y + 1] = marg[y] + rows[y];
  }
  if (total > 0) {
    if (marg) for (int y = 0; y <= H; ++y) marg[y] /= total;
    if (pdf) for (size_t i = 0; i < (size_t)W * H; ++i) pdf[i] /= total;
  }
  free(rows);
  return total;
}

double oracle_hdri_total_power(const double* rgb, int32_t width, int32_t height) {
  return build_distribution(rgb, width, height, NULL, NULL, NULL);
}

static void mark_top(OScene* os, int g) {
  const rt_hittable* h = &os->d->hittables[g];
  if (h->kind == RT_BVH_NODE) {
    mark_top(os, h->a);
    if (h->b != h->a) mark_top(os, h->b);
  } else if (h->kind == RT_BVH_LEAF) {
    for (int i = 0; i < h->b; ++i) os->is_top[os->d->children[h->a + i]] = 1;
  } else {
    os->is_top[g] = 1;
  }
}

static int oscene_init(OScene* os, const rt_scene_desc* d) {
  memset(os, 0, sizeof(*os));
  if (!d || d->num_hittables <= 0 || d->root < 0 || d->root >= d->num_hittables) return RT_ERR_INVALID;
  os->d = d;
  os->is_top = (unsigned char*)calloc((size_t)d->num_hittables, 1);
  os->vol_id = (int*)malloc(sizeof(int) * (size_t)d->num_hittables);
  for (int i = 0; i < d->num_hittables; ++i) {
    os->vol_id[i] = -1;
    if (d->hittables[i].kind == RT_VOLUME) os->vol_id[i] = os->nvol++;
  }
  const rt_hittable* r = &d->hittables[d->root];
  if (r->kind == RT_LIST) {
    for (int i = 0; i < r->b; ++i) os->is_top[d->children[r->a + i]] = 1;
  } else {
    mark_top(os, d->root);
  }
  const rt_environment* e = d->environment;
  if (e && e->rgb && e->width > 0 && e->height > 0) {
    os->env_valid = 1;
    os->env_w = e->width;
    os->env_h = e->height;
    os->env_rgb = e->rgb;
    os->env_rotation = e->rotation;
    os->env_use_is = e->use_importance_sampling != 0;
    if (os->env_use_is) {
      size_t n = (size_t)e->width * e->height;
      os->env_pdf = (double*)malloc(n * sizeof(double));
      os->env_marg = (double*)malloc(((size_t)e->height + 1) * sizeof(double));
      os->env_cond = (double*)malloc((size_t)e->height * (e->width + 1) * sizeof(double));
      os->env_total_power = build_distribution(e->rgb, e->width, e->height, os->env_pdf, os->env_marg, os->env_cond);
    }
  }
  return 0;
}

static void oscene_free(OScene* os) {
  free(os->is_top); free(os->vol_id); free(os->env_pdf); free(os->env_marg); free(os->env_cond);
}

/* ------------------------------------------------------------ fp64 instantiation */
#define REAL double
#define SUF _d
#define SQRT sqrt
#define FABS fabs
#define LOG log
#define COS cos
#define SIN sin
#define ATAN2 atan2
#define ASIN asin
#define ACOS acos
#define FLOOR floor
#define POW5(x) pow((x), 5.0)
#define PI_R M_PI
#define UNITVEC_LO 1e-160
#define BOX_LO(x) (x)
#define BOX_HI(x) (x)
#define TRI_P_BARY 0
#include "oracle_impl.h"
#undef REAL
#undef SUF
#undef SQRT
#undef FABS
#undef LOG
#undef COS
#undef SIN
#undef ATAN2
#undef ASIN
#undef ACOS
#undef FLOOR
#undef POW5
#undef PI_R
#undef UNITVEC_LO
#undef BOX_LO
#undef BOX_HI
#undef TRI_P_BARY

/* ------------------------------------------------------------ fp32 instantiation */
static inline float o_pow5f(float x) { float x2 = x * x; return (x2 * x2) * x; }
/* ln(x) of the volume free flight (volume.go:66) in fp32 mode: the device's
 * libm-free algorithm (device_common.h rt_logf), restated so both sides give
 * the same bits: x = m*2^e, m in [sqrt(1/2), sqrt(2)),
 * ln m = f - f^2/2 + s*(f^2/2 + R(s^2)), f = m-1, s = f/(2+f) (fdlibm's form,
 * series to s^9), e*ln2 split hi/lo.  x <= 0 -> -inf. */
static inline float o_logf(float x) {
  if (!(x > 0.0f)) return -INFINITY;
  uint32_t b;
  memcpy(&b, &x, 4);
  int e = (int)(b >> 23) - 127;
  uint32_t mb = (b & 0x7FFFFFu) | 0x3F800000u;
  float m;
  memcpy(&m, &mb, 4);
  if (m > 1.41421356f) { m = m * 0.5f; e += 1; }
  const float f = m - 1.0f;
  const float hfsq = 0.5f * f * f;
  const float s = f / (2.0f + f);
  const float z = s * s;
  const float R = z * (0.666666687f + z * (0.400000006f + z * (0.285714298f + z * 0.222222224f)));
  const float fe = (float)e;
  return fe * 0.693145752f - ((hfsq - (s * (hfsq + R) + fe * 1.42860677e-06f)) - f);
}
void oracle_logf32(const float* in, float* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) out[i] = o_logf(in[i]);
}
static inline float o_round_down(double x) {
  float f = (float)x;
  if (isfinite(x) && (double)f > x) f = nextafterf(f, -INFINITY);
  return f;
}
static inline float o_round_up(double x) {
  float f = (float)x;
  if (isfinite(x) && (double)f < x) f = nextafterf(f, INFINITY);
  return f;
}
#define REAL float
#define SUF _f
#define SQRT sqrtf
#define FABS fabsf
#define LOG o_logf
#define COS cosf
#define SIN sinf
#define ATAN2 atan2f
#define ASIN asinf
#define ACOS acosf
#define FLOOR floorf
#define POW5(x) o_pow5f(x)
#define PI_R 3.14159265358979323846f
#define UNITVEC_LO 0.0f
#define BOX_LO(x) o_round_down(x)
#define BOX_HI(x) o_round_up(x)
#define TRI_P_BARY 1
#include "oracle_impl.h"

/* ------------------------------------------------------------ public API */
static void default_buckets(int W, int H, rt_bucket** out, int* n) {   /* generateBuckets */
  int bs = 32, cnt = 0;
  for (int y = 0; y < H; y += bs)
    for (int x = 0; x < W; x += bs) cnt++;
  rt_bucket* b = (rt_bucket*)malloc(sizeof(rt_bucket) * (size_t)cnt);
  int k = 0;
  for (int y = 0; y < H; y += bs)
    for (int x = 0; x < W; x += bs) {
      b[k].x = x; b[k].y = y;
      b[k].width = W - x < bs ? W - x : bs;
      b[k].height = H - y < bs ? H - y : bs;
      k++;
    }
  *out = b;
  *n = cnt;
}

int oracle_render(const rt_scene_desc* scene, const rt_camera_desc* cam, const rt_render_params* p, int fp32,
                  int nthreads, double* accum) {
  if (!scene || !cam || !p || !accum) return RT_ERR_INVALID;
  OScene os;
  int rc = oscene_init(&os, scene);
  if (rc) return rc;
  rt_bucket* own = NULL;
  const rt_bucket* bk = p->buckets;
  int nb = p->num_buckets;
  if (!bk) { default_buckets(cam->image_width, cam->image_height, &own, &nb); bk = own; }
  rc = fp32 ? render_f(&os, cam, p, nthreads, bk, nb, accum) : render_d(&os, cam, p, nthreads, bk, nb, accum);
  free(own);
  oscene_free(&os);
  return rc;
}

int oracle_primary_hits(const rt_scene_desc* scene, const rt_camera_desc* cam, uint32_t seed, int32_t sample, int fp32,
                        int32_t* top, int32_t* prim, double* t) {
  if (!scene || !cam || !top || !prim || !t) return RT_ERR_INVALID;
  OScene os;
  int rc = oscene_init(&os, scene);
  if (rc) return rc;
  rc = fp32 ? primary_f(&os, cam, seed, sample, top, prim, t) : primary_d(&os, cam, seed, sample, top, prim, t);
  oscene_free(&os);
  return rc;
}

int oracle_path_records(const rt_scene_desc* scene, const rt_camera_desc* cam, uint32_t seed, int32_t sample,
                        int32_t num_bounces, int fp32, int nthreads, int32_t* top, int32_t* prim, double* t,
                        double* ray, int32_t* nee) {
  if (!scene || !cam || !top || !prim || !t || !ray || !nee || num_bounces <= 0) return RT_ERR_INVALID;
  const size_t n = (size_t)cam->image_width * (size_t)cam->image_height * (size_t)num_bounces;
  for (size_t i = 0; i < n; ++i) {
    top[i] = prim[i] = -2;
    t[i] = -1.0;
    nee[i] = 0;
  }
  memset(ray, 0, n * 6 * sizeof(double));
  OScene os;
  int rc = oscene_init(&os, scene);
  if (rc) return rc;
  rc = fp32 ? paths_f(&os, cam, seed, sample, num_bounces, nthreads, top, prim, t, ray, nee)
            : paths_d(&os, cam, seed, sample, num_bounces, nthreads, top, prim, t, ray, nee);
  oscene_free(&os);
  return rc;
}

void oracle_tonemap(const float* accum, int64_t npix, int32_t spp, uint8_t* rgba) {   /* bucket_renderer.go:276-285 */
  double sc = 1.0 / (double)spp;
  for (int64_t i = 0; i < npix; ++i) {
    for (int c = 0; c < 3; ++c) {
      double v = (double)accum[i * 3 + c] * sc;
      double g = v > 0 ? sqrt(v) : 0;                  /* LinearToGamma utils.go:85-90 */
      if (g < 0.0) g = 0.0;                            /* Interval{0,0.999}.Clamp */
      if (g > 0.999) g = 0.999;
      rgba[i * 4 + c] = (uint8_t)(256 * g);
    }
    rgba[i * 4 + 3] = 255;
  }
}

/* ------------------------------------------------------------ NewBVHNode (bvh.go:69-217) */
typedef struct { int index; double box[6]; double c[3]; } OPrim;

static void pad_box(double* b) {                       /* padToMinimums aabb.go:117-128 */
  for (int a = 0; a < 3; ++a)
    if (b[2 * a + 1] - b[2 * a] < 0.0001) { b[2 * a] -= 0.0001; b[2 * a + 1] += 0.0001; }
}
static void union_box(double* a, const double* b) {    /* NewAABBFromBoxes */
  for (int k = 0; k < 3; ++k) {
    if (b[2 * k] < a[2 * k]) a[2 * k] = b[2 * k];
    if (b[2 * k + 1] > a[2 * k + 1]) a[2 * k + 1] = b[2 * k + 1];
  }
}
static int g_axis;
static int prim_less(const OPrim* x, const OPrim* y) {
  double a = x->c[g_axis], b = y->c[g_axis];
  if (isnan(a) || isnan(b)) return isnan(a) && !isnan(b);
  return a < b;
}
/* stable merge sort (ties keep input order; NaN first) */
static void msort(OPrim* v, OPrim* tmp, int n) {
  if (n < 2) return;
  int m = n / 2;
  msort(v, tmp, m);
  msort(v + m, tmp, n - m);
  int i = 0, j = m, k = 0;
  while (i < m && j < n) tmp[k++] = prim_less(&v[j], &v[i]) ? v[j++] : v[i++];
  while (i < m) tmp[k++] = v[i++];
  while (j < n) tmp[k++] = v[j++];
  memcpy(v, tmp, sizeof(OPrim) * (size_t)n);
}
static int bvh_rec(OPrim* p, OPrim* tmp, int n, int32_t* out, int len, int cap) {
  double cb[6];
  for (int a = 0; a < 3; ++a) { cb[2 * a] = p[0].c[a]; cb[2 * a + 1] = p[0].c[a]; }
  pad_box(cb);
  for (int i = 1; i < n; ++i) {
    double q[6];
    for (int a = 0; a < 3; ++a) { q[2 * a] = fmin(p[i].c[a], p[i].c[a]); q[2 * a + 1] = q[2 * a]; }
    pad_box(q);
    union_box(cb, q);
  }
  if (n <= 4) {
    if (len + 1 + n > cap) return -1;
    out[len++] = n;
    for (int i = 0; i < n; ++i) out[len++] = p[i].index;
    return len;
  }
  double xs = cb[1] - cb[0], ys = cb[3] - cb[2], zs = cb[5] - cb[4];   /* LongestAxis aabb.go:139-150 */
  g_axis = (xs > ys && xs > zs) ? 0 : (ys > zs ? 1 : 2);
  msort(p, tmp, n);
  if (len + 1 > cap) return -1;
  out[len++] = -1;
  int m = n / 2;
  len = bvh_rec(p, tmp, m, out, len, cap);
  if (len < 0) return -1;
  return bvh_rec(p + m, tmp, n - m, out, len, cap);
}
int oracle_build_bvh(const double* boxes, int32_t n, int32_t* out, int32_t cap) {
  if (n <= 0) return 0;
  OPrim* p = (OPrim*)malloc(sizeof(OPrim) * (size_t)n);
  OPrim* tmp = (OPrim*)malloc(sizeof(OPrim) * (size_t)n);
  for (int i = 0; i < n; ++i) {
    p[i].index = i;
    memcpy(p[i].box, boxes + (size_t)i * 6, sizeof(double) * 6);
    for (int a = 0; a < 3; ++a) p[i].c[a] = (p[i].box[2 * a] + p[i].box[2 * a + 1]) * 0.5;   /* Centroid */
  }
  int r = bvh_rec(p, tmp, n, out, 0, cap);
  free(p);
  free(tmp);
  return r;
}

/* ------------------------------------------------------------ LoadHDR (image_loader.go:165-383) */
int oracle_load_hdr(const char* path, int32_t* width, int32_t* height, double* rgb, int64_t cap) {
  FILE* f = fopen(path, "rb");
  if (!f) return RT_ERR_INVALID;
  char line[512];
  if (!fgets(line, sizeof line, f) || strncmp(line, "#?", 2) != 0) { fclose(f); return RT_ERR_INVALID; }
  for (;;) {
    if (!fgets(line, sizeof line, f)) { fclose(f); return RT_ERR_INVALID; }
    char* s = line;
    while (*s == ' ' || *s == '\t' || *s == '\r' || *s == '\n') s++;
    if (*s == 0) break;
  }
  if (!fgets(line, sizeof line, f)) { fclose(f); return RT_ERR_INVALID; }
  char a0[8], a2[8];
  long n1, n3;
  if (sscanf(line, "%7s %ld %7s %ld", a0, &n1, a2, &n3) != 4) { fclose(f); return RT_ERR_INVALID; }
  int W, H;
  if (!strcmp(a0, "-Y") && !strcmp(a2, "+X")) { H = (int)n1; W = (int)n3; }
  else if (!strcmp(a0, "+X") && !strcmp(a2, "-Y")) { W = (int)n1; H = (int)n3; }
  else { fclose(f); return RT_ERR_INVALID; }
  if (width) *width = W;
  if (height) *height = H;
  if (!rgb) { fclose(f); return 0; }
  if (cap < (int64_t)W * H * 3) { fclose(f); return RT_ERR_INVALID; }
  unsigned char* comp = (unsigned char*)malloc((size_t)W * 4);
  int rc = 0;
  for (int y = 0; y < H && !rc; ++y) {
    unsigned char hd[4];
    if (fread(hd, 1, 4, f) != 4) { rc = RT_ERR_INVALID; break; }
    unsigned char* pix[1];
    (void)pix;
    if (hd[0] == 2 && hd[1] == 2) {
      if (((hd[2] << 8) | hd[3]) != W) { rc = RT_ERR_INVALID; break; }
      for (int c = 0; c < 4 && !rc; ++c) {
        int x = 0;
        while (x < W) {
          int code = fgetc(f);
          if (code == EOF) { rc = RT_ERR_INVALID; break; }
          if (code > 128) {
            int cnt = code - 128, v = fgetc(f);
            if (v == EOF) { rc = RT_ERR_INVALID; break; }
            for (int i = 0; i < cnt && x < W; ++i) comp[(size_t)c * W + x++] = (unsigned char)v;
          } else {
            for (int i = 0; i < code && x < W; ++i) {
              int v = fgetc(f);
              if (v == EOF) { rc = RT_ERR_INVALID; break; }
              comp[(size_t)c * W + x++] = (unsigned char)v;
            }
            if (rc) break;
          }
        }
      }
      for (int x = 0; x < W && !rc; ++x) {
        unsigned char q[4] = {comp[x], comp[W + x], comp[2 * W + x], comp[3 * W + x]};
        double* o = rgb + ((size_t)y * W + x) * 3;
        if (q[3] == 0) { o[0] = o[1] = o[2] = 0; continue; }
        double sc = ldexp(1.0, (int)q[3] - 128 - 8);
        o[0] = ((double)q[0] + 0.5) * sc; o[1] = ((double)q[1] + 0.5) * sc; o[2] = ((double)q[2] + 0.5) * sc;
      }
    } else {
      for (int x = 0; x < W; ++x) {
        unsigned char q[4];
        if (x == 0) memcpy(q, hd, 4);
        else if (fread(q, 1, 4, f) != 4) { rc = RT_ERR_INVALID; break; }
        double* o = rgb + ((size_t)y * W + x) * 3;
        if (q[3] == 0) { o[0] = o[1] = o[2] = 0; continue; }
        double sc = ldexp(1.0, (int)q[3] - 128 - 8);
        o[0] = ((double)q[0] + 0.5) * sc; o[1] = ((double)q[1] + 0.5) * sc; o[2] = ((double)q[2] + 0.5) * sc;
      }
    }
  }
  free(comp);
  fclose(f);
  return rc;
}
