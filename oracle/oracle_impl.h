/*
 * oracle_impl.h — body of the oracle, included twice by oracle.c:
 *   REAL=double, SUF=_d  : the reference's float64 arithmetic
 *   REAL=float,  SUF=_f  : operation-for-operation mirror of render.hip
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Every function names the Go code it restates.
 */
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)
#define FN(n) CAT(n, SUF)

typedef struct { REAL x, y, z; } FN(V3);
#define V3R FN(V3)

static inline V3R FN(mk)(REAL x, REAL y, REAL z) { V3R r; r.x = x; r.y = y; r.z = z; return r; }
/* vec3.go:21-38 */
static inline V3R FN(add)(V3R a, V3R b) { return FN(mk)(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3R FN(sub)(V3R a, V3R b) { return FN(mk)(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V3R FN(mul)(V3R a, V3R b) { return FN(mk)(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline V3R FN(scale)(V3R v, REAL t) { return FN(mk)(t * v.x, t * v.y, t * v.z); }
static inline V3R FN(divs)(V3R v, REAL t) { return FN(scale)(v, (REAL)1 / t); }
static inline V3R FN(neg)(V3R v) { return FN(mk)(-v.x, -v.y, -v.z); }
static inline REAL FN(dot)(V3R a, V3R b) { return a.x * b.x + a.y * b.y + a.z * b.z; }     /* vec3.go:77-79 */
static inline V3R FN(cross)(V3R a, V3R b) {                                              /* vec3.go:81-87 */
  return FN(mk)(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline REAL FN(len2)(V3R v) { return v.x * v.x + v.y * v.y + v.z * v.z; }
static inline REAL FN(len)(V3R v) { return SQRT(FN(len2)(v)); }
static inline V3R FN(unit)(V3R v) { REAL l = FN(len)(v); if (l == 0) return v; return FN(divs)(v, l); } /* vec3.go:30-36 */
static inline int FN(near_zero)(V3R v) {                                                  /* vec3.go:38-41 */
  const REAL s = (REAL)1e-8;
  return FABS(v.x) < s && FABS(v.y) < s && FABS(v.z) < s;
}
static inline V3R FN(reflect)(V3R v, V3R n) { return FN(sub)(v, FN(scale)(n, 2 * FN(dot)(v, n))); } /* :104-106 */
static inline REAL FN(gomin)(REAL x, REAL y) { return !(x >= y) ? x : y; }               /* math.Min */
static inline V3R FN(refract)(V3R uv, V3R n, REAL eta) {                                  /* vec3.go:108-115 */
  REAL c = FN(dot)(FN(neg)(uv), n);
  REAL ct = c < 1 ? c : 1;
  V3R perp = FN(scale)(FN(add)(uv, FN(scale)(n, ct)), eta);
  V3R par = FN(scale)(n, -SQRT(FABS(1 - FN(len2)(perp))));
  return FN(add)(perp, par);
}
static inline V3R FN(ld3)(const REAL* p) { return FN(mk)(p[0], p[1], p[2]); }

/* ------------------------------------------------------------ scene copy */
typedef struct {
  REAL p[16];
  REAL box[6];
} FN(HR);

typedef struct {
  const OScene* os;
  FN(HR)* h;                     /* per hittable, REAL copies */
  REAL* env_tex;                 /* W*H*3 */
  REAL* env_pdf;
  REAL* env_marg;
  REAL* env_cond;
  REAL env_rot;
  REAL cam_center[3], cam_p00[3], cam_du[3], cam_dv[3], cam_disk_u[3], cam_disk_v[3], cam_bg[3];
  int cam_defocus, cam_sky, cam_phantom, cam_max_depth;
  int cam_slow, cam_free, cam_w, cam_h;                          /* GetRay slow path (camera.go:390-434) */
  REAL cam_corig[3], cam_cdir[3], cam_laorig[3], cam_ladir[3], cam_vup[3], cam_fwd[3];
  REAL cam_vw, cam_vh, cam_focus, cam_rad;
} FN(OS);

static int FN(prep)(FN(OS)* S, const OScene* os, const rt_camera_desc* cam) {
  const rt_scene_desc* d = os->d;
  memset(S, 0, sizeof(*S));
  S->os = os;
  S->h = (FN(HR)*)calloc((size_t)d->num_hittables, sizeof(FN(HR)));
  if (!S->h) return RT_ERR_OOM;
  for (int i = 0; i < d->num_hittables; ++i) {
    for (int k = 0; k < 16; ++k) S->h[i].p[k] = (REAL)d->hittables[i].p[k];
    for (int a = 0; a < 3; ++a) {
      S->h[i].box[2 * a] = BOX_LO(d->hittables[i].bbox[2 * a]);
      S->h[i].box[2 * a + 1] = BOX_HI(d->hittables[i].bbox[2 * a + 1]);
    }
  }
  if (os->env_valid) {
    size_t n = (size_t)os->env_w * os->env_h;
    S->env_tex = (REAL*)malloc(n * 3 * sizeof(REAL));
    for (size_t i = 0; i < n * 3; ++i) S->env_tex[i] = (REAL)os->env_rgb[i];
    S->env_rot = (REAL)os->env_rotation;
    if (os->env_use_is) {
      S->env_pdf = (REAL*)malloc(n * sizeof(REAL));
      S->env_marg = (REAL*)malloc(((size_t)os->env_h + 1) * sizeof(REAL));
      S->env_cond = (REAL*)malloc((size_t)os->env_h * (os->env_w + 1) * sizeof(REAL));
      for (size_t i = 0; i < n; ++i) S->env_pdf[i] = (REAL)os->env_pdf[i];
      for (int i = 0; i <= os->env_h; ++i) S->env_marg[i] = (REAL)os->env_marg[i];
      for (size_t i = 0; i < (size_t)os->env_h * (os->env_w + 1); ++i) S->env_cond[i] = (REAL)os->env_cond[i];
    }
  }
  for (int a = 0; a < 3; ++a) {
    S->cam_center[a] = (REAL)cam->center[a];
    S->cam_p00[a] = (REAL)cam->pixel00[a];
    S->cam_du[a] = (REAL)cam->pixel_delta_u[a];
    S->cam_dv[a] = (REAL)cam->pixel_delta_v[a];
    S->cam_disk_u[a] = (REAL)cam->defocus_disk_u[a];
    S->cam_disk_v[a] = (REAL)cam->defocus_disk_v[a];
    S->cam_bg[a] = (REAL)cam->background[a];
  }
  S->cam_defocus = cam->defocus_angle > 0;
  S->cam_sky = cam->use_sky_gradient != 0;
  S->cam_phantom = cam->phantom_hdri != 0;
  S->cam_max_depth = cam->max_depth;
  S->cam_slow = cam->camera_motion || cam->free_camera;
  S->cam_free = cam->free_camera != 0;
  S->cam_w = cam->image_width;
  S->cam_h = cam->image_height;
  for (int a = 0; a < 3; ++a) {
    S->cam_corig[a] = (REAL)cam->center_motion_orig[a];
    S->cam_cdir[a] = (REAL)cam->center_motion_dir[a];
    S->cam_laorig[a] = (REAL)cam->look_at_motion_orig[a];
    S->cam_ladir[a] = (REAL)cam->look_at_motion_dir[a];
    S->cam_vup[a] = (REAL)cam->vup[a];
    S->cam_fwd[a] = (REAL)cam->forward[a];
  }
  S->cam_vw = (REAL)cam->viewport_width;
  S->cam_vh = (REAL)cam->viewport_height;
  S->cam_focus = (REAL)cam->focus_dist;
  S->cam_rad = (REAL)cam->defocus_radius;
  return 0;
}

static void FN(unprep)(FN(OS)* S) {
  free(S->h); free(S->env_tex); free(S->env_pdf); free(S->env_marg); free(S->env_cond);
}

/* ------------------------------------------------------------ per-thread ctx */
typedef struct {
  const FN(OS)* S;
  uint32_t key;
  uint32_t bounce;
  uint32_t voldom;
  int* volcount;                 /* per vol_id Hit-call counter for this traversal */
  /* path recorder (oracle_path_records; NULL r_top: off): per bounce b < r_nb,
   * element b * r_npix + r_pix */
  int32_t* r_top;
  int32_t* r_prim;
  double* r_t;
  double* r_ray;                 /* 6 per element: incoming ray o, d */
  int32_t* r_nee;                /* bits 0/1 area/HDRI shadow ray traced, 2/3 unoccluded */
  int r_nb;
  size_t r_npix, r_pix;
} FN(TC);

static inline REAL FN(rnd)(const FN(TC)* c, uint32_t dom, uint32_t idx) {
  return (REAL)((double)(o_draw(c->key, o_ctr(c->bounce, dom, idx)) >> 8) * 0x1p-24);
}

/* RandomUnitVector vec3.go:45-54 (rejection in the cube). */
static V3R FN(random_unit_vector)(const FN(TC)* c, uint32_t dom, uint32_t base) {
  for (int k = 0; k < O_MAX_TRIES; ++k) {
    uint32_t i = base + 3u * (uint32_t)k;
    V3R p = FN(mk)(-1 + 2 * FN(rnd)(c, dom, i), -1 + 2 * FN(rnd)(c, dom, i + 1), -1 + 2 * FN(rnd)(c, dom, i + 2));
    REAL l2 = FN(len2)(p);
    if (UNITVEC_LO < l2 && l2 <= 1) return FN(divs)(p, SQRT(l2));
  }
  return FN(mk)(0, 0, 1);
}

typedef struct {
  V3R P, N;
  int mat;
  REAL t;
  int front;
  int top, prim;
  REAL u, v;                     /* HitRecord.U/V (kept from earlier hits where a Hit leaves them) */
} FN(Rec);

typedef struct { V3R o, d; REAL tm; } FN(Ray);

static inline V3R FN(at)(FN(Ray) r, REAL t) { return FN(add)(r.o, FN(scale)(r.d, t)); }   /* ray.go:19-21 */

static inline void FN(set_face)(FN(Rec)* rec, FN(Ray) r, V3R out) {                      /* hittable.go:20-30 */
  rec->front = FN(dot)(r.d, out) < 0;
  rec->N = rec->front ? out : FN(neg)(out);
}

/* AABB.Hit aabb.go:59-116 */
static int FN(aabb_hit)(const REAL* b, FN(Ray) r, REAL mn, REAL mx) {
  const REAL o[3] = {r.o.x, r.o.y, r.o.z}, dd[3] = {r.d.x, r.d.y, r.d.z};
  for (int a = 0; a < 3; ++a) {
    REAL adinv = (REAL)1 / dd[a];
    REAL t0 = (b[2 * a] - o[a]) * adinv;
    REAL t1 = (b[2 * a + 1] - o[a]) * adinv;
    if (adinv < 0) { REAL s = t0; t0 = t1; t1 = s; }
    if (t0 > mn) mn = t0;
    if (t1 < mx) mx = t1;
    if (mx <= mn) return 0;
  }
  return 1;
}

static int FN(hit)(FN(TC)* c, int g, FN(Ray) r, REAL mn, REAL mx, FN(Rec)* rec);

/* Sphere.Hit sphere.go:63-94 */
static int FN(sphere_hit)(FN(TC)* c, int g, FN(Ray) r, REAL mn, REAL mx, FN(Rec)* rec) {
  const REAL* p = c->S->h[g].p;
  V3R center = FN(add)(FN(mk)(p[0], p[1], p[2]), FN(scale)(FN(mk)(p[3], p[4], p[5]), r.tm));
  V3R oc = FN(sub)(center, r.o);
  REAL a = FN(len2)(r.d);
  REAL h = FN(dot)(r.d, oc);
  REAL cc = FN(len2)(oc) - p[6] * p[6];
  REAL disc = h * h - a * cc;
  if (disc < 0) return 0;
  REAL sq = SQRT(disc);
  REAL root = (h - sq) / a;
  if (!(mn < root && root < mx)) {
    root = (h + sq) / a;
    if (!(mn < root && root < mx)) return 0;
  }
  rec->t = root;
  rec->P = FN(at)(r, root);
  V3R outward = FN(divs)(FN(sub)(rec->P, center), p[6]);
  FN(set_face)(rec, r, outward);
  rec->u = (ATAN2(-outward.z, outward.x) + PI_R) / (2 * PI_R);   /* getSphereUV sphere.go:53-59 */
  rec->v = ACOS(-outward.y) / PI_R;
  rec->mat = c->S->os->d->hittables[g].material;
  rec->prim = g;
  return 1;
}

/* Quad.Hit quad.go:44-84 */
static int FN(quad_hit)(FN(TC)* c, int g, FN(Ray) r, REAL mn, REAL mx, FN(Rec)* rec) {
  const REAL* p = c->S->h[g].p;
  V3R n = FN(mk)(p[12], p[13], p[14]);
  REAL denom = FN(dot)(n, r.d);
  if (FABS(denom) < (REAL)1e-8) return 0;
  REAL t = (p[15] - FN(dot)(n, r.o)) / denom;
  if (!(mn <= t && t <= mx)) return 0;
  V3R P = FN(at)(r, t);
  V3R ph = FN(sub)(P, FN(mk)(p[0], p[1], p[2]));
  V3R w = FN(mk)(p[9], p[10], p[11]);
  REAL alpha = FN(dot)(w, FN(cross)(ph, FN(mk)(p[6], p[7], p[8])));
  REAL beta = FN(dot)(w, FN(cross)(FN(mk)(p[3], p[4], p[5]), ph));
  if (!(0 <= alpha && alpha <= 1) || !(0 <= beta && beta <= 1)) return 0;
  rec->t = t;
  rec->P = P;
  rec->u = alpha;                                                /* quad.go:81-82 */
  rec->v = beta;
  rec->mat = c->S->os->d->hittables[g].material;
  FN(set_face)(rec, r, n);
  rec->prim = g;
  return 1;
}

/* Triangle.Hit triangle.go:57-104 */
static int FN(tri_hit)(FN(TC)* c, int g, FN(Ray) r, REAL mn, REAL mx, FN(Rec)* rec) {
  const REAL* p = c->S->h[g].p;
  V3R v0 = FN(mk)(p[0], p[1], p[2]);
  V3R e1 = FN(sub)(FN(mk)(p[3], p[4], p[5]), v0);
  V3R e2 = FN(sub)(FN(mk)(p[6], p[7], p[8]), v0);
  V3R h = FN(cross)(r.d, e2);
  REAL a = FN(dot)(e1, h);
  if (FABS(a) < (REAL)1e-8) return 0;
  REAL f = (REAL)1 / a;
  V3R s = FN(sub)(r.o, v0);
  REAL u = f * FN(dot)(s, h);
  if (u < 0 || u > 1) return 0;
  V3R q = FN(cross)(s, e1);
  REAL v = f * FN(dot)(r.d, q);
  if (v < 0 || u + v > 1) return 0;
  REAL t = f * FN(dot)(e2, q);
  if (!(mn <= t && t <= mx)) return 0;
  rec->t = t;
  /* triangle.go:97 r.At(t); the fp32 mode takes v0 + u*e1 + v*e2 like the
   * device (make_record), which removes fp32's self-intersection bias
   * (DESIGN.md §5); in float64 the two agree to ~1e-13. */
  rec->P = TRI_P_BARY ? FN(add)(v0, FN(add)(FN(scale)(e1, u), FN(scale)(e2, v))) : FN(at)(r, t);
  rec->u = u;                                                    /* triangle.go:100-101 */
  rec->v = v;
  rec->mat = c->S->os->d->hittables[g].material;
  FN(set_face)(rec, r, FN(mk)(p[9], p[10], p[11]));
  rec->prim = g;
  return 1;
}

/* Circle.Hit circle.go:37-72 */
static int FN(circle_hit)(FN(TC)* c, int g, FN(Ray) r, REAL mn, REAL mx, FN(Rec)* rec) {
  const REAL* p = c->S->h[g].p;
  V3R n = FN(mk)(p[3], p[4], p[5]);
  REAL denom = FN(dot)(n, r.d);
  if (FABS(denom) < (REAL)1e-8) return 0;
  REAL t = (p[7] - FN(dot)(n, r.o)) / denom;
  if (!(mn <= t && t <= mx)) return 0;
  V3R P = FN(at)(r, t);
  V3R ctr = FN(mk)(p[0], p[1], p[2]);
  if (FN(len)(FN(sub)(P, ctr)) > p[6]) return 0;
  rec->t = t;
  rec->P = P;
  rec->mat = c->S->os->d->hittables[g].material;
  FN(set_face)(rec, r, n);
  V3R bu = FN(unit)(FN(cross)(FABS(n.y) > (REAL)0.9 ? FN(mk)(1, 0, 0) : FN(mk)(0, 1, 0), n));
  V3R bv = FN(cross)(n, bu);
  V3R lp = FN(sub)(P, ctr);
  rec->u = (FN(dot)(lp, bu) / p[6] + 1) * (REAL)0.5;
  rec->v = (FN(dot)(lp, bv) / p[6] + 1) * (REAL)0.5;
  rec->prim = g;
  return 1;
}

/* Plane.Hit plane.go:24-42 */
static int FN(plane_hit)(FN(TC)* c, int g, FN(Ray) r, REAL mn, REAL mx, FN(Rec)* rec) {
  const REAL* p = c->S->h[g].p;
  V3R n = FN(mk)(p[3], p[4], p[5]);
  REAL denom = FN(dot)(n, r.d);
  if (FABS(denom) < (REAL)1e-8) return 0;
  REAL t = FN(dot)(FN(sub)(FN(mk)(p[0], p[1], p[2]), r.o), n) / denom;
  if (!(mn < t && t < mx)) return 0;
  rec->t = t;
  rec->P = FN(at)(r, t);
  FN(set_face)(rec, r, n);
  rec->mat = c->S->os->d->hittables[g].material;
  rec->prim = g;
  return 1;
}

/* Volume.Hit volume.go:34-79 */
static int FN(volume_hit)(FN(TC)* c, int g, FN(Ray) r, REAL mn, REAL mx, FN(Rec)* rec) {
  const rt_hittable* hh = &c->S->os->d->hittables[g];
  FN(Rec) r1, r2;
  memset(&r1, 0, sizeof(r1));
  memset(&r2, 0, sizeof(r2));
  if (!FN(hit)(c, hh->a, r, -(REAL)INFINITY, (REAL)INFINITY, &r1)) return 0;
  if (!FN(hit)(c, hh->a, r, r1.t + (REAL)0.0001, (REAL)INFINITY, &r2)) return 0;
  if (r1.t < mn) r1.t = mn;
  if (r2.t > mx) r2.t = mx;
  if (r1.t >= r2.t) return 0;
  if (r1.t < 0) r1.t = 0;
  REAL rl = FN(len)(r.d);
  REAL dist = (r2.t - r1.t) * rl;
  int vid = c->S->os->vol_id[g];
  int k = c->volcount[vid]++;
  if (k > 3) k = 3;
  REAL u = FN(rnd)(c, c->voldom, (uint32_t)vid * 4u + (uint32_t)k);
  REAL hd = c->S->h[g].p[0] * LOG(u);
  if (hd > dist) return 0;
  rec->t = r1.t + hd / rl;
  rec->P = FN(at)(r, rec->t);
  rec->N = FN(mk)(1, 0, 0);
  rec->front = 1;
  rec->mat = hh->material;
  rec->prim = g;
  return 1;
}

static int FN(hit)(FN(TC)* c, int g, FN(Ray) r, REAL mn, REAL mx, FN(Rec)* rec) {
  const OScene* os = c->S->os;
  const rt_hittable* h = &os->d->hittables[g];
  const int* ch = os->d->children;
  int ok = 0;
  switch (h->kind) {
    case RT_SPHERE: ok = FN(sphere_hit)(c, g, r, mn, mx, rec); break;
    case RT_QUAD: ok = FN(quad_hit)(c, g, r, mn, mx, rec); break;
    case RT_TRIANGLE: ok = FN(tri_hit)(c, g, r, mn, mx, rec); break;
    case RT_PLANE: ok = FN(plane_hit)(c, g, r, mn, mx, rec); break;
    case RT_CIRCLE: ok = FN(circle_hit)(c, g, r, mn, mx, rec); break;
    case RT_VOLUME: ok = FN(volume_hit)(c, g, r, mn, mx, rec); break;
    case RT_LIST: {                                   /* hittable_list.go:31-45 */
      FN(Rec) tmp;
      memset(&tmp, 0, sizeof(tmp));
      REAL closest = mx;
      for (int i = 0; i < h->b; ++i)
        if (FN(hit)(c, ch[h->a + i], r, mn, closest, &tmp)) { ok = 1; closest = tmp.t; *rec = tmp; }
      break;
    }
    case RT_BVH_LEAF: {                               /* bvh.go:26-37 */
      REAL closest = mx;
      for (int i = 0; i < h->b; ++i)
        if (FN(hit)(c, ch[h->a + i], r, mn, closest, rec)) { ok = 1; closest = rec->t; }
      break;
    }
    case RT_BVH_NODE: {                               /* bvh.go:219-239 */
      if (!FN(aabb_hit)(c->S->h[g].box, r, mn, mx)) return 0;
      int hl = FN(hit)(c, h->a, r, mn, mx, rec);
      REAL rmax = hl ? rec->t : mx;
      int hr = FN(hit)(c, h->b, r, mn, rmax, rec);
      ok = hl || hr;
      break;
    }
    case RT_TRANSLATE: {                              /* transform.go:93-102 */
      const REAL* p = c->S->h[g].p;
      FN(Ray) o = r;
      o.o = FN(sub)(r.o, FN(mk)(p[0], p[1], p[2]));
      if (!FN(hit)(c, h->a, o, mn, mx, rec)) return 0;
      rec->P = FN(add)(rec->P, FN(mk)(p[0], p[1], p[2]));
      ok = 1;
      break;
    }
    case RT_ROTATE_Y: {                               /* transform.go:159-187 */
      REAL s = c->S->h[g].p[0], cs = c->S->h[g].p[1];
      FN(Ray) o = r;
      o.o.x = cs * r.o.x - s * r.o.z; o.o.z = s * r.o.x + cs * r.o.z;
      o.d.x = cs * r.d.x - s * r.d.z; o.d.z = s * r.d.x + cs * r.d.z;
      if (!FN(hit)(c, h->a, o, mn, mx, rec)) return 0;
      V3R P = rec->P, N = rec->N;
      P.x = cs * rec->P.x + s * rec->P.z; P.z = -s * rec->P.x + cs * rec->P.z;
      N.x = cs * rec->N.x + s * rec->N.z; N.z = -s * rec->N.x + cs * rec->N.z;
      rec->P = P; rec->N = N;
      ok = 1;
      break;
    }
    case RT_ROTATE_X: {                               /* transform.go:229-263 (as written) */
      REAL s = c->S->h[g].p[0], cs = c->S->h[g].p[1];
      FN(Ray) o = r;
      o.o.y = cs * r.o.y - s * r.o.z; o.o.z = s * r.o.y + cs * r.o.z;
      o.d.y = cs * r.d.y - s * r.d.z; o.d.z = s * r.d.y + cs * r.d.z;
      if (!FN(hit)(c, h->a, o, mn, mx, rec)) return 0;
      V3R P = rec->P, N = rec->N;
      P.y = cs * rec->P.y - s * rec->P.z; P.z = s * rec->P.y + cs * rec->P.z;
      N.y = cs * rec->N.y - s * rec->N.z; N.z = s * rec->N.y + cs * rec->N.z;
      rec->P = P; rec->N = N;
      ok = 1;
      break;
    }
    case RT_ROTATE_Z: {                               /* transform.go:310-344 (as written) */
      REAL s = c->S->h[g].p[0], cs = c->S->h[g].p[1];
      FN(Ray) o = r;
      o.o.x = cs * r.o.x - s * r.o.y; o.o.y = s * r.o.x + cs * r.o.y;
      o.d.x = cs * r.d.x - s * r.d.y; o.d.y = s * r.d.x + cs * r.d.y;
      if (!FN(hit)(c, h->a, o, mn, mx, rec)) return 0;
      V3R P = rec->P, N = rec->N;
      P.x = cs * rec->P.x - s * rec->P.y; P.y = s * rec->P.x + cs * rec->P.y;
      N.x = cs * rec->N.x - s * rec->N.y; N.y = s * rec->N.x + cs * rec->N.y;
      rec->P = P; rec->N = N;
      ok = 1;
      break;
    }
    case RT_SCALE: {                                  /* transform.go:408-440 */
      const REAL* p = c->S->h[g].p;
      FN(Ray) o = r;
      o.o = FN(mk)(r.o.x * p[3], r.o.y * p[4], r.o.z * p[5]);
      o.d = FN(mk)(r.d.x * p[3], r.d.y * p[4], r.d.z * p[5]);
      if (!FN(hit)(c, h->a, o, mn, mx, rec)) return 0;
      rec->P = FN(mk)(rec->P.x * p[0], rec->P.y * p[1], rec->P.z * p[2]);
      rec->N = FN(unit)(FN(mk)(rec->N.x * p[3], rec->N.y * p[4], rec->N.z * p[5]));
      ok = 1;
      break;
    }
    default: return 0;
  }
  if (ok && os->is_top[g]) rec->top = g;
  return ok;
}

/* Camera.world.Hit from the integrator: fresh per-traversal volume counters. */
static int FN(world_hit)(FN(TC)* c, uint32_t dom, FN(Ray) r, REAL mn, REAL mx, FN(Rec)* rec) {
  if (c->S->os->nvol) memset(c->volcount, 0, sizeof(int) * (size_t)c->S->os->nvol);
  c->voldom = dom;
  rec->top = rec->prim = -1;
  rec->u = rec->v = 0;                                   /* rec := &HitRecord{} (camera.go:449) */
  return FN(hit)(c, c->S->os->d->root, r, mn, mx, rec);
}

/* ------------------------------------------------------------ textures / HDRI */
/* Perlin.Noise / Turb noise.go:31-67, 84-100 */
static REAL FN(perlin_noise)(const rt_perlin* P, V3R pt) {
  REAL fx = FLOOR(pt.x), fy = FLOOR(pt.y), fz = FLOOR(pt.z);
  REAL u = pt.x - fx, v = pt.y - fy, w = pt.z - fz;
  int i = (int)fx, j = (int)fy, k = (int)fz;
  REAL accum = 0;
  for (int di = 0; di < 2; ++di)
    for (int dj = 0; dj < 2; ++dj)
      for (int dk = 0; dk < 2; ++dk) {
        int idx = P->perm_x[(i + di) & 255] ^ P->perm_y[(j + dj) & 255] ^ P->perm_z[(k + dk) & 255];
        V3R cv = FN(mk)((REAL)P->randvec[idx][0], (REAL)P->randvec[idx][1], (REAL)P->randvec[idx][2]);
        V3R wv = FN(mk)(u - (REAL)di, v - (REAL)dj, w - (REAL)dk);
        accum += ((REAL)di * u + (1 - (REAL)di) * (1 - u)) * ((REAL)dj * v + (1 - (REAL)dj) * (1 - v)) *
                 ((REAL)dk * w + (1 - (REAL)dk) * (1 - w)) * FN(dot)(cv, wv);
      }
  return accum;
}
static REAL FN(perlin_turb)(const rt_perlin* P, V3R pt, int depth) {
  REAL accum = 0, weight = 1;
  V3R tp = pt;
  for (int i = 0; i < depth; ++i) {
    accum += weight * FN(perlin_noise)(P, tp);
    weight *= (REAL)0.5;
    tp = FN(scale)(tp, 2);
  }
  return FABS(accum);
}

static V3R FN(tex_value)(const FN(OS)* S, int ti, REAL tu, REAL tv, V3R p) {   /* texture.go:43-85 */
  const rt_texture* t = &S->os->d->textures[ti];
  if (t->kind == RT_TEX_NOISE) {                                       /* texture.go:81-85 */
    const rt_perlin* P = &S->os->d->perlins[t->perlin];
    REAL sc = (REAL)t->scale;
    REAL s = sc * p.z + 10 * FN(perlin_turb)(P, FN(scale)(p, sc), 7);
    REAL gv = (REAL)0.5 * (1 + SIN(s));
    return FN(mk)(gv, gv, gv);
  }
  if (t->kind == RT_TEX_IMAGE) {                                       /* image_texture.go:26-41 */
    const rt_image* im = &S->os->d->images[t->image];
    if (im->height <= 0 || !im->rgb) return FN(mk)(0, 1, 1);
    REAL cu = tu < 0 ? 0 : (tu > 1 ? 1 : tu);
    REAL cv = 1 - (tv < 0 ? 0 : (tv > 1 ? 1 : tv));
    int x = (int)(cu * (REAL)im->width), y = (int)(cv * (REAL)im->height);
    x = x < 0 ? 0 : (x < im->width ? x : im->width - 1);              /* image_loader.go:97-120 */
    y = y < 0 ? 0 : (y < im->height ? y : im->height - 1);
    const double* px = im->rgb + 3 * ((size_t)y * (size_t)im->width + (size_t)x);
    return FN(mk)((REAL)px[0], (REAL)px[1], (REAL)px[2]);
  }
  if (t->kind == RT_TEX_CHECKER) {
    const REAL eps = (REAL)1e-4;
    REAL inv = (REAL)t->inv_scale;
    int xi = (int)FLOOR(inv * p.x + eps), yi = (int)FLOOR(inv * p.y + eps), zi = (int)FLOOR(inv * p.z + eps);
    int even = ((xi + yi + zi) % 2) == 0;
    const rt_texture* s = &S->os->d->textures[even ? t->even : t->odd];
    return FN(mk)((REAL)s->albedo[0], (REAL)s->albedo[1], (REAL)s->albedo[2]);
  }
  return FN(mk)((REAL)t->albedo[0], (REAL)t->albedo[1], (REAL)t->albedo[2]);
}

static inline int FN(iclamp)(int x, int lo, int hi) { if (x < lo) return lo; if (x < hi) return x; return hi - 1; }

static void FN(dir_to_uv)(const FN(OS)* S, V3R dir, REAL* u, REAL* v) {   /* hdri.go:75-94 */
  V3R d = FN(unit)(dir);
  REAL phi = ATAN2(d.z, d.x);
  REAL dy = d.y > 1 ? 1 : (d.y < -1 ? -1 : d.y);
  REAL theta = ASIN(dy);
  REAL uu = (REAL)0.5 + phi / (2 * PI_R);
  REAL vv = (REAL)0.5 - theta / PI_R;
  uu = uu + S->env_rot / (2 * PI_R);
  uu = uu - FLOOR(uu);
  *u = uu;
  *v = vv;
}
static V3R FN(texel)(const FN(OS)* S, int x, int y) {
  const REAL* t = S->env_tex + ((size_t)y * S->os->env_w + x) * 3;
  return FN(mk)(t[0], t[1], t[2]);
}
static V3R FN(env_sample)(const FN(OS)* S, V3R dir) {    /* hdri.go:120-128, image_loader.go:398-436 */
  const int W = S->os->env_w, H = S->os->env_h;
  REAL u, v;
  FN(dir_to_uv)(S, dir, &u, &v);
  REAL px = u * (REAL)W - (REAL)0.5, py = v * (REAL)H - (REAL)0.5;
  int x0 = (int)FLOOR(px), y0 = (int)FLOOR(py);
  int x1 = x0 + 1, y1 = y0 + 1;
  REAL fx = px - (REAL)x0, fy = py - (REAL)y0;
  x0 = ((x0 % W) + W) % W;
  x1 = ((x1 % W) + W) % W;
  y0 = FN(iclamp)(y0, 0, H);
  y1 = FN(iclamp)(y1, 0, H);
  V3R c00 = FN(texel)(S, x0, y0), c10 = FN(texel)(S, x1, y0), c01 = FN(texel)(S, x0, y1), c11 = FN(texel)(S, x1, y1);
  V3R c0 = FN(add)(FN(scale)(c00, 1 - fx), FN(scale)(c10, fx));
  V3R c1 = FN(add)(FN(scale)(c01, 1 - fx), FN(scale)(c11, fx));
  return FN(add)(FN(scale)(c0, 1 - fy), FN(scale)(c1, fy));
}
static int FN(search_cdf)(const REAL* cdf, int n, REAL xi) {                /* hdri.go:300-322 */
  int lo = 0, hi = n;
  while (lo < hi) {
    int mid = (lo + hi) / 2;
    if (cdf[mid + 1] <= xi) lo = mid + 1; else hi = mid;
  }
  if (lo >= n) lo = n - 1;
  if (lo < 0) lo = 0;
  return lo;
}
static REAL FN(env_pdf)(const FN(OS)* S, V3R dir) {                          /* hdri.go:262-297 */
  const int W = S->os->env_w, H = S->os->env_h;
  REAL u, v;
  FN(dir_to_uv)(S, dir, &u, &v);
  int x = (int)(u * (REAL)W), y = (int)(v * (REAL)H);
  x = FN(iclamp)(x, 0, W);
  y = FN(iclamp)(y, 0, H);
  REAL theta = ((REAL)0.5 - v) * PI_R;
  REAL st = COS(theta);
  if (st < (REAL)1e-10) st = (REAL)1e-10;
  REAL p = S->env_pdf[(size_t)y * W + x] * (REAL)(W * H) / (2 * PI_R * PI_R * st);
  if (p < (REAL)1e-10) return (REAL)1e-10;
  return p;
}

/* ------------------------------------------------------------ integrator */
static V3R FN(sample_lights)(FN(TC)* c, const FN(Rec)* rec, V3R rdir, V3R att) {   /* camera.go:538-678 */
  const FN(OS)* S = c->S;
  const OScene* os = S->os;
  const rt_scene_desc* d = os->d;
  const int nl = d->num_lights;
  int li = (int)(FN(rnd)(c, O_DOM_NEE, 0) * (REAL)nl);
  if (li >= nl) li = nl - 1;
  V3R total = FN(mk)(0, 0, 0);
  if (os->env_valid && os->env_use_is) {                                    /* sampleHDRILight :565-607 */
    V3R ldir, em;
    REAL pdfH;
    if (!(os->env_total_power > 0)) {
      ldir = FN(random_unit_vector)(c, O_DOM_NEE, 5);
      em = FN(env_sample)(S, ldir);
      pdfH = (REAL)1 / (4 * PI_R);
    } else {
      const int W = os->env_w, H = os->env_h;
      REAL xi1 = FN(rnd)(c, O_DOM_NEE, 3);
      int y = FN(search_cdf)(S->env_marg, H, xi1);
      REAL xi2 = FN(rnd)(c, O_DOM_NEE, 4);
      int x = FN(search_cdf)(S->env_cond + (size_t)y * (W + 1), W, xi2);
      REAL uu = ((REAL)x + (REAL)0.5) / (REAL)W;
      REAL vv = ((REAL)y + (REAL)0.5) / (REAL)H;
      uu = uu - S->env_rot / (2 * PI_R);                                    /* UVToDirection hdri.go:97-113 */
      uu = uu - FLOOR(uu);
      REAL phi = (uu - (REAL)0.5) * 2 * PI_R;
      REAL th = ((REAL)0.5 - vv) * PI_R;
      REAL ct = COS(th);
      ldir = FN(mk)(ct * COS(phi), SIN(th), ct * SIN(phi));
      em = FN(texel)(S, x, y);
      pdfH = FN(env_pdf)(S, ldir);
    }
    REAL cth = FN(dot)(rec->N, ldir);
    if (cth > 0) {
      FN(Ray) sr;
      sr.o = rec->P; sr.d = ldir; sr.tm = 0;
      FN(Rec) srec;
      const int occluded = FN(world_hit)(c, O_DOM_VOL_SH_HDRI, sr, (REAL)0.001, (REAL)INFINITY, &srec);
      if (c->r_nee && (int)c->bounce < c->r_nb)                             /* path recorder */
        c->r_nee[(size_t)c->bounce * c->r_npix + c->r_pix] |= 2 | (occluded ? 0 : 8);
      if (!occluded) {
        REAL c2 = FN(dot)(rec->N, ldir);
        REAL pdfB = c2 < 0 ? 0 : c2 / PI_R;                                   /* Lambertian.PDF */
        REAL w = pdfH / (pdfH + pdfB);
        V3R ctb = FN(mul)(FN(scale)(em, cth / pdfH * w), att);
        total = FN(add)(total, FN(mk)(FN(gomin)(ctb.x, 20), FN(gomin)(ctb.y, 20), FN(gomin)(ctb.z, 20)));
      }
    }
  }
  if (nl > 0 && li < nl) {                                                  /* sampleAreaLight :610-678 */
    int lg = d->lights[li];
    const rt_hittable* lh = &d->hittables[lg];
    if (lh->kind == RT_QUAD) {
      const REAL* p = S->h[lg].p;
      REAL al = FN(rnd)(c, O_DOM_NEE, 1), be = FN(rnd)(c, O_DOM_NEE, 2);
      V3R lu = FN(mk)(p[3], p[4], p[5]), lv = FN(mk)(p[6], p[7], p[8]);
      V3R lp = FN(add)(FN(add)(FN(mk)(p[0], p[1], p[2]), FN(scale)(lu, al)), FN(scale)(lv, be));
      V3R tl = FN(sub)(lp, rec->P);
      REAL dist = FN(len)(tl);
      V3R ldir = FN(unit)(tl);
      REAL cth = FN(dot)(rec->N, ldir);
      if (cth > 0) {
        FN(Ray) sr;
        sr.o = rec->P; sr.d = ldir; sr.tm = 0;
        FN(Rec) srec;
        const int occluded = FN(world_hit)(c, O_DOM_VOL_SH_AREA, sr, (REAL)0.001, dist - (REAL)0.001, &srec);
        if (c->r_nee && (int)c->bounce < c->r_nb &&                         /* path recorder: a ray whose */
            !(FABS(FN(dot)(FN(mk)(p[12], p[13], p[14]), FN(neg)(ldir))) < (REAL)0.001))   /* light term counts */
          c->r_nee[(size_t)c->bounce * c->r_npix + c->r_pix] |= 1 | (occluded ? 0 : 4);
        if (!occluded) {
          const rt_material* lm = &d->materials[lh->material];
          V3R em = lm->kind == RT_DIFFUSE_LIGHT ? FN(tex_value)(S, lm->texture, 0, 0, lp) : FN(mk)(0, 0, 0);
          REAL area = FN(len)(FN(cross)(lu, lv));
          REAL cl = FABS(FN(dot)(FN(mk)(p[12], p[13], p[14]), FN(neg)(ldir)));
          if (!(cl < (REAL)0.001)) {
            REAL pdfL = (dist * dist) / (cl * area);
            REAL c2 = FN(dot)(rec->N, ldir);
            REAL pdfB = c2 < 0 ? 0 : c2 / PI_R;
            REAL w = pdfL / (pdfL + pdfB);
            V3R ctb = FN(scale)(FN(mul)(FN(scale)(em, cth / pdfL * w), att), (REAL)nl);
            total = FN(add)(total, FN(mk)(FN(gomin)(ctb.x, 20), FN(gomin)(ctb.y, 20), FN(gomin)(ctb.z, 20)));
          }
        }
      }
    }
  }
  return total;
}

/* rayColorInternal camera.go:443-518 (recursive, as the reference). */
static V3R FN(ray_color)(FN(TC)* c, FN(Ray) r, int depth, uint32_t bounce, int allow) {
  const FN(OS)* S = c->S;
  const OScene* os = S->os;
  if (depth <= 0) return FN(mk)(0, 0, 0);
  c->bounce = bounce;
  FN(Rec) rec;
  const int hit = FN(world_hit)(c, O_DOM_VOL, r, (REAL)0.001, (REAL)INFINITY, &rec);
  if (c->r_top && (int)bounce < c->r_nb) {                                   /* path recorder */
    const size_t e = (size_t)bounce * c->r_npix + c->r_pix;
    c->r_top[e] = hit ? rec.top : -1;
    c->r_prim[e] = hit ? rec.prim : -1;
    c->r_t[e] = hit ? (double)rec.t : -1.0;
    const double ray[6] = {(double)r.o.x, (double)r.o.y, (double)r.o.z, (double)r.d.x, (double)r.d.y, (double)r.d.z};
    memcpy(c->r_ray + e * 6, ray, sizeof ray);
  }
  if (!hit) {
    if (os->env_valid) {
      if (S->cam_phantom && depth == S->cam_max_depth) return FN(mk)(0, 0, 0);
      return FN(env_sample)(S, r.d);
    }
    if (S->cam_sky) {                                                        /* SkyGradient :520-526 */
      V3R ud = FN(unit)(r.d);
      REAL a = (REAL)0.5 * (ud.y + 1);
      return FN(add)(FN(scale)(FN(mk)(1, 1, 1), 1 - a), FN(scale)(FN(mk)((REAL)0.5, (REAL)0.7, 1), a));
    }
    return FN(ld3)(S->cam_bg);
  }
  const rt_material* m = &os->d->materials[rec.mat];
  V3R Le = FN(mk)(0, 0, 0);
  if (m->kind == RT_DIFFUSE_LIGHT) Le = FN(tex_value)(S, m->texture, rec.u, rec.v, rec.P);  /* Emitted */
  V3R att, sd;
  int scat = 1;
  switch (m->kind) {
    case RT_LAMBERTIAN:                                                      /* material.go:57-68 */
      sd = FN(add)(rec.N, FN(random_unit_vector)(c, O_DOM_SCATTER, 0));
      if (FN(near_zero)(sd)) sd = rec.N;
      att = FN(tex_value)(S, m->texture, rec.u, rec.v, rec.P);
      break;
    case RT_METAL: {                                                         /* material.go:113-119 */
      V3R refl = FN(reflect)(r.d, rec.N);
      refl = FN(add)(FN(unit)(refl), FN(scale)(FN(random_unit_vector)(c, O_DOM_SCATTER, 0), (REAL)m->fuzz));
      sd = refl;
      att = FN(mk)((REAL)m->albedo[0], (REAL)m->albedo[1], (REAL)m->albedo[2]);
      scat = FN(dot)(sd, rec.N) > 0;
      break;
    }
    case RT_DIELECTRIC: {                                                    /* material.go:164-188 */
      att = FN(mk)(1, 1, 1);
      REAL ior = (REAL)m->refraction_index;
      REAL ri = rec.front ? ((REAL)1 / ior) : ior;
      V3R ud = FN(unit)(r.d);
      REAL cc = FN(dot)(FN(neg)(ud), rec.N);
      REAL ct = cc < 1 ? cc : 1;
      REAL st = SQRT(1 - ct * ct);
      int cannot = ri * st > 1;
      int reflect = cannot;
      if (!cannot) {
        REAL r0 = (1 - ri) / (1 + ri);                                        /* reflectance :284-288 */
        r0 = r0 * r0;
        REAL rf = r0 + (1 - r0) * POW5(1 - ct);
        reflect = rf > FN(rnd)(c, O_DOM_FRESNEL, 0);
      }
      sd = reflect ? FN(reflect)(ud, rec.N) : FN(refract)(ud, rec.N, ri);
      break;
    }
    case RT_ISOTROPIC:                                                       /* material.go:266-270 */
      sd = FN(random_unit_vector)(c, O_DOM_SCATTER, 0);
      att = FN(tex_value)(S, m->texture, rec.u, rec.v, rec.P);
      break;
    default:                                                                 /* DiffuseLight */
      scat = 0;
      break;
  }
  if (!scat) return allow ? Le : FN(mk)(0, 0, 0);
  FN(Ray) sr;
  sr.o = rec.P; sr.d = sd; sr.tm = r.tm;
  int use_mis = m->kind == RT_LAMBERTIAN && os->d->num_lights > 0;
  if (!use_mis) {
    V3R L = FN(ray_color)(c, sr, depth - 1, bounce + 1, 1);
    c->bounce = bounce;
    return FN(add)(Le, FN(mul)(att, L));
  }
  c->bounce = bounce;
  V3R direct = FN(sample_lights)(c, &rec, r.d, att);
  V3R ind = FN(mul)(att, FN(ray_color)(c, sr, depth - 1, bounce + 1, 0));
  c->bounce = bounce;
  return FN(add)(FN(add)(Le, direct), ind);
}

/* RandomInUnitDisk (vec3.go:66-77) on the camera counters */
static V3R FN(disk_point)(FN(TC)* c) {
  V3R p = FN(mk)(0, 0, 0);
  for (int k = 0; k < O_MAX_TRIES; ++k) {
    uint32_t idx = 3u + 2u * (uint32_t)k;
    REAL x = -1 + 2 * FN(rnd)(c, O_DOM_CAMERA, idx), y = -1 + 2 * FN(rnd)(c, O_DOM_CAMERA, idx + 1);
    if (x * x + y * y + (REAL)0 * (REAL)0 < 1) { p = FN(mk)(x, y, 0); break; }
  }
  return p;
}

/* GetRay slow path camera.go:390-434 (CameraMotion / FreeCamera): the basis
 * and pixel grid are rebuilt at rayTime from the cached viewport size. */
static FN(Ray) FN(get_ray_slow)(FN(TC)* c, int i, int j, REAL ox, REAL oy, REAL tm) {
  const FN(OS)* S = c->S;
  V3R center = FN(add)(FN(ld3)(S->cam_corig), FN(scale)(FN(ld3)(S->cam_cdir), tm));   /* centerMotion.At */
  V3R w;
  if (S->cam_free) w = FN(neg)(FN(ld3)(S->cam_fwd));
  else w = FN(unit)(FN(sub)(center, FN(add)(FN(ld3)(S->cam_laorig), FN(scale)(FN(ld3)(S->cam_ladir), tm))));
  V3R u = FN(unit)(FN(cross)(FN(ld3)(S->cam_vup), w));
  V3R v = FN(cross)(w, u);
  V3R vu = FN(scale)(u, S->cam_vw);
  V3R vv = FN(scale)(FN(neg)(v), S->cam_vh);
  V3R du = FN(divs)(vu, (REAL)S->cam_w);
  V3R dv = FN(divs)(vv, (REAL)S->cam_h);
  V3R ul = FN(sub)(FN(sub)(FN(sub)(center, FN(scale)(w, S->cam_focus)), FN(divs)(vu, 2)), FN(divs)(vv, 2));
  V3R p00 = FN(add)(ul, FN(scale)(FN(add)(du, dv), (REAL)0.5));
  V3R ps = FN(add)(FN(add)(p00, FN(scale)(du, (REAL)i + ox)), FN(scale)(dv, (REAL)j + oy));
  V3R ro = center;
  if (S->cam_defocus) {
    V3R p = FN(disk_point)(c);
    ro = FN(add)(FN(add)(center, FN(scale)(FN(scale)(u, S->cam_rad), p.x)), FN(scale)(FN(scale)(v, S->cam_rad), p.y));
  }
  FN(Ray) r;
  r.o = ro;
  r.d = FN(sub)(ps, ro);
  r.tm = tm;
  return r;
}

/* GetRay camera.go:368-388 */
static FN(Ray) FN(get_ray)(FN(TC)* c, int i, int j) {
  const FN(OS)* S = c->S;
  c->bounce = 0;
  REAL ox = FN(rnd)(c, O_DOM_CAMERA, 0) - (REAL)0.5;
  REAL oy = FN(rnd)(c, O_DOM_CAMERA, 1) - (REAL)0.5;
  REAL tm = FN(rnd)(c, O_DOM_CAMERA, 2);
  if (S->cam_slow) return FN(get_ray_slow)(c, i, j, ox, oy, tm);
  V3R ps = FN(add)(FN(add)(FN(ld3)(S->cam_p00), FN(scale)(FN(ld3)(S->cam_du), (REAL)i + ox)),
                   FN(scale)(FN(ld3)(S->cam_dv), (REAL)j + oy));
  V3R ro = FN(ld3)(S->cam_center);
  if (S->cam_defocus) {                                                      /* defocusDiskSample :354-362 */
    V3R p = FN(disk_point)(c);
    ro = FN(add)(FN(add)(ro, FN(scale)(FN(ld3)(S->cam_disk_u), p.x)), FN(scale)(FN(ld3)(S->cam_disk_v), p.y));
  }
  FN(Ray) r;
  r.o = ro;
  r.d = FN(sub)(ps, ro);
  r.tm = tm;
  return r;
}

/* ------------------------------------------------------------ bucket driver */
typedef struct {
  const FN(OS)* S;
  const rt_bucket* buckets;
  int nb;
  int W;
  const rt_render_params* p;
  double* accum;
  atomic_int next;
} FN(Job);

static void* FN(worker)(void* arg) {                    /* bucket_renderer.go:246-301 */
  FN(Job)* J = (FN(Job)*)arg;
  int* vc = (int*)calloc((size_t)(J->S->os->nvol > 0 ? J->S->os->nvol : 1), sizeof(int));
  FN(TC) c;
  memset(&c, 0, sizeof(c));
  c.S = J->S;
  c.volcount = vc;
  for (;;) {
    int b = atomic_fetch_add(&J->next, 1);
    if (b >= J->nb) break;
    const rt_bucket* bk = &J->buckets[b];
    for (int y = bk->y; y < bk->y + bk->height; ++y)
      for (int x = bk->x; x < bk->x + bk->width; ++x) {
        const uint32_t pix = (uint32_t)y * (uint32_t)J->W + (uint32_t)x;
        double sx = 0, sy = 0, sz = 0;
        for (int s = 0; s < J->p->samples_per_pixel; ++s) {
          c.key = o_path_key(J->p->seed, pix, (uint32_t)(J->p->sample_offset + s));
          FN(Ray) r = FN(get_ray)(&c, x, y);
          V3R L = FN(ray_color)(&c, r, J->p->max_depth, 0, 1);
          sx += (double)L.x; sy += (double)L.y; sz += (double)L.z;
        }
        double* o = J->accum + (size_t)pix * 3;
        if (J->p->accumulate) { o[0] += sx; o[1] += sy; o[2] += sz; }
        else { o[0] = sx; o[1] = sy; o[2] = sz; }
      }
  }
  free(vc);
  return NULL;
}

static int FN(render)(const OScene* os, const rt_camera_desc* cam, const rt_render_params* p, int nthreads,
                      const rt_bucket* buckets, int nb, double* accum) {
  FN(OS) S;
  int rc = FN(prep)(&S, os, cam);
  if (rc) return rc;
  FN(Job) J;
  J.S = &S;
  J.buckets = buckets;
  J.nb = nb;
  J.W = cam->image_width;
  J.p = p;
  J.accum = accum;
  atomic_init(&J.next, 0);
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
  for (int i = 0; i < nthreads; ++i) pthread_create(&th[i], NULL, FN(worker), &J);
  for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
  free(th);
  FN(unprep)(&S);
  return 0;
}

static int FN(primary)(const OScene* os, const rt_camera_desc* cam, uint32_t seed, int sample, int32_t* top,
                       int32_t* prim, double* tout) {
  FN(OS) S;
  int rc = FN(prep)(&S, os, cam);
  if (rc) return rc;
  int* vc = (int*)calloc((size_t)(os->nvol > 0 ? os->nvol : 1), sizeof(int));
  FN(TC) c;
  memset(&c, 0, sizeof(c));
  c.S = &S;
  c.volcount = vc;
  const int W = cam->image_width, H = cam->image_height;
  for (int j = 0; j < H; ++j)
    for (int i = 0; i < W; ++i) {
      uint32_t pix = (uint32_t)j * (uint32_t)W + (uint32_t)i;
      c.key = o_path_key(seed, pix, (uint32_t)sample);
      FN(Ray) r = FN(get_ray)(&c, i, j);
      FN(Rec) rec;
      int h = FN(world_hit)(&c, O_DOM_VOL, r, (REAL)0.001, (REAL)INFINITY, &rec);
      top[pix] = h ? rec.top : -1;
      prim[pix] = h ? rec.prim : -1;
      tout[pix] = h ? (double)rec.t : -1.0;
    }
  free(vc);
  FN(unprep)(&S);
  return 0;
}

/* Every bounce of one sample per pixel (rayColorInternal camera.go:443-518 to
 * depth nb): world.Hit ids, t and the incoming ray per bounce, the NEE
 * shadow rays traced and their visibility (sampleHDRILight :582,
 * sampleAreaLight :639).  Outputs are filled by the caller (ended paths keep
 * the fill).  Pixels are split over nthreads. */
typedef struct {
  const FN(OS)* S;
  uint32_t seed;
  int sample, nb, t0, nth;
  int32_t *top, *prim, *nee;
  double *t, *ray;
} FN(PJob);

static void* FN(path_worker)(void* arg) {
  FN(PJob)* J = (FN(PJob)*)arg;
  const FN(OS)* S = J->S;
  int* vc = (int*)calloc((size_t)(S->os->nvol > 0 ? S->os->nvol : 1), sizeof(int));
  FN(TC) c;
  memset(&c, 0, sizeof(c));
  c.S = S;
  c.volcount = vc;
  c.r_top = J->top; c.r_prim = J->prim; c.r_t = J->t; c.r_ray = J->ray; c.r_nee = J->nee;
  c.r_nb = J->nb;
  const int W = S->cam_w, H = S->cam_h;
  c.r_npix = (size_t)W * (size_t)H;
  for (size_t pix = (size_t)J->t0; pix < c.r_npix; pix += (size_t)J->nth) {
    c.r_pix = pix;
    c.key = o_path_key(J->seed, (uint32_t)pix, (uint32_t)J->sample);
    FN(Ray) r = FN(get_ray)(&c, (int)(pix % (size_t)W), (int)(pix / (size_t)W));
    (void)FN(ray_color)(&c, r, J->nb, 0, 1);
  }
  (void)H;
  free(vc);
  return NULL;
}

static int FN(paths)(const OScene* os, const rt_camera_desc* cam, uint32_t seed, int sample, int nb, int nthreads,
                     int32_t* top, int32_t* prim, double* t, double* ray, int32_t* nee) {
  FN(OS) S;
  int rc = FN(prep)(&S, os, cam);
  if (rc) return rc;
  if (nthreads < 1) nthreads = 1;
  FN(PJob)* J = (FN(PJob)*)malloc(sizeof(FN(PJob)) * (size_t)nthreads);
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
  for (int i = 0; i < nthreads; ++i) {
    J[i].S = &S; J[i].seed = seed; J[i].sample = sample; J[i].nb = nb; J[i].t0 = i; J[i].nth = nthreads;
    J[i].top = top; J[i].prim = prim; J[i].nee = nee; J[i].t = t; J[i].ray = ray;
    pthread_create(&th[i], NULL, FN(path_worker), &J[i]);
  }
  for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
  free(th);
  free(J);
  FN(unprep)(&S);
  return 0;
}

#undef V3R
#undef FN
#undef CAT
#undef CAT2
