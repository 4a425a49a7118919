// rt_host.cpp — constructors, BVH builder, loaders, camera setup and scenes of
// the host-side rt mirror (see rt_host.h).  Every function cites the Go code
// whose behaviour it reproduces.
#include "rt_host.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <sys/stat.h>

namespace rt {

// ============================================================ emit (graph desc)
static rt_hittable blank(int kind, const AABB& b) {
  rt_hittable h;
  std::memset(&h, 0, sizeof(h));
  h.kind = kind;
  h.material = -1;
  b.to(h.bbox);
  return h;
}
static void put3(double* p, const Vec3& v) { p[0] = v.X; p[1] = v.Y; p[2] = v.Z; }

int SolidColor::emit(Emitter& e) const {
  rt_texture t{};
  t.kind = RT_TEX_SOLID;
  put3(t.albedo, Albedo);
  e.textures.push_back(t);
  return int(e.textures.size()) - 1;
}
int CheckerTexture::emit(Emitter& e) const {
  int ev = e.emit_texture(even), od = e.emit_texture(odd);
  rt_texture t{};
  t.kind = RT_TEX_CHECKER;
  t.even = ev;
  t.odd = od;
  t.inv_scale = invScale;
  e.textures.push_back(t);
  return int(e.textures.size()) - 1;
}
int NoiseTexture::emit(Emitter& e) const {
  int pi;
  if (!e.seen(noise.get(), pi)) {
    rt_perlin p{};
    for (int i = 0; i < 256; ++i) {
      p.randvec[i][0] = noise->randvec[i].X; p.randvec[i][1] = noise->randvec[i].Y; p.randvec[i][2] = noise->randvec[i].Z;
      p.perm_x[i] = noise->permX[i]; p.perm_y[i] = noise->permY[i]; p.perm_z[i] = noise->permZ[i];
    }
    e.perlins.push_back(p);
    pi = int(e.perlins.size()) - 1;
    e.memo[noise.get()] = pi;
  }
  rt_texture t{};
  t.kind = RT_TEX_NOISE;
  t.scale = scale;
  t.perlin = pi;
  e.textures.push_back(t);
  return int(e.textures.size()) - 1;
}
int ImageTexture::emit(Emitter& e) const {
  int ii;
  if (!e.seen(image.get(), ii)) {
    rt_image im{};
    im.width = image->width;
    im.height = image->height;
    im.rgb = image->rgb.empty() ? nullptr : image->rgb.data();
    e.images.push_back(im);
    ii = int(e.images.size()) - 1;
    e.memo[image.get()] = ii;
  }
  rt_texture t{};
  t.kind = RT_TEX_IMAGE;
  t.image = ii;
  e.textures.push_back(t);
  return int(e.textures.size()) - 1;
}
static int push_mat(Emitter& e, const rt_material& m) { e.materials.push_back(m); return int(e.materials.size()) - 1; }
int Lambertian::emit(Emitter& e) const { rt_material m{}; m.kind = RT_LAMBERTIAN; m.texture = e.emit_texture(tex); return push_mat(e, m); }
int Metal::emit(Emitter& e) const { rt_material m{}; m.kind = RT_METAL; m.texture = -1; put3(m.albedo, Albedo); m.fuzz = Fuzz; return push_mat(e, m); }
int Dielectric::emit(Emitter& e) const { rt_material m{}; m.kind = RT_DIELECTRIC; m.texture = -1; m.refraction_index = RefractionIndex; return push_mat(e, m); }
int DiffuseLight::emit(Emitter& e) const { rt_material m{}; m.kind = RT_DIFFUSE_LIGHT; m.texture = e.emit_texture(tex); return push_mat(e, m); }
int Isotropic::emit(Emitter& e) const { rt_material m{}; m.kind = RT_ISOTROPIC; m.texture = e.emit_texture(tex); return push_mat(e, m); }

int Sphere::emit(Emitter& e) const {
  rt_hittable h = blank(RT_SPHERE, bbox);
  h.material = e.emit_material(Mat);
  put3(h.p, c0); put3(h.p + 3, vel); h.p[6] = Radius;
  return e.add(h);
}
int Quad::emit(Emitter& e) const {
  rt_hittable h = blank(RT_QUAD, bbox);
  h.material = e.emit_material(mat);
  put3(h.p, Q); put3(h.p + 3, u); put3(h.p + 6, v); put3(h.p + 9, w); put3(h.p + 12, normal); h.p[15] = D;
  return e.add(h);
}
int Triangle::emit(Emitter& e) const {
  rt_hittable h = blank(RT_TRIANGLE, bbox);
  h.material = e.emit_material(mat);
  put3(h.p, v0); put3(h.p + 3, v1); put3(h.p + 6, v2); put3(h.p + 9, normal);
  return e.add(h);
}
int Circle::emit(Emitter& e) const {
  rt_hittable h = blank(RT_CIRCLE, bbox);
  h.material = e.emit_material(mat);
  put3(h.p, center); put3(h.p + 3, normal); h.p[6] = radius; h.p[7] = D;
  return e.add(h);
}
int Plane::emit(Emitter& e) const {
  rt_hittable h = blank(RT_PLANE, bbox);
  h.material = e.emit_material(Mat);
  put3(h.p, Point); put3(h.p + 3, Normal);
  return e.add(h);
}
static int emit_list(Emitter& e, int kind, const AABB& box, const std::vector<HittablePtr>& objs) {
  std::vector<int> idx;
  idx.reserve(objs.size());
  for (const auto& o : objs) idx.push_back(e.emit_hittable(o));
  rt_hittable h = blank(kind, box);
  h.a = int(e.children.size());
  h.b = int(idx.size());
  for (int i : idx) e.children.push_back(i);
  return e.add(h);
}
int HittableList::emit(Emitter& e) const { return emit_list(e, RT_LIST, bbox, Objects); }
int BVHLeaf::emit(Emitter& e) const { return emit_list(e, RT_BVH_LEAF, bbox, objects); }
int BVHNode::emit(Emitter& e) const {
  int l = e.emit_hittable(left);
  int r = e.emit_hittable(right);   // memoised: the leaf wrapper gets l == r
  rt_hittable h = blank(RT_BVH_NODE, bbox);
  h.a = l;
  h.b = r;
  return e.add(h);
}
int Translate::emit(Emitter& e) const {
  int c = e.emit_hittable(Obj);
  rt_hittable h = blank(RT_TRANSLATE, bbox);
  h.a = c; put3(h.p, Offset);
  return e.add(h);
}
int Rotate::emit(Emitter& e) const {
  int c = e.emit_hittable(Obj);
  rt_hittable h = blank(axis == 0 ? RT_ROTATE_X : axis == 1 ? RT_ROTATE_Y : RT_ROTATE_Z, bbox);
  h.a = c; h.p[0] = SinTheta; h.p[1] = CosTheta;
  return e.add(h);
}
int ScaleH::emit(Emitter& e) const {
  int c = e.emit_hittable(Obj);
  rt_hittable h = blank(RT_SCALE, bbox);
  h.a = c; put3(h.p, Factor); put3(h.p + 3, InvFactor);
  return e.add(h);
}
int Volume::emit(Emitter& e) const {
  int c = e.emit_hittable(boundary);
  rt_hittable h = blank(RT_VOLUME, boundary->BoundingBox());
  h.a = c; h.material = e.emit_material(phase); h.p[0] = negInvDensity;
  return e.add(h);
}

void Emitter::build(const HittablePtr& world, const Camera& cam) {
  root = emit_hittable(world);
  for (const auto& l : cam.Lights) lights.push_back(emit_hittable(l));
  if (cam.Environment && cam.Environment->IsValid()) {
    env_rgb = cam.Environment->data;
    env.width = cam.Environment->width;
    env.height = cam.Environment->height;
    env.rgb = env_rgb.data();
    env.rotation = cam.Environment->rotation;
    env.use_importance_sampling = cam.Environment->useImportanceSampling ? 1 : 0;
  }
}
rt_scene_desc Emitter::desc() const {
  rt_scene_desc d{};
  d.hittables = hittables.data();
  d.num_hittables = int(hittables.size());
  d.children = children.data();
  d.num_children = int(children.size());
  d.root = root;
  d.materials = materials.data();
  d.num_materials = int(materials.size());
  d.textures = textures.data();
  d.num_textures = int(textures.size());
  d.lights = lights.data();
  d.num_lights = int(lights.size());
  d.environment = env.rgb ? &env : nullptr;
  d.images = images.empty() ? nullptr : images.data();
  d.num_images = int(images.size());
  d.perlins = perlins.empty() ? nullptr : perlins.data();
  d.num_perlins = int(perlins.size());
  return d;
}

// ============================================================ constructors
HittablePtr NewSphere(Point3 c, double r, MaterialPtr m) {   // sphere.go:14-22
  auto s = std::make_shared<Sphere>();
  Vec3 rv{r, r, r};
  s->c0 = c; s->vel = {0, 0, 0}; s->Radius = std::fmax(0, r); s->Mat = std::move(m);
  s->bbox = AABB::FromPoints(c.Sub(rv), c.Add(rv));
  return s;
}
HittablePtr NewMovingSphere(Point3 c1, Point3 c2, double r, MaterialPtr m) {   // sphere.go:24-43
  auto s = std::make_shared<Sphere>();
  Vec3 rv{r, r, r};
  s->c0 = c1; s->vel = c2.Sub(c1); s->Radius = std::fmax(0, r); s->Mat = std::move(m);
  s->bbox = AABB::FromBoxes(AABB::FromPoints(c1.Sub(rv), c1.Add(rv)), AABB::FromPoints(c2.Sub(rv), c2.Add(rv)));
  return s;
}
std::shared_ptr<Quad> NewQuad(Point3 Q, Vec3 u, Vec3 v, MaterialPtr m) {   // quad.go:16-38
  auto q = std::make_shared<Quad>();
  q->Q = Q; q->u = u; q->v = v; q->mat = std::move(m);
  Vec3 n = Cross(u, v);
  q->normal = n.Unit();
  q->D = Dot(q->normal, Q);
  q->w = n.Scale(1.0 / Dot(n, n));
  q->bbox = AABB::FromBoxes(AABB::FromPoints(Q, Q.Add(u).Add(v)), AABB::FromPoints(Q.Add(u), Q.Add(v)));
  return q;
}
HittablePtr NewTriangle(Point3 a, Point3 b, Point3 c, MaterialPtr m) {   // triangle.go:17-50
  auto t = std::make_shared<Triangle>();
  t->v0 = a; t->v1 = b; t->v2 = c; t->mat = std::move(m);
  t->normal = Cross(b.Sub(a), c.Sub(a)).Unit();
  Point3 mn{std::fmin(a.X, std::fmin(b.X, c.X)), std::fmin(a.Y, std::fmin(b.Y, c.Y)), std::fmin(a.Z, std::fmin(b.Z, c.Z))};
  Point3 mx{std::fmax(a.X, std::fmax(b.X, c.X)), std::fmax(a.Y, std::fmax(b.Y, c.Y)), std::fmax(a.Z, std::fmax(b.Z, c.Z))};
  t->bbox = AABB::FromPoints(mn, mx);
  return t;
}
HittablePtr NewPlane(Point3 p, Vec3 n, MaterialPtr m) {   // plane.go:12-19
  auto pl = std::make_shared<Plane>();
  pl->Point = p; pl->Normal = n.Unit(); pl->Mat = std::move(m);
  pl->bbox = AABB::FromIntervals(Interval::Universe(), Interval::Universe(), Interval::Universe());
  return pl;
}

HittablePtr NewCircle(Point3 c, Vec3 n, double r, MaterialPtr m) {   // circle.go:14-31
  auto ci = std::make_shared<Circle>();
  ci->normal = n.Unit(); ci->center = c; ci->radius = r; ci->mat = std::move(m);
  ci->D = Dot(ci->normal, c);
  Vec3 rv{r, r, r};
  ci->bbox = AABB::FromPoints(c.Sub(rv), c.Add(rv));
  return ci;
}

std::shared_ptr<Perlin> NewPerlin(SceneRng& R) {   // noise.go:15-29, 70-82
  auto p = std::make_shared<Perlin>();
  for (int i = 0; i < 256; ++i) {
    Vec3 v{R.Range(-1, 1), R.Range(-1, 1), R.Range(-1, 1)};   // RandomVec3Range(-1, 1)
    p->randvec[i] = v.Unit();
  }
  for (int* perm : {p->permX, p->permY, p->permZ}) {
    for (int i = 0; i < 256; ++i) perm[i] = i;
    for (int i = 255; i > 0; --i) {                            // permute: RandomInt(0, i)
      const int target = std::min(i, int(R.RandomDouble() * double(i + 1)));
      std::swap(perm[i], perm[target]);
    }
  }
  return p;
}

bool LoadPPM(const std::string& path, ImageData& img, std::string& err) {
  std::ifstream f(path, std::ios::binary);
  if (!f) { err = "image not found: " + path; return false; }
  std::string magic;
  int w = 0, h = 0, maxv = 0;
  f >> magic >> w >> h >> maxv;
  f.get();
  if (magic != "P6" || w <= 0 || h <= 0 || maxv != 255) { err = "not an 8-bit binary PPM: " + path; return false; }
  std::vector<unsigned char> px(size_t(w) * h * 3);
  if (!f.read(reinterpret_cast<char*>(px.data()), std::streamsize(px.size()))) { err = "truncated PPM: " + path; return false; }
  img.width = w;
  img.height = h;
  img.rgb.resize(px.size());
  for (size_t i = 0; i < px.size(); ++i) {
    const double lin = double(px[i]) / 255.0;           // RGBA() 16-bit / 65535 of an 8-bit channel
    img.rgb[i] = lin > 0 ? std::sqrt(lin) : 0.0;        // LinearToGamma (utils.go:85-90)
  }
  return true;
}

HittablePtr NewTranslate(HittablePtr o, Vec3 off) {   // transform.go:84-91
  auto t = std::make_shared<Translate>();
  t->bbox = o->BoundingBox().Translate(off);
  t->Obj = std::move(o); t->Offset = off;
  return t;
}
static HittablePtr make_rot(int axis, HittablePtr o, double deg) {   // transform.go:120-157, 201-238, 282-319
  double rad = DegreesToRadians(deg);
  double s = std::sin(rad), c = std::cos(rad);
  AABB b = o->BoundingBox();
  const double inf = std::numeric_limits<double>::infinity();
  Point3 mn{inf, inf, inf}, mx{-inf, -inf, -inf};
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j)
      for (int k = 0; k < 2; ++k) {
        double x = double(i) * b.X.Max + double(1 - i) * b.X.Min;
        double y = double(j) * b.Y.Max + double(1 - j) * b.Y.Min;
        double z = double(k) * b.Z.Max + double(1 - k) * b.Z.Min;
        Vec3 t{x, y, z};
        if (axis == 1) { t.X = c * x + s * z; t.Z = -s * x + c * z; }
        else if (axis == 0) { t.Y = c * y - s * z; t.Z = s * y + c * z; }
        else { t.X = c * x - s * y; t.Y = s * x + c * y; }
        mn.X = std::fmin(mn.X, t.X); mx.X = std::fmax(mx.X, t.X);
        mn.Y = std::fmin(mn.Y, t.Y); mx.Y = std::fmax(mx.Y, t.Y);
        mn.Z = std::fmin(mn.Z, t.Z); mx.Z = std::fmax(mx.Z, t.Z);
      }
  auto r = std::make_shared<Rotate>();
  r->axis = axis; r->Obj = std::move(o); r->SinTheta = s; r->CosTheta = c;
  r->bbox = AABB::FromPoints(mn, mx);
  return r;
}
HittablePtr Rx(HittablePtr o, double deg) { return make_rot(0, std::move(o), deg); }
HittablePtr Ry(HittablePtr o, double deg) { return make_rot(1, std::move(o), deg); }
HittablePtr Rz(HittablePtr o, double deg) { return make_rot(2, std::move(o), deg); }
HittablePtr NewScale(HittablePtr o, Vec3 f) {   // transform.go:367-402
  auto s = std::make_shared<ScaleH>();
  s->Factor = f;
  s->InvFactor = {1.0 / f.X, 1.0 / f.Y, 1.0 / f.Z};
  AABB b = o->BoundingBox();
  Point3 mn{b.X.Min * f.X, b.Y.Min * f.Y, b.Z.Min * f.Z}, mx{b.X.Max * f.X, b.Y.Max * f.Y, b.Z.Max * f.Z};
  if (mn.X > mx.X) std::swap(mn.X, mx.X);
  if (mn.Y > mx.Y) std::swap(mn.Y, mx.Y);
  if (mn.Z > mx.Z) std::swap(mn.Z, mx.Z);
  s->bbox = AABB::FromPoints(mn, mx);
  s->Obj = std::move(o);
  return s;
}
HittablePtr Transform::Apply(HittablePtr obj) const {   // transform.go:24-46
  HittablePtr r = std::move(obj);
  if (Scale.X != 1.0 || Scale.Y != 1.0 || Scale.Z != 1.0) r = NewScale(r, Scale);
  if (Rotation.X != 0) r = Rx(r, Rotation.X);
  if (Rotation.Y != 0) r = Ry(r, Rotation.Y);
  if (Rotation.Z != 0) r = Rz(r, Rotation.Z);
  if (Position.X != 0 || Position.Y != 0 || Position.Z != 0) r = NewTranslate(r, Position);
  return r;
}
HittablePtr NewVolumeFromColor(HittablePtr boundary, double density, Color albedo) {   // volume.go:25-31
  auto v = std::make_shared<Volume>();
  v->boundary = std::move(boundary);
  v->negInvDensity = -1.0 / density;
  v->phase = std::make_shared<Isotropic>(NewSolidColor(albedo));
  return v;
}
HittablePtr Box(Point3 a, Point3 b, MaterialPtr m) {   // primitives.go:5-37
  auto sides = NewHittableList();
  Point3 mn{std::fmin(a.X, b.X), std::fmin(a.Y, b.Y), std::fmin(a.Z, b.Z)};
  Point3 mx{std::fmax(a.X, b.X), std::fmax(a.Y, b.Y), std::fmax(a.Z, b.Z)};
  Vec3 dx{mx.X - mn.X, 0, 0}, dy{0, mx.Y - mn.Y, 0}, dz{0, 0, mx.Z - mn.Z};
  sides->Add(NewQuad({mn.X, mn.Y, mx.Z}, dx, dy, m));
  sides->Add(NewQuad({mx.X, mn.Y, mx.Z}, dz.Neg(), dy, m));
  sides->Add(NewQuad({mx.X, mn.Y, mn.Z}, dx.Neg(), dy, m));
  sides->Add(NewQuad({mn.X, mn.Y, mn.Z}, dz, dy, m));
  sides->Add(NewQuad({mn.X, mx.Y, mx.Z}, dx, dz.Neg(), m));
  sides->Add(NewQuad({mn.X, mn.Y, mn.Z}, dx, dz, m));
  return sides;
}

HittablePtr Pyramid(Point3 bc, double base, double height, MaterialPtr m) {   // primitives.go:39-80
  auto sides = NewHittableList();
  sides->Add(NewQuad({bc.X - base / 2, bc.Y, bc.Z - base / 2}, {base, 0, 0}, {0, 0, base}, m));
  const Point3 apex{bc.X, bc.Y + height, bc.Z};
  const double hs = base / 2;
  const Point3 corners[4] = {{bc.X + hs, bc.Y, bc.Z - hs}, {bc.X + hs, bc.Y, bc.Z + hs},
                             {bc.X - hs, bc.Y, bc.Z + hs}, {bc.X - hs, bc.Y, bc.Z - hs}};
  for (int i = 0; i < 4; ++i) sides->Add(NewTriangle(corners[i], corners[(i + 1) % 4], apex, m));
  return sides;
}

// ============================================================ BVH (bvh.go)
namespace {
struct BvhPrim { size_t index; AABB bbox; Vec3 centroid; };
double axis_of(const Vec3& c, int a) { return a == 0 ? c.X : a == 1 ? c.Y : c.Z; }

std::shared_ptr<BVHNode> build_node(const std::vector<HittablePtr>& objects, std::vector<BvhPrim>& prims, size_t lo,
                                    size_t hi) {
  const size_t n = hi - lo;
  AABB bounds = prims[lo].bbox;
  AABB cb = AABB::FromPoints(prims[lo].centroid, prims[lo].centroid);
  for (size_t i = lo + 1; i < hi; ++i) {
    bounds = AABB::FromBoxes(bounds, prims[i].bbox);
    cb = AABB::FromBoxes(cb, AABB::FromPoints(prims[i].centroid, prims[i].centroid));
  }
  auto node = std::make_shared<BVHNode>();
  node->bbox = bounds;
  if (n <= 4) {   // bvhLeafMaxSize; BVHNode{left: leaf, right: leaf} (bvh.go:133-142)
    auto leaf = std::make_shared<BVHLeaf>();
    leaf->bbox = bounds;
    for (size_t i = lo; i < hi; ++i) leaf->objects.push_back(objects[prims[i].index]);
    node->left = leaf;
    node->right = leaf;
    return node;
  }
  const int axis = cb.LongestAxis();
  // sort.Slice by centroid (bvh.go:148-157).  Stable here; NaN centroids
  // (planes, universe bbox) sort first so the order is total.
  std::stable_sort(prims.begin() + long(lo), prims.begin() + long(hi), [axis](const BvhPrim& a, const BvhPrim& b) {
    double x = axis_of(a.centroid, axis), y = axis_of(b.centroid, axis);
    if (std::isnan(x) || std::isnan(y)) return std::isnan(x) && !std::isnan(y);
    return x < y;
  });
  const size_t mid = lo + n / 2;
  node->left = build_node(objects, prims, lo, mid);
  node->right = build_node(objects, prims, mid, hi);
  return node;
}
}  // namespace

std::shared_ptr<BVHNode> NewBVHNode(const std::vector<HittablePtr>& objects, size_t start, size_t end) {
  if (end <= start) return std::make_shared<BVHNode>();
  std::vector<BvhPrim> prims(end - start);
  for (size_t i = 0; i < prims.size(); ++i) {
    AABB b = objects[start + i]->BoundingBox();
    prims[i] = {start + i, b, b.Centroid()};
  }
  return build_node(objects, prims, 0, prims.size());
}
std::shared_ptr<BVHNode> NewBVHNodeFromList(const HittableList& list) {
  return NewBVHNode(list.Objects, 0, list.Objects.size());
}

// ============================================================ camera
void Camera::Initialize() {   // camera.go:286-344
  centerMotionOrig = LookFrom;
  lookAtMotionOrig = LookAt;
  centerMotionDir = CameraMotion ? LookFrom2.Sub(LookFrom) : Vec3{0, 0, 0};
  lookAtMotionDir = CameraMotion ? LookAt2.Sub(LookAt) : Vec3{0, 0, 0};
  ImageHeight = std::max(int(double(ImageWidth) / AspectRatio), 1);
  pixelsSamplesScale = 1.0 / double(SamplesPerPixel);
  center = LookFrom;
  double theta = DegreesToRadians(Vfov);
  double h = std::tan(theta / 2);
  double vh = 2 * h * FocusDist;
  double vw = vh * (double(ImageWidth) / double(ImageHeight));
  viewportHeight = vh;
  viewportWidth = vw;
  w = FreeCamera ? Forward.Neg() : center.Sub(LookAt).Unit();
  u = Cross(Vup, w).Unit();
  v = Cross(w, u);
  Vec3 vu = u.Scale(vw), vv = v.Neg().Scale(vh);
  pixelDeltaU = vu.Div(double(ImageWidth));
  pixelDeltaV = vv.Div(double(ImageHeight));
  Point3 ul = center.Sub(w.Scale(FocusDist)).Sub(vu.Div(2)).Sub(vv.Div(2));
  pixel00Loc = ul.Add(pixelDeltaU.Add(pixelDeltaV).Scale(0.5));
  double dr = FocusDist * std::tan(DegreesToRadians(DefocusAngle / 2));
  defocusDiskU = u.Scale(dr);
  defocusDiskV = v.Scale(dr);
}
rt_camera_desc Camera::desc() const {
  rt_camera_desc d{};
  d.image_width = ImageWidth;
  d.image_height = ImageHeight;
  d.samples_per_pixel = SamplesPerPixel;
  d.max_depth = MaxDepth;
  put3(d.center, center);
  put3(d.pixel00, pixel00Loc);
  put3(d.pixel_delta_u, pixelDeltaU);
  put3(d.pixel_delta_v, pixelDeltaV);
  d.defocus_angle = DefocusAngle;
  put3(d.defocus_disk_u, defocusDiskU);
  put3(d.defocus_disk_v, defocusDiskV);
  put3(d.background, Background);
  d.use_sky_gradient = UseSkyGradient;
  d.phantom_hdri = PhantomHDRI;
  d.camera_motion = CameraMotion;
  d.free_camera = FreeCamera;
  put3(d.center_motion_orig, centerMotionOrig);
  put3(d.center_motion_dir, centerMotionDir);
  put3(d.look_at_motion_orig, lookAtMotionOrig);
  put3(d.look_at_motion_dir, lookAtMotionDir);
  put3(d.vup, Vup);
  put3(d.forward, Forward);
  d.viewport_width = viewportWidth;
  d.viewport_height = viewportHeight;
  d.focus_dist = FocusDist;
  d.defocus_radius = FocusDist * std::tan(DegreesToRadians(DefocusAngle / 2));   // camera.go:356
  return d;
}

// ============================================================ HDR (image_loader.go)
static double ldexp1(int e) { return std::ldexp(1.0, e); }
bool LoadHDR(const std::string& path, HDRIEnvironment& env, std::string& err) {
  std::ifstream f(path, std::ios::binary);
  if (!f) { err = "cannot open " + path; return false; }
  std::string line;
  if (!std::getline(f, line) || line.rfind("#?", 0) != 0) { err = "missing #? signature"; return false; }
  for (;;) {   // header until empty line (parseHDRHeader :204-233)
    if (!std::getline(f, line)) { err = "unexpected end of header"; return false; }
    size_t a = line.find_first_not_of(" \t\r\n");
    if (a == std::string::npos) break;
  }
  if (!std::getline(f, line)) { err = "missing resolution"; return false; }
  std::istringstream rs(line);
  std::string t0, t2;
  long n1 = 0, n3 = 0;
  if (!(rs >> t0 >> n1 >> t2 >> n3)) { err = "bad resolution line"; return false; }
  int W, H;
  if (t0 == "-Y" && t2 == "+X") { H = int(n1); W = int(n3); }
  else if (t0 == "+X" && t2 == "-Y") { W = int(n1); H = int(n3); }
  else { err = "unsupported resolution format"; return false; }
  if (W <= 0 || H <= 0) { err = "bad size"; return false; }
  std::vector<double> data(size_t(W) * H * 3, 0.0);
  auto put = [&](const unsigned char* rgbe, int y, int x) {   // rgbeToColor :364-383
    size_t i = (size_t(y) * W + x) * 3;
    if (rgbe[3] == 0) { data[i] = data[i + 1] = data[i + 2] = 0; return; }
    double sc = ldexp1(int(rgbe[3]) - 128 - 8);
    data[i] = (double(rgbe[0]) + 0.5) * sc;
    data[i + 1] = (double(rgbe[1]) + 0.5) * sc;
    data[i + 2] = (double(rgbe[2]) + 0.5) * sc;
  };
  std::vector<unsigned char> comp(size_t(W) * 4);
  for (int y = 0; y < H; ++y) {   // readHDRScanline :274-309
    unsigned char hd[4];
    if (!f.read(reinterpret_cast<char*>(hd), 4)) { err = "short scanline header"; return false; }
    if (hd[0] == 2 && hd[1] == 2) {
      int sw = (int(hd[2]) << 8) | int(hd[3]);
      if (sw != W) { err = "scanline width mismatch"; return false; }
      for (int c = 0; c < 4; ++c) {   // readRLEScanline :312-361
        int x = 0;
        while (x < W) {
          int code = f.get();
          if (code == EOF) { err = "short RLE"; return false; }
          if (code > 128) {
            int cnt = code - 128, val = f.get();
            if (val == EOF) { err = "short RLE value"; return false; }
            for (int i = 0; i < cnt && x < W; ++i) comp[size_t(c) * W + x++] = (unsigned char)val;
          } else {
            for (int i = 0; i < code && x < W; ++i) {
              int val = f.get();
              if (val == EOF) { err = "short raw run"; return false; }
              comp[size_t(c) * W + x++] = (unsigned char)val;
            }
          }
        }
      }
      for (int x = 0; x < W; ++x) {
        unsigned char px[4] = {comp[x], comp[size_t(W) + x], comp[size_t(2) * W + x], comp[size_t(3) * W + x]};
        put(px, y, x);
      }
    } else {
      put(hd, y, 0);
      for (int x = 1; x < W; ++x) {
        unsigned char px[4];
        if (!f.read(reinterpret_cast<char*>(px), 4)) { err = "short flat scanline"; return false; }
        put(px, y, x);
      }
    }
  }
  env.width = W;
  env.height = H;
  env.data.swap(data);
  return true;
}

// ============================================================ OBJ + synthetic Lucy
HittablePtr LoadOBJ(const std::string& path, MaterialPtr mat, std::string& err) {   // obj_loader.go:15-113
  std::ifstream f(path);
  if (!f) { err = "failed to open OBJ file: " + path; return nullptr; }
  std::vector<Point3> verts;
  std::vector<HittablePtr> tris;
  std::string line;
  int ln = 0;
  while (std::getline(f, line)) {
    ++ln;
    std::istringstream ss(line);
    std::string tag;
    if (!(ss >> tag) || tag[0] == '#') continue;
    if (tag == "v") {
      double x, y, z;
      if (!(ss >> x >> y >> z)) { err = "invalid vertex at line " + std::to_string(ln); return nullptr; }
      verts.push_back({x, y, z});
    } else if (tag == "f") {
      std::vector<long> idx;
      std::string tok;
      while (ss >> tok) {
        long i;
        try { i = std::stol(tok.substr(0, tok.find('/'))); } catch (...) {
          err = "invalid face index at line " + std::to_string(ln); return nullptr;
        }
        if (i < 0) i = long(verts.size()) + i + 1;
        idx.push_back(i - 1);
      }
      if (idx.size() < 3) continue;
      for (size_t i = 1; i + 1 < idx.size(); ++i) {
        long a = idx[0], b = idx[i], c = idx[i + 1];
        long nv = long(verts.size());
        if (a < 0 || a >= nv || b < 0 || b >= nv || c < 0 || c >= nv) {
          err = "vertex index out of bounds at line " + std::to_string(ln); return nullptr;
        }
        tris.push_back(NewTriangle(verts[a], verts[b], verts[c], mat));
      }
    }
  }
  return NewBVHNode(tris, 0, tris.size());
}

std::vector<HittablePtr> SyntheticLucyTriangles(int rings, int cols, MaterialPtr mat) {
  // Closed displaced surface: y in [0,1] along the body, radius profile with
  // "wing" and "head" bulges plus deterministic ripples; poles close it.
  std::vector<Point3> V;
  V.reserve(size_t(rings) * cols + 2);
  for (int r = 0; r < rings; ++r) {
    double t = (double(r) + 0.5) / double(rings);   // (0,1)
    double base = 0.18 + 0.22 * std::sin(Pi * t) + 0.10 * std::exp(-std::pow((t - 0.62) / 0.08, 2)) * 2.2 +
                  0.08 * std::exp(-std::pow((t - 0.9) / 0.05, 2));
    for (int c = 0; c < cols; ++c) {
      double a = 2.0 * Pi * double(c) / double(cols);
      double rip = 1.0 + 0.12 * std::sin(3 * a + 9 * t) + 0.06 * std::sin(7 * a - 23 * t) + 0.035 * std::sin(17 * a + 41 * t) +
                   0.02 * std::sin(31 * a - 73 * t);
      double wing = 1.0 + 1.4 * std::exp(-std::pow((t - 0.62) / 0.12, 2)) * std::pow(std::cos(a), 2);
      double rad = base * rip;
      V.push_back({rad * wing * std::cos(a), t + 0.01 * std::sin(5 * a + 13 * t), rad * std::sin(a)});
    }
  }
  const size_t south = V.size();
  V.push_back({0, 0, 0});
  const size_t north = V.size();
  V.push_back({0, 1, 0});
  // fit to Lucy's bounds [-465,-0.025,-267]..[465,1597,267] (scenes.go:765)
  Point3 mn{1e300, 1e300, 1e300}, mx{-1e300, -1e300, -1e300};
  for (auto& p : V) {
    mn.X = std::fmin(mn.X, p.X); mn.Y = std::fmin(mn.Y, p.Y); mn.Z = std::fmin(mn.Z, p.Z);
    mx.X = std::fmax(mx.X, p.X); mx.Y = std::fmax(mx.Y, p.Y); mx.Z = std::fmax(mx.Z, p.Z);
  }
  const double lo[3] = {-465, -0.025, -267}, hi[3] = {465, 1597, 267};
  for (auto& p : V) {
    p.X = lo[0] + (p.X - mn.X) / (mx.X - mn.X) * (hi[0] - lo[0]);
    p.Y = lo[1] + (p.Y - mn.Y) / (mx.Y - mn.Y) * (hi[1] - lo[1]);
    p.Z = lo[2] + (p.Z - mn.Z) / (mx.Z - mn.Z) * (hi[2] - lo[2]);
  }
  std::vector<HittablePtr> T;
  T.reserve(size_t(2) * rings * cols);
  auto at = [&](int r, int c) { return V[size_t(r) * cols + size_t((c % cols + cols) % cols)]; };
  for (int r = 0; r + 1 < rings; ++r)
    for (int c = 0; c < cols; ++c) {
      T.push_back(NewTriangle(at(r, c), at(r + 1, c), at(r + 1, c + 1), mat));
      T.push_back(NewTriangle(at(r, c), at(r + 1, c + 1), at(r, c + 1), mat));
    }
  for (int c = 0; c < cols; ++c) {
    T.push_back(NewTriangle(V[south], at(0, c + 1), at(0, c), mat));
    T.push_back(NewTriangle(V[north], at(rings - 1, c), at(rings - 1, c + 1), mat));
  }
  return T;
}

bool WriteOBJ(const std::string& path, const std::vector<HittablePtr>& tris, std::string& err) {
  FILE* fp = std::fopen(path.c_str(), "w");
  if (!fp) { err = "cannot write " + path; return false; }
  std::fprintf(fp, "# synthetic mesh\n");
  for (const auto& h : tris) {
    auto* t = dynamic_cast<Triangle*>(h.get());
    if (!t) continue;
    std::fprintf(fp, "v %.17g %.17g %.17g\nv %.17g %.17g %.17g\nv %.17g %.17g %.17g\nf -3 -2 -1\n", t->v0.X, t->v0.Y,
                 t->v0.Z, t->v1.X, t->v1.Y, t->v1.Z, t->v2.X, t->v2.Y, t->v2.Z);
  }
  std::fclose(fp);
  return true;
}

// ============================================================ scenes (scenes.go)
static void apply_overrides(Camera& cam, const SceneOptions& o) {
  if (o.width > 0) cam.ImageWidth = o.width;
  if (o.aspect > 0) cam.AspectRatio = o.aspect;
  if (o.spp > 0) cam.SamplesPerPixel = o.spp;
  if (o.max_depth > 0) cam.MaxDepth = o.max_depth;
  cam.Initialize();
}

static Scene simple_scene() {   // scenes.go:172-209
  Scene s;
  s.world = NewHittableList();
  auto ground = NewLambertian({0.8, 0.8, 0.0});
  auto center = NewLambertian({0.1, 0.2, 0.5});
  auto left = NewDielectric(1.5);
  auto bubble = NewDielectric(1.0 / 1.5);
  auto right = NewMetal({0.8, 0.6, 0.2}, 0.0);
  s.world->Add(NewPlane({0, -0.5, -1}, {0, 1, 0}, ground));
  s.world->Add(NewSphere({0, 0, -1}, 0.5, center));
  s.world->Add(NewSphere({-1, 0, -1}, 0.5, left));
  s.world->Add(NewSphere({-1, 0, -1}, 0.4, bubble));
  s.world->Add(NewSphere({1, 0, -1}, 0.5, right));
  s.camera = std::make_shared<Camera>();
  s.camera->SetResolution(400, 16.0 / 9.0).SetQuality(100, 50).SetPosition({0, 0, 2}, {0, 0, -1}, {0, 1, 0})
      .SetLens(90, 0, 10).EnableSkyGradient(true).Build();
  return s;
}

static Scene random_scene(uint64_t seed) {   // scenes.go:30-130 (DefaultSceneConfig)
  SceneRng R(seed);
  Scene s;
  s.world = NewHittableList();
  auto checker = NewCheckerTextureFromColors(0.32, {0.5, 0.5, 0.5}, {0.9, 0.9, 0.9});
  s.world->Add(NewPlane({0, 0, -1}, {0, 1, 0}, NewLambertianTexture(checker)));
  for (int a = -10; a < 10; ++a)
    for (int b = -10; b < 10; ++b) {
      double choose = R.RandomDouble();
      Point3 c{double(a) + 0.9 * R.RandomDouble(), 0.2, 0};
      c.Z = double(b) + 0.9 * R.RandomDouble();
      if (c.Sub({4, 0.2, 0}).Len() > 0.9) {   // addRandomSphere :85-116
        if (choose < 0.3) {
          Color al;
          al.X = R.RandomDouble() * R.RandomDouble();
          al.Y = R.RandomDouble() * R.RandomDouble();
          al.Z = R.RandomDouble() * R.RandomDouble();
          Point3 c2 = c.Add({0, R.Range(0, 0.5), 0});
          s.world->Add(NewMovingSphere(c, c2, 0.2, NewLambertian(al)));
        } else if (choose < 0.6) {
          Color al;
          al.X = 0.5 + R.RandomDouble() * 0.5;
          al.Y = 0.5 + R.RandomDouble() * 0.5;
          al.Z = 0.5 + R.RandomDouble() * 0.5;
          double fuzz = R.RandomDouble() * 0.5;
          s.world->Add(NewSphere(c, 0.2, NewMetal(al, fuzz)));
        } else if (choose < 0.9) {
          s.world->Add(NewSphere(c, 0.2, NewDielectric(1.5)));
        }
      }
    }
  s.world->Add(NewSphere({0, 1, 0}, 1.0, NewDielectric(1.5)));
  s.world->Add(NewSphere({-4, 1, 0}, 1.0, NewLambertian({0.4, 0.2, 0.1})));
  s.world->Add(NewSphere({4, 1, 0}, 1.0, NewMetal({0.7, 0.6, 0.5}, 0.0)));
  s.camera = std::make_shared<Camera>();
  s.camera->SetResolution(1200, 16.0 / 9.0).SetQuality(500, 50).SetPosition({13, 2, 3}, {0, 0, 0}, {0, 1, 0})
      .SetLens(20, 0.6, 10.0).EnableSkyGradient(true).Build();
  return s;
}

static std::shared_ptr<Quad> cornell_walls(HittableList& w, MaterialPtr white, MaterialPtr red, MaterialPtr green,
                                           MaterialPtr light) {   // scenes.go:472-509 / :723-760
  auto area = NewQuad({213, 554, 227}, {130, 0, 0}, {0, 0, 105}, light);
  w.Add(area);
  w.Add(NewQuad({555, 0, 0}, {0, 555, 0}, {0, 0, 555}, green));
  w.Add(NewQuad({0, 0, 0}, {0, 555, 0}, {0, 0, 555}, red));
  w.Add(NewQuad({0, 0, 0}, {555, 0, 0}, {0, 0, 555}, white));
  w.Add(NewQuad({555, 555, 555}, {-555, 0, 0}, {0, 0, -555}, white));
  w.Add(NewQuad({0, 0, 555}, {555, 0, 0}, {0, 555, 0}, white));
  return area;
}

static Scene cornell_scene() {   // scenes.go:463-562
  Scene s;
  s.world = NewHittableList();
  auto white = NewLambertian({0.73, 0.73, 0.73});
  auto red = NewLambertian({0.65, 0.05, 0.05});
  auto green = NewLambertian({0.12, 0.45, 0.15});
  auto light = NewDiffuseLight(NewSolidColor({3, 3, 3}));
  auto area = cornell_walls(*s.world, white, red, green, light);
  auto box1 = Box({0, 0, 0}, {165, 330, 165}, white);
  s.world->Add(Transform().SetScale({1, 1, 1}).SetRotationY(15).SetPosition({265, 0, 295}).Apply(box1));
  auto box2 = Box({0, 0, 0}, {165, 165, 165}, white);
  s.world->Add(Transform().SetScale({1, 1, 1}).SetRotationY(-18).SetPosition({130, 0, 65}).Apply(box2));
  auto fog = Box({0, 0, 0}, {555, 555, 555}, white);
  s.world->Add(NewVolumeFromColor(fog, 0.001, {1, 1, 1}));
  s.camera = std::make_shared<Camera>();
  s.camera->SetResolution(600, 1.0).SetQuality(500, 5).SetPosition({278, 278, -800}, {278, 278, 0}, {0, 1, 0})
      .SetLens(40, 0, 10).SetBackground({0, 0, 0}).AddLight(area).Build();
  return s;
}

static Scene cornell_smoke() {   // scenes.go:820-925
  Scene s;
  s.world = NewHittableList();
  auto white = NewLambertian({0.73, 0.73, 0.73});
  auto red = NewLambertian({0.65, 0.05, 0.05});
  auto green = NewLambertian({0.12, 0.45, 0.15});
  auto light = NewDiffuseLight(NewSolidColor({3, 3, 3}));
  auto area = NewQuad({113, 554, 127}, {330, 0, 0}, {0, 0, 305}, light);
  s.world->Add(area);
  s.world->Add(NewQuad({555, 0, 0}, {0, 555, 0}, {0, 0, 555}, green));
  s.world->Add(NewQuad({0, 0, 0}, {0, 555, 0}, {0, 0, 555}, red));
  s.world->Add(NewQuad({0, 0, 0}, {555, 0, 0}, {0, 0, 555}, white));
  s.world->Add(NewQuad({555, 555, 555}, {-555, 0, 0}, {0, 0, -555}, white));
  s.world->Add(NewQuad({0, 0, 555}, {555, 0, 0}, {0, 555, 0}, white));
  auto b1 = Transform().SetRotationY(15).SetPosition({265, 0, 295}).Apply(Box({0, 0, 0}, {165, 330, 165}, white));
  s.world->Add(NewVolumeFromColor(b1, 0.01, {0, 0, 0}));
  auto b2 = Transform().SetRotationY(-18).SetPosition({130, 0, 65}).Apply(Box({0, 0, 0}, {165, 165, 165}, white));
  s.world->Add(NewVolumeFromColor(b2, 0.01, {1, 1, 1}));
  s.camera = std::make_shared<Camera>();
  s.camera->SetResolution(600, 1.0).SetQuality(150, 5).SetPosition({278, 278, -800}, {278, 278, 0}, {0, 1, 0})
      .SetLens(40, 0, 10).SetBackground({0, 0, 0}).AddLight(area).Build();
  return s;
}

// Test-only variant (RotateX/RotateZ parity): the Cornell room
// with boxes, a pyramid and a sphere under RotateX / RotateZ wrappers built by
// Transform.Apply (Scale -> RotX -> RotY -> RotZ -> Translate,
// transform.go:24-46).  RotateX/RotateZ rotate the ray the same way as their
// bbox (transform.go:201-353, "as written"), so the objects Hit sees are not
// inside the bboxes the world BVH culls with; the reference clips them there
// and so must the device (it keeps the caller's world topology for them).
static Scene cornell_rotations() {
  Scene s;
  s.world = NewHittableList();
  auto white = NewLambertian({0.73, 0.73, 0.73});
  auto red = NewLambertian({0.65, 0.05, 0.05});
  auto green = NewLambertian({0.12, 0.45, 0.15});
  auto light = NewDiffuseLight(NewSolidColor({15, 15, 15}));
  auto area = cornell_walls(*s.world, white, red, green, light);
  auto blue = NewLambertian({0.2, 0.3, 0.8});
  s.world->Add(Transform().SetRotation({30, 0, 0}).SetPosition({120, 80, 220}).Apply(Box({0, 0, 0}, {140, 200, 120}, white)));
  s.world->Add(Transform().SetRotation({0, 0, -25}).SetPosition({360, 40, 300}).Apply(Box({0, 0, 0}, {120, 160, 120}, blue)));
  s.world->Add(Transform().SetScale({1.2, 0.8, 1.0}).SetRotation({15, 40, -10}).SetPosition({280, 260, 150})
                   .Apply(Box({0, 0, 0}, {90, 90, 90}, red)));
  s.world->Add(Transform().SetRotation({-20, 0, 35}).SetPosition({170, 330, 380}).Apply(Pyramid({0, 0, 0}, 110, 130, green)));
  s.world->Add(Transform().SetRotation({0, 0, 50}).SetPosition({430, 300, 200}).Apply(NewSphere({40, 0, 0}, 55, white)));
  s.world->Add(Transform().SetRotation({70, 0, 0}).SetPosition({300, 420, 420}).Apply(NewSphere({0, 0, -30}, 40, blue)));
  s.camera = std::make_shared<Camera>();
  s.camera->SetResolution(600, 1.0).SetQuality(50, 5).SetPosition({278, 278, -800}, {278, 278, 0}, {0, 1, 0})
      .SetLens(40, 0, 10).SetBackground({0, 0, 0}).AddLight(area).Build();
  return s;
}

static bool file_exists(const std::string& p) { struct stat st; return ::stat(p.c_str(), &st) == 0; }

static bool cornell_lucy(const SceneOptions& o, Scene& s, std::string& err) {   // scenes.go:714-817
  s.world = NewHittableList();
  auto white = NewLambertian({0.73, 0.73, 0.73});
  auto red = NewLambertian({0.65, 0.05, 0.05});
  auto green = NewLambertian({0.12, 0.45, 0.15});
  auto light = NewDiffuseLight(NewSolidColor({15, 15, 15}));
  auto area = cornell_walls(*s.world, white, red, green, light);
  auto lucyMat = NewLambertian({0.9, 0.9, 0.9});
  const double scale = 0.15;
  HittablePtr mesh;
  if (!o.obj_path.empty()) {
    mesh = LoadOBJ(o.obj_path, lucyMat, err);
    if (!mesh) return false;
  } else {
    auto tris = SyntheticLucyTriangles(o.lucy_rings, o.lucy_cols, lucyMat);
    mesh = NewBVHNode(tris, 0, tris.size());
  }
  const struct { Vec3 pos; double rot; } P[] = {
      {{150, 0, 150}, 45}, {{400, 0, 150}, 315}, {{150, 0, 400}, 135}, {{400, 0, 400}, 225}, {{278, 0, 278}, 0},
      {{100, 0, 278}, 90}, {{450, 0, 278}, 270}, {{278, 0, 100}, 180}, {{278, 0, 450}, 0},   {{200, 0, 350}, 60}};
  for (const auto& in : P)
    s.world->Add(Transform().SetScale({scale, scale, scale}).SetRotationY(in.rot).SetPosition(in.pos).Apply(mesh));
  s.camera = std::make_shared<Camera>();
  s.camera->SetResolution(600, 1.0).SetQuality(50, 5).SetPosition({278, 278, -800}, {278, 278, 0}, {0, 1, 0})
      .SetLens(40, 0, 10).SetBackground({0, 0, 0}).AddLight(area).Build();
  return true;
}

static bool hdri_scene(const SceneOptions& o, Scene& s, std::string& err, bool with_light) {   // scenes.go:406-458
  s.world = NewHittableList();
  auto glass = NewDielectric(1.5);
  auto mirror = NewMetal({1.0, 1.0, 1.0}, 0.0);
  auto gold = NewMetal({1.0, 0.84, 0.0}, 0.1);
  auto ground = NewLambertianTexture(NewCheckerTextureFromColors(0.5, {0.1, 0.1, 0.1}, {0.9, 0.9, 0.9}));
  s.world->Add(NewPlane({0, 0, 0}, {0, 1, 0}, ground));
  s.world->Add(NewSphere({0, 1, 0}, 1.0, glass));
  s.world->Add(NewSphere({-2.5, 1, 0}, 1.0, mirror));
  s.world->Add(NewSphere({2.5, 1, 0}, 1.0, gold));
  s.world->Add(NewSphere({-1.2, 0.4, 2}, 0.4, glass));
  s.world->Add(NewSphere({1.2, 0.4, 2}, 0.4, glass));
  s.camera = std::make_shared<Camera>();
  auto env = std::make_shared<HDRIEnvironment>();
  std::string dir = o.asset_dir.empty() ? std::string("assets") : o.asset_dir;
  std::string path = dir + "/hdri/abandoned_hall_01_1k.hdr";
  if (!file_exists(path)) { err = "HDRI asset not found: " + path; return false; }
  if (!LoadHDR(path, *env, err)) return false;
  env->SetRotation(0);
  s.camera->Environment = env;
  if (with_light) {
    // Test-only variant: an HDRI AND a quad light, so the
    // sampleHDRILight path (camera.go:565-607) is exercised.
    auto lq = NewQuad({-1, 4, -1}, {2, 0, 0}, {0, 0, 2}, NewDiffuseLightColor({4, 4, 4}));
    s.world->Add(lq);
    s.camera->AddLight(lq);
  }
  s.camera->SetResolution(800, 16.0 / 9.0).SetQuality(200, 20).SetPosition({0, 2.5, 8}, {0, 1, 0}, {0, 1, 0})
      .SetLens(40, 0, 10).SetPhantomHDRI(true).Build();
  return true;
}

static Scene checkered_spheres_scene() {   // scenes.go:132-170
  Scene s;
  s.world = NewHittableList();
  auto checker = NewLambertianTexture(NewCheckerTextureFromColors(0.32, {0.2, 0.3, 0.1}, {0.9, 0.9, 0.9}));
  s.world->Add(NewSphere({0, -10, 0}, 10, checker));
  s.world->Add(NewSphere({0, 10, 0}, 10, checker));
  s.camera = std::make_shared<Camera>();
  s.camera->SetResolution(600, 16.0 / 9.0).SetQuality(100, 50).SetPosition({13, 2, 3}, {0, 0, 0}, {0, 1, 0})
      .SetLens(20, 0, 10).EnableSkyGradient(true).Build();
  return s;
}

static Scene glossy_metal_scene() {   // scenes.go:564-604 (GlossyMetalTest)
  Scene s;
  s.world = NewHittableList();
  s.world->Add(NewPlane({0, 0, 0}, {0, 1, 0}, NewLambertian({0.5, 0.5, 0.5})));
  s.world->Add(NewSphere({-2.5, 1, 0}, 1.0, NewMetal({0.8, 0.6, 0.2}, 0.0)));
  s.world->Add(NewSphere({0, 1, 0}, 1.0, NewMetal({0.8, 0.6, 0.2}, 0.2)));
  s.world->Add(NewSphere({2.5, 1, 0}, 1.0, NewMetal({0.8, 0.6, 0.2}, 0.5)));
  auto area = NewQuad({-2, 5, -2}, {4, 0, 0}, {0, 0, 4}, NewDiffuseLight(NewSolidColor({4, 4, 4})));
  s.world->Add(area);
  s.camera = std::make_shared<Camera>();
  s.camera->SetResolution(640, 16.0 / 9.0).SetQuality(100, 10).SetPosition({0, 2, 10}, {0, 1, 0}, {0, 1, 0})
      .SetLens(40, 0, 10).SetBackground({0, 0, 0}).AddLight(area).Build();
  return s;
}

static Scene cornell_glossy_scene() {   // scenes.go:606-712 (CornellBoxGlossy)
  Scene s;
  s.world = NewHittableList();
  auto white = NewLambertian({0.73, 0.73, 0.73});
  auto red = NewLambertian({0.65, 0.05, 0.05});
  auto green = NewLambertian({0.12, 0.45, 0.15});
  s.world->Add(NewQuad({555, 0, 0}, {0, 555, 0}, {0, 0, 555}, green));
  s.world->Add(NewQuad({0, 0, 0}, {0, 555, 0}, {0, 0, 555}, red));
  s.world->Add(NewQuad({0, 0, 0}, {555, 0, 0}, {0, 0, 555}, white));
  s.world->Add(NewQuad({555, 555, 555}, {-555, 0, 0}, {0, 0, -555}, white));
  s.world->Add(NewQuad({0, 0, 555}, {555, 0, 0}, {0, 555, 0}, white));
  auto area = NewQuad({213, 554, 227}, {130, 0, 0}, {0, 0, 105}, NewDiffuseLight(NewSolidColor({15, 15, 15})));
  s.world->Add(area);
  s.world->Add(NewSphere({150, 100, 400}, 100, NewMetal({1.0, 0.84, 0.0}, 0.05)));
  s.world->Add(NewSphere({278, 100, 400}, 100, NewMetal({1.0, 0.84, 0.0}, 0.15)));
  s.world->Add(NewSphere({410, 100, 400}, 100, NewMetal({0.95, 0.95, 0.98}, 0.25)));
  s.world->Add(NewSphere({278, 130, 180}, 130, NewDielectric(1.5)));
  s.camera = std::make_shared<Camera>();
  s.camera->SetResolution(600, 1.0).SetQuality(200, 5).SetPosition({278, 278, -800}, {278, 200, 200}, {0, 1, 0})
      .SetLens(40, 0, 10).SetBackground({0, 0, 0}).AddLight(area).Build();
  return s;
}

static Scene quads_scene() {   // scenes.go:274-313
  Scene s;
  s.world = NewHittableList();
  auto leftRed = NewLambertian({1.0, 0.2, 0.2});
  auto backGreen = NewLambertian({0.2, 1.0, 0.2});
  auto rightBlue = NewLambertian({0.2, 0.2, 1.0});
  auto upperOrange = NewLambertian({1.0, 0.5, 0.0});
  auto lowerTeal = NewLambertian({0.2, 0.8, 0.8});
  s.world->Add(NewQuad({-3, -2, 5}, {0, 0, -4}, {0, 4, 0}, leftRed));
  s.world->Add(NewQuad({-2, -2, 0}, {4, 0, 0}, {0, 4, 0}, backGreen));
  s.world->Add(NewQuad({3, -2, 1}, {0, 0, 4}, {0, 4, 0}, rightBlue));
  s.world->Add(NewQuad({-2, 3, 1}, {4, 0, 0}, {0, 0, 4}, upperOrange));
  s.world->Add(NewQuad({-2, -3, 5}, {4, 0, 0}, {0, 0, -4}, lowerTeal));
  s.camera = std::make_shared<Camera>();
  s.camera->SetResolution(400, 1.0).SetQuality(100, 50).SetPosition({0, 0, 9}, {0, 0, 0}, {0, 1, 0})
      .SetLens(80, 0, 10).EnableSkyGradient(true).Build();
  return s;
}

static Scene primitives_scene() {   // scenes.go:315-410
  Scene s;
  s.world = NewHittableList();
  auto redMat = NewLambertian({0.8, 0.1, 0.1});
  auto greenMat = NewLambertian({0.1, 0.8, 0.1});
  auto blueMat = NewLambertian({0.1, 0.1, 0.8});
  auto metalMat = NewMetal({1.0, 1.0, 1.0}, 0);
  auto lightMat = NewDiffuseLight(NewSolidColor({2, 2, 2}));
  auto checkerMat = NewLambertianTexture(NewCheckerTextureFromColors(1.0, {0.0, 0.0, 0.0}, {0.9, 0.9, 0.9}));
  s.world->Add(NewPlane({0, -1, 0}, {0, 1, 0}, checkerMat));
  s.world->Add(NewCircle({-5, 0, 0}, {0, 1, 0}, 0.9, redMat));
  s.world->Add(Pyramid({-2.5, -1, 0}, 1.4, 1.8, greenMat));
  s.world->Add(NewSphere({0, 0.6, 0}, 0.8, NewDielectric(1.5)));
  const double cubeX = 2.5, cubeSize = 1.0;
  s.world->Add(Box({cubeX - cubeSize / 2, -1, -cubeSize / 2}, {cubeX + cubeSize / 2, -1 + cubeSize, cubeSize / 2}, blueMat));
  auto areaLight = NewQuad({-2, 5, -2}, {4, 0, 0}, {0, 0, 4}, lightMat);
  s.world->Add(areaLight);
  s.world->Add(NewSphere({5, 0.6, 0}, 0.8, metalMat));
  s.camera = std::make_shared<Camera>();
  s.camera->SetResolution(800, 16.0 / 9.0).SetQuality(300, 25).SetPosition({0, 2, 10}, {0, 0, 0}, {0, 1, 0})
      .SetLens(45, 0, 10).SetBackground({0, 0, 0}).EnableSkyGradient(true).AddLight(areaLight).Build();
  return s;
}

static Scene perlin_scene(uint64_t seed) {   // scenes.go:244-270 (PerlinSpheresScene)
  SceneRng R(seed);
  Scene s;
  s.world = NewHittableList();
  auto pertext = std::make_shared<NoiseTexture>(NewPerlin(R), 4.0);
  auto perlMaterial = NewLambertianTexture(pertext);
  s.world->Add(NewSphere({0, 2, 0}, 2, perlMaterial));
  s.world->Add(NewPlane({0, 0, -1}, {0, 1, 0}, perlMaterial));
  s.camera = std::make_shared<Camera>();
  s.camera->SetResolution(600, 16.0 / 9.0).SetQuality(100, 50).SetPosition({13, 2, -10}, {0, 1.5, 0}, {0, 1, 0})
      .SetLens(20, 0, 10).EnableSkyGradient(true).Build();
  return s;
}

static bool earth_scene(const SceneOptions& o, Scene& s, std::string& err) {   // scenes.go:210-242
  auto img = std::make_shared<ImageData>();
  const std::string dir = o.asset_dir.empty() ? std::string("assets") : o.asset_dir;
  if (!LoadPPM(dir + "/images/earthmap.ppm", *img, err)) return false;
  s.world = NewHittableList();
  auto earthSurface = NewLambertianTexture(std::make_shared<ImageTexture>(img));
  s.world->Add(NewSphere({0, 0, 0}, 2, earthSurface));
  s.camera = std::make_shared<Camera>();
  s.camera->SetResolution(800, 16.0 / 9.0).SetQuality(100, 50).SetPosition({0, 0, 12}, {0, 0, 0}, {0, 1, 0})
      .SetLens(20, 0, 10).EnableSkyGradient(true).Build();
  return true;
}

bool MakeScene(const std::string& name, const SceneOptions& opt, Scene& out, std::string& err) {
  out = Scene{};
  out.name = name;
  if (name == "simple") out = simple_scene();
  else if (name == "random") out = random_scene(opt.seed);
  else if (name == "cornell") out = cornell_scene();
  else if (name == "cornell-smoke") out = cornell_smoke();
  else if (name == "cornell-rotations") out = cornell_rotations();
  else if (name == "cornell-lucy") { if (!cornell_lucy(opt, out, err)) return false; }
  else if (name == "hdri-test") { if (!hdri_scene(opt, out, err, false)) return false; }
  else if (name == "hdri-nee") { if (!hdri_scene(opt, out, err, true)) return false; }
  else if (name == "checkered-spheres") out = checkered_spheres_scene();
  else if (name == "glossy-metal") out = glossy_metal_scene();
  else if (name == "cornell-glossy") out = cornell_glossy_scene();
  else if (name == "quads") out = quads_scene();
  else if (name == "primitives") out = primitives_scene();
  else if (name == "perlin") out = perlin_scene(opt.seed);
  else if (name == "earth") { if (!earth_scene(opt, out, err)) return false; }
  else { err = "unknown scene: " + name; return false; }
  out.name = name;
  apply_overrides(*out.camera, opt);
  return true;
}

}  // namespace rt
