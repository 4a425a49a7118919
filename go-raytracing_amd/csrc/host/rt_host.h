// rt_host.h — C++ host-side mirror of the reference's package rt API surface
// (the part a caller of rt.NewBucketRenderer touches), standing in for the Go
// host because this image has no Go toolchain.  It builds the same object
// graph the Go builders build — same types, same constructors, same
// BoundingBox() values, same NewBVHNode topology — and hands it to the GPU
// through the C-ABI of include/rtgpu.h.  It contains NO CPU rendering path:
// Hit/Scatter run only on the device (render.hip).
//
// Reference files mirrored: vec3.go, interval.go, aabb.go, hittable.go,
// hittable_list.go, sphere.go, quad.go, triangle.go, plane.go, bvh.go,
// transform.go, volume.go, primitives.go, material.go, texture.go, hdri.go,
// image_loader.go (HDR part), obj_loader.go, camera.go (builder +
// Initialize), scenes.go (the five BASELINE scenes + CornellSmoke).
#pragma once
#include <cmath>
#include <cstdint>
#include <limits>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../../include/rtgpu.h"

namespace rt {

constexpr double Pi = 3.1415926535897932385;   // utils.go:10-12
inline double DegreesToRadians(double d) { return d * Pi / 180.0; }

struct Vec3 {
  double X = 0, Y = 0, Z = 0;
  Vec3() = default;
  Vec3(double x, double y, double z) : X(x), Y(y), Z(z) {}
  Vec3 Add(const Vec3& u) const { return {X + u.X, Y + u.Y, Z + u.Z}; }
  Vec3 Sub(const Vec3& u) const { return {X - u.X, Y - u.Y, Z - u.Z}; }
  Vec3 Mult(const Vec3& u) const { return {X * u.X, Y * u.Y, Z * u.Z}; }
  Vec3 Scale(double t) const { return {t * X, t * Y, t * Z}; }
  Vec3 Div(double t) const { return Scale(1 / t); }
  Vec3 Neg() const { return {-X, -Y, -Z}; }
  double Len2() const { return X * X + Y * Y + Z * Z; }
  double Len() const { return std::sqrt(Len2()); }
  Vec3 Unit() const { double l = Len(); return l == 0 ? *this : Div(l); }
};
using Point3 = Vec3;
using Color = Vec3;
inline double Dot(const Vec3& a, const Vec3& b) { return a.X * b.X + a.Y * b.Y + a.Z * b.Z; }
inline Vec3 Cross(const Vec3& a, const Vec3& b) {
  return {a.Y * b.Z - a.Z * b.Y, a.Z * b.X - a.X * b.Z, a.X * b.Y - a.Y * b.X};
}

struct Interval {
  double Min = std::numeric_limits<double>::infinity(), Max = -std::numeric_limits<double>::infinity();
  Interval() = default;
  Interval(double mn, double mx) : Min(mn), Max(mx) {}
  double Size() const { return Max - Min; }
  Interval Expand(double d) const { return {Min - d, Max + d}; }
  Interval Add(double d) const { return {Min + d, Max + d}; }
  static Interval Universe() {
    return {-std::numeric_limits<double>::infinity(), std::numeric_limits<double>::infinity()};
  }
  static Interval Union(const Interval& a, const Interval& b) {   // NewIntervalFromIntervals
    double mn = a.Min, mx = a.Max;
    if (b.Min < a.Min) mn = b.Min;
    if (b.Max > a.Max) mx = b.Max;
    return {mn, mx};
  }
};

struct AABB {
  Interval X, Y, Z;
  static AABB FromIntervals(Interval x, Interval y, Interval z) { AABB b{x, y, z}; b.pad(); return b; }
  static AABB FromPoints(const Point3& a, const Point3& b) {
    AABB r{Interval(std::fmin(a.X, b.X), std::fmax(a.X, b.X)), Interval(std::fmin(a.Y, b.Y), std::fmax(a.Y, b.Y)),
           Interval(std::fmin(a.Z, b.Z), std::fmax(a.Z, b.Z))};
    r.pad();
    return r;
  }
  static AABB FromBoxes(const AABB& a, const AABB& b) {
    return {Interval::Union(a.X, b.X), Interval::Union(a.Y, b.Y), Interval::Union(a.Z, b.Z)};
  }
  void pad() {   // padToMinimums aabb.go:117-128
    const double d = 0.0001;
    if (X.Size() < d) X = X.Expand(d);
    if (Y.Size() < d) Y = Y.Expand(d);
    if (Z.Size() < d) Z = Z.Expand(d);
  }
  AABB Translate(const Vec3& o) const { return FromIntervals(X.Add(o.X), Y.Add(o.Y), Z.Add(o.Z)); }
  int LongestAxis() const {
    double x = X.Size(), y = Y.Size(), z = Z.Size();
    if (x > y && x > z) return 0;
    if (y > z) return 1;
    return 2;
  }
  Vec3 Centroid() const { return {(X.Min + X.Max) * 0.5, (Y.Min + Y.Max) * 0.5, (Z.Min + Z.Max) * 0.5}; }
  void to(double* o) const { o[0] = X.Min; o[1] = X.Max; o[2] = Y.Min; o[3] = Y.Max; o[4] = Z.Min; o[5] = Z.Max; }
};

// ------------------------------------------------------------------ desc emitter
class Emitter;

struct Texture {
  virtual ~Texture() = default;
  virtual int emit(Emitter& e) const = 0;
};
using TexturePtr = std::shared_ptr<Texture>;
struct SolidColor : Texture {
  Color Albedo;
  explicit SolidColor(Color c) : Albedo(c) {}
  int emit(Emitter& e) const override;
};
struct CheckerTexture : Texture {
  double invScale;
  TexturePtr even, odd;
  CheckerTexture(double scale, TexturePtr e, TexturePtr o) : invScale(1.0 / scale), even(std::move(e)), odd(std::move(o)) {}
  int emit(Emitter& e) const override;
};
struct SceneRng;
// Perlin (noise.go:8-29): tables drawn from the scene RNG (the Go code draws
// them from the global math/rand).
struct Perlin {
  Vec3 randvec[256];
  int permX[256], permY[256], permZ[256];
};
std::shared_ptr<Perlin> NewPerlin(SceneRng& rng);
struct NoiseTexture : Texture {   // texture.go:19-28, 81-85
  std::shared_ptr<Perlin> noise;
  double scale;
  NoiseTexture(std::shared_ptr<Perlin> p, double s) : noise(std::move(p)), scale(s) {}
  int emit(Emitter& e) const override;
};
// ImageLoader data (image_loader.go:17-24): rgb after LinearToGamma.
struct ImageData {
  int width = 0, height = 0;
  std::vector<double> rgb;
};
struct ImageTexture : Texture {   // image_texture.go:5-41
  std::shared_ptr<ImageData> image;
  explicit ImageTexture(std::shared_ptr<ImageData> i) : image(std::move(i)) {}
  int emit(Emitter& e) const override;
};
// image_loader.go:45-80 for an 8-bit binary PPM (P6): channel v -> LinearToGamma(v/255)
// (Go: RGBA() 16-bit / 65535 of an 8-bit image).
bool LoadPPM(const std::string& path, ImageData& img, std::string& err);
inline TexturePtr NewSolidColor(Color c) { return std::make_shared<SolidColor>(c); }
inline TexturePtr NewCheckerTextureFromColors(double scale, Color a, Color b) {
  return std::make_shared<CheckerTexture>(scale, NewSolidColor(a), NewSolidColor(b));
}

struct Material {
  virtual ~Material() = default;
  virtual int emit(Emitter& e) const = 0;
};
using MaterialPtr = std::shared_ptr<Material>;
struct Lambertian : Material { TexturePtr tex; explicit Lambertian(TexturePtr t) : tex(std::move(t)) {} int emit(Emitter& e) const override; };
struct Metal : Material { Color Albedo; double Fuzz; Metal(Color a, double f) : Albedo(a), Fuzz(f > 1 ? 1 : f) {} int emit(Emitter& e) const override; };
struct Dielectric : Material { double RefractionIndex; explicit Dielectric(double r) : RefractionIndex(r) {} int emit(Emitter& e) const override; };
struct DiffuseLight : Material { TexturePtr tex; explicit DiffuseLight(TexturePtr t) : tex(std::move(t)) {} int emit(Emitter& e) const override; };
struct Isotropic : Material { TexturePtr tex; explicit Isotropic(TexturePtr t) : tex(std::move(t)) {} int emit(Emitter& e) const override; };
inline MaterialPtr NewLambertian(Color c) { return std::make_shared<Lambertian>(NewSolidColor(c)); }
inline MaterialPtr NewLambertianTexture(TexturePtr t) { return std::make_shared<Lambertian>(std::move(t)); }
inline MaterialPtr NewMetal(Color c, double f) { return std::make_shared<Metal>(c, f); }
inline MaterialPtr NewDielectric(double r) { return std::make_shared<Dielectric>(r); }
inline MaterialPtr NewDiffuseLight(TexturePtr t) { return std::make_shared<DiffuseLight>(std::move(t)); }
inline MaterialPtr NewDiffuseLightColor(Color c) { return std::make_shared<DiffuseLight>(NewSolidColor(c)); }

// ------------------------------------------------------------------ hittables
struct Hittable {
  virtual ~Hittable() = default;
  virtual AABB BoundingBox() const = 0;
  virtual int emit(Emitter& e) const = 0;
};
using HittablePtr = std::shared_ptr<Hittable>;

struct Sphere : Hittable {   // sphere.go
  Point3 c0; Vec3 vel; double Radius; MaterialPtr Mat; AABB bbox;
  AABB BoundingBox() const override { return bbox; }
  int emit(Emitter& e) const override;
};
HittablePtr NewSphere(Point3 c, double r, MaterialPtr m);
HittablePtr NewMovingSphere(Point3 c1, Point3 c2, double r, MaterialPtr m);

struct Quad : Hittable {     // quad.go
  Point3 Q; Vec3 u, v, w, normal; double D; MaterialPtr mat; AABB bbox;
  AABB BoundingBox() const override { return bbox; }
  int emit(Emitter& e) const override;
};
std::shared_ptr<Quad> NewQuad(Point3 Q, Vec3 u, Vec3 v, MaterialPtr m);

struct Triangle : Hittable { // triangle.go
  Point3 v0, v1, v2; Vec3 normal; MaterialPtr mat; AABB bbox;
  AABB BoundingBox() const override { return bbox; }
  int emit(Emitter& e) const override;
};
HittablePtr NewTriangle(Point3 a, Point3 b, Point3 c, MaterialPtr m);

struct Plane : Hittable {    // plane.go
  Point3 Point; Vec3 Normal; MaterialPtr Mat; AABB bbox;
  AABB BoundingBox() const override { return bbox; }
  int emit(Emitter& e) const override;
};
HittablePtr NewPlane(Point3 p, Vec3 n, MaterialPtr m);

struct Circle : Hittable {   // circle.go
  Point3 center; Vec3 normal; double radius, D; MaterialPtr mat; AABB bbox;
  AABB BoundingBox() const override { return bbox; }
  int emit(Emitter& e) const override;
};
HittablePtr NewCircle(Point3 c, Vec3 n, double r, MaterialPtr m);

struct HittableList : Hittable {
  std::vector<HittablePtr> Objects;
  AABB bbox{Interval(), Interval(), Interval()};
  void Add(HittablePtr o) { bbox = AABB::FromBoxes(bbox, o->BoundingBox()); Objects.push_back(std::move(o)); }
  AABB BoundingBox() const override { return bbox; }
  int emit(Emitter& e) const override;
};
using HittableListPtr = std::shared_ptr<HittableList>;
inline HittableListPtr NewHittableList() { return std::make_shared<HittableList>(); }

struct BVHLeaf : Hittable {
  std::vector<HittablePtr> objects; AABB bbox;
  AABB BoundingBox() const override { return bbox; }
  int emit(Emitter& e) const override;
};
struct BVHNode : Hittable {
  HittablePtr left, right; AABB bbox;
  AABB BoundingBox() const override { return bbox; }
  int emit(Emitter& e) const override;
};
// bvh.go:64-217 (stable sort; NaN centroids ordered first).
std::shared_ptr<BVHNode> NewBVHNode(const std::vector<HittablePtr>& objects, size_t start, size_t end);
std::shared_ptr<BVHNode> NewBVHNodeFromList(const HittableList& list);

struct Translate : Hittable { HittablePtr Obj; Vec3 Offset; AABB bbox; AABB BoundingBox() const override { return bbox; } int emit(Emitter& e) const override; };
struct Rotate : Hittable {   // RotateX / RotateY / RotateZ
  int axis; HittablePtr Obj; double SinTheta, CosTheta; AABB bbox;
  AABB BoundingBox() const override { return bbox; }
  int emit(Emitter& e) const override;
};
struct ScaleH : Hittable { HittablePtr Obj; Vec3 Factor, InvFactor; AABB bbox; AABB BoundingBox() const override { return bbox; } int emit(Emitter& e) const override; };
HittablePtr NewTranslate(HittablePtr o, Vec3 off);
HittablePtr Rx(HittablePtr o, double deg);
HittablePtr Ry(HittablePtr o, double deg);
HittablePtr Rz(HittablePtr o, double deg);
HittablePtr NewScale(HittablePtr o, Vec3 f);

struct Transform {           // transform.go:9-71
  Vec3 Scale{1, 1, 1}, Rotation{0, 0, 0}, Position{0, 0, 0};
  Transform& SetScale(Vec3 s) { Scale = s; return *this; }
  Transform& SetRotationY(double a) { Rotation.Y = a; return *this; }
  Transform& SetRotation(Vec3 r) { Rotation = r; return *this; }
  Transform& SetPosition(Vec3 p) { Position = p; return *this; }
  HittablePtr Apply(HittablePtr obj) const;
};

struct Volume : Hittable {   // volume.go
  HittablePtr boundary; double negInvDensity; MaterialPtr phase;
  AABB BoundingBox() const override { return boundary->BoundingBox(); }
  int emit(Emitter& e) const override;
};
HittablePtr NewVolumeFromColor(HittablePtr boundary, double density, Color albedo);

HittablePtr Box(Point3 a, Point3 b, MaterialPtr m);   // primitives.go:5-37
HittablePtr Pyramid(Point3 baseCenter, double baseSize, double height, MaterialPtr m);   // primitives.go:39-80

// ------------------------------------------------------------------ HDRI
struct HDRIEnvironment {     // hdri.go:13-26 (distribution built on upload)
  int width = 0, height = 0;
  std::vector<double> data;  // ImageLoader.data, rgb
  double rotation = 0;
  bool useImportanceSampling = true;
  bool IsValid() const { return !data.empty(); }
  void SetRotation(double deg) { rotation = deg * Pi / 180.0; }
};
// image_loader.go:165-383 (Radiance RGBE, new RLE + flat scanlines).
bool LoadHDR(const std::string& path, HDRIEnvironment& env, std::string& err);

// ------------------------------------------------------------------ camera
struct Camera {              // camera.go:18-57, NewCamera :63-83
  double AspectRatio = 1.0;
  int ImageWidth = 800, ImageHeight = 0, SamplesPerPixel = 10, MaxDepth = 50;
  double Vfov = 90;
  Point3 LookFrom{0, 0, 0}, LookAt{0, 0, -1};
  Vec3 Vup{0, 1, 0};
  Point3 LookFrom2{0, 0, 0}, LookAt2{0, 0, 0};
  Vec3 Forward{0, 0, -1};
  double DefocusAngle = 0, FocusDist = 1;
  bool CameraMotion = false, FreeCamera = false, UseSkyGradient = false, PhantomHDRI = false;
  Color Background{0, 0, 0};
  std::vector<HittablePtr> Lights;
  std::shared_ptr<HDRIEnvironment> Environment;
  // Initialize() outputs
  Point3 center, pixel00Loc; Vec3 pixelDeltaU, pixelDeltaV, u, v, w, defocusDiskU, defocusDiskV;
  Point3 centerMotionOrig, lookAtMotionOrig; Vec3 centerMotionDir, lookAtMotionDir;
  double viewportHeight = 0, viewportWidth = 0;
  double pixelsSamplesScale = 0;

  Camera& SetResolution(int width, double aspect) { ImageWidth = width; AspectRatio = aspect; return *this; }
  Camera& SetQuality(int spp, int depth) { SamplesPerPixel = spp; MaxDepth = depth; return *this; }
  Camera& SetPosition(Point3 from, Point3 at, Vec3 up) { LookFrom = from; LookAt = at; Vup = up; return *this; }
  Camera& SetLens(double vfov, double defocus, double focus) { Vfov = vfov; DefocusAngle = defocus; FocusDist = focus; return *this; }
  Camera& SetBackground(Color c) { Background = c; return *this; }
  Camera& EnableSkyGradient(bool e) { UseSkyGradient = e; return *this; }
  Camera& SetPhantomHDRI(bool p) { PhantomHDRI = p; return *this; }
  Camera& AddLight(HittablePtr l) { Lights.push_back(std::move(l)); return *this; }
  Camera& SetMotion(Point3 from2, Point3 at2) { LookFrom2 = from2; LookAt2 = at2; CameraMotion = true; return *this; }
  Camera& EnableFreeCamera(Point3 pos, Vec3 fwd, Vec3 up) {   // camera.go:226-232
    LookFrom = pos; Forward = fwd.Unit(); Vup = up.Unit(); FreeCamera = true; return *this;
  }
  Camera& Build() { Initialize(); return *this; }
  void Initialize();         // camera.go:286-344
  rt_camera_desc desc() const;
};
using CameraPtr = std::shared_ptr<Camera>;

// ------------------------------------------------------------------ OBJ + mesh
// obj_loader.go:15-113: v/f records, fan triangulation, negative indices,
// returns the mesh BVH (NewBVHNode over the triangles).
HittablePtr LoadOBJ(const std::string& path, MaterialPtr mat, std::string& err);
// Deterministic synthetic stand-in for the absent Lucy mesh:
// a displaced closed surface of `rings`x`cols` vertices + 2 poles
// (2*rings*cols triangles), fitted to Lucy's bounds (scenes.go:765).
std::vector<HittablePtr> SyntheticLucyTriangles(int rings, int cols, MaterialPtr mat);
bool WriteOBJ(const std::string& path, const std::vector<HittablePtr>& tris, std::string& err);

// ------------------------------------------------------------------ scenes
struct SceneOptions {
  uint64_t seed = 0x5EED;       // RandomScene generator seed
  int width = 0;                // 0: scene default
  double aspect = 0;            // 0: scene default
  int spp = 0, max_depth = 0;   // 0: scene default
  std::string asset_dir;        // where assets/hdri, assets/models live
  std::string obj_path;         // Lucy OBJ override (real mesh)
  int lucy_rings = 350, lucy_cols = 400;   // synthetic Lucy resolution
};
struct Scene {
  HittableListPtr world;
  CameraPtr camera;
  std::string name;
};
// Deterministic replacement for the global math/rand used by scenes.go.
struct SceneRng {
  uint64_t s;
  explicit SceneRng(uint64_t seed) : s(seed) {}
  double RandomDouble() {      // splitmix64 -> [0,1) with 53 bits
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return double(z >> 11) * 0x1p-53;
  }
  double Range(double mn, double mx) { return mn + (mx - mn) * RandomDouble(); }
};
bool MakeScene(const std::string& name, const SceneOptions& opt, Scene& out, std::string& err);

// ------------------------------------------------------------------ emitter
class Emitter {
 public:
  std::vector<rt_hittable> hittables;
  std::vector<int32_t> children;
  std::vector<rt_material> materials;
  std::vector<rt_texture> textures;
  std::vector<int32_t> lights;
  std::vector<rt_image> images;
  std::vector<rt_perlin> perlins;
  rt_environment env{};
  std::vector<double> env_rgb;
  std::map<const void*, int> memo;
  int root = -1;

  int add(const rt_hittable& h) { hittables.push_back(h); return int(hittables.size()) - 1; }
  bool seen(const void* p, int& idx) const { auto it = memo.find(p); if (it == memo.end()) return false; idx = it->second; return true; }
  int emit_material(const MaterialPtr& m) {
    int i; if (seen(m.get(), i)) return i;
    i = m->emit(*this); memo[m.get()] = i; return i;
  }
  int emit_texture(const TexturePtr& t) {
    int i; if (seen(t.get(), i)) return i;
    i = t->emit(*this); memo[t.get()] = i; return i;
  }
  int emit_hittable(const HittablePtr& h) {
    int i; if (seen(h.get(), i)) return i;
    i = h->emit(*this); memo[h.get()] = i; return i;
  }
  // The world handed to NewBucketRenderer (main.go:77 wraps it in a BVH).
  void build(const HittablePtr& world, const Camera& cam);
  rt_scene_desc desc() const;
};

}  // namespace rt
