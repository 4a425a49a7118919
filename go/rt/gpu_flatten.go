// gpu_flatten.go — flattens the rt object graph into the rtgpu mirror tables
// (include/rtgpu.h rt_scene_desc / rt_camera_desc).
//
// COMPILE-UNVERIFIED: no Go toolchain in this repository's build image.  The
// file belongs in package rt of byvfx/go-raytracing (copy it to rt/) because
// most fields it reads are unexported (Quad.u, Triangle.v0, BVHNode.left,
// Lambertian.tex, Volume.boundary, ...).  The node layouts (P[] per kind) are
// the ones rtgpu.h documents; tests/test_go_binding.py pins the mirror
// structs' layout against the header.
package rt

import (
	"fmt"
	"math"
	"unsafe"

	"go-raytracing/rtgpu"
)

// gpuFlat is one flattening pass.  Every map memoises by the Go value, so an
// object shared by several parents (the Lucy mesh BVH under ten transforms,
// rt/scenes.go) becomes one node referenced several times, which is what
// lets the library instance it instead of copying it.
type gpuFlat struct {
	scene    rtgpu.Scene
	nodes    map[Hittable]int32
	mats     map[Material]int32
	texs     map[Texture]int32
	perlins  map[*Perlin]int32
	images   map[*ImageLoader]int32
	unsupErr error
}

// errGPUUnsupported marks a Go type the GPU path does not take; the caller
// keeps the CPU BucketRenderer (the same answer rt_scene_upload gives with
// RT_ERR_UNSUPPORTED).
type errGPUUnsupported struct{ what string }

func (e errGPUUnsupported) Error() string { return "gpu path does not support " + e.what }

// FlattenForGPU flattens the world the caller would hand to NewBucketRenderer
// (main.go:77-86) and the camera's lights and environment.
func FlattenForGPU(world Hittable, camera *Camera) (*rtgpu.Scene, error) {
	f := &gpuFlat{
		nodes:   map[Hittable]int32{},
		mats:    map[Material]int32{},
		texs:    map[Texture]int32{},
		perlins: map[*Perlin]int32{},
		images:  map[*ImageLoader]int32{},
	}
	f.scene.Root = f.hittable(world)
	for _, l := range camera.Lights { // camera.go:38
		f.scene.Lights = append(f.scene.Lights, f.hittable(l))
	}
	if env := camera.Environment; env != nil && env.IsValid() { // camera.go:39, hdri.go:66-68
		f.scene.Env = &rtgpu.Environment{
			Image:              imageOf(env.image),
			Rotation:           env.rotation,
			ImportanceSampling: env.useImportanceSampling,
		}
	}
	if f.unsupErr != nil {
		return nil, f.unsupErr
	}
	return &f.scene, nil
}

func v3(v Vec3) [3]float64 { return [3]float64{v.X, v.Y, v.Z} }

func b2i(b bool) int32 {
	if b {
		return 1
	}
	return 0
}

func (f *gpuFlat) unsupported(what string) {
	if f.unsupErr == nil {
		f.unsupErr = errGPUUnsupported{what}
	}
}

// hittable emits one node per concrete Hittable (children first) and
// returns its index.
func (f *gpuFlat) hittable(h Hittable) int32 {
	if i, ok := f.nodes[h]; ok {
		return i
	}
	var n rtgpu.Node
	b := h.BoundingBox()
	n.BBox = [6]float64{b.X.Min, b.X.Max, b.Y.Min, b.Y.Max, b.Z.Min, b.Z.Max}
	n.Material = -1
	switch o := h.(type) {
	case *Sphere: // sphere.go:6-11
		n.Kind, n.Material = rtgpu.KindSphere, f.material(o.Mat)
		c, v := o.Center.Origin(), o.Center.Direction()
		n.P = [16]float64{c.X, c.Y, c.Z, v.X, v.Y, v.Z, o.Radius}
	case *Quad: // quad.go:5-14
		n.Kind, n.Material = rtgpu.KindQuad, f.material(o.mat)
		n.P = [16]float64{o.Q.X, o.Q.Y, o.Q.Z, o.u.X, o.u.Y, o.u.Z, o.v.X, o.v.Y, o.v.Z,
			o.w.X, o.w.Y, o.w.Z, o.normal.X, o.normal.Y, o.normal.Z, o.D}
	case *Triangle: // triangle.go:8-14
		n.Kind, n.Material = rtgpu.KindTriangle, f.material(o.mat)
		n.P = [16]float64{o.v0.X, o.v0.Y, o.v0.Z, o.v1.X, o.v1.Y, o.v1.Z, o.v2.X, o.v2.Y, o.v2.Z,
			o.normal.X, o.normal.Y, o.normal.Z}
	case *Plane: // plane.go:5-10
		n.Kind, n.Material = rtgpu.KindPlane, f.material(o.Mat)
		n.P = [16]float64{o.Point.X, o.Point.Y, o.Point.Z, o.Normal.X, o.Normal.Y, o.Normal.Z}
	case *Circle: // circle.go:5-12
		n.Kind, n.Material = rtgpu.KindCircle, f.material(o.mat)
		n.P = [16]float64{o.center.X, o.center.Y, o.center.Z, o.normal.X, o.normal.Y, o.normal.Z, o.radius, o.D}
	case *HittableList: // hittable_list.go:3-6
		n.Kind = rtgpu.KindList
		n.A, n.B = f.list(o.Objects)
	case *BVHNode: // bvh.go:13-17; the leaf wrapper BVHNode{leaf, leaf} gets A == B
		n.Kind = rtgpu.KindBVHNode
		n.A = f.hittable(o.left)
		n.B = f.hittable(o.right)
	case *BVHLeaf: // bvh.go:21-24
		n.Kind = rtgpu.KindBVHLeaf
		n.A, n.B = f.list(o.objects)
	case *Translate: // transform.go:78-82
		n.Kind, n.A = rtgpu.KindTranslate, f.hittable(o.Obj)
		n.P[0], n.P[1], n.P[2] = o.Offset.X, o.Offset.Y, o.Offset.Z
	case *RotateX: // transform.go:194-199
		n.Kind, n.A = rtgpu.KindRotateX, f.hittable(o.Obj)
		n.P[0], n.P[1] = o.SinTheta, o.CosTheta
	case *RotateY: // transform.go:113-118
		n.Kind, n.A = rtgpu.KindRotateY, f.hittable(o.Obj)
		n.P[0], n.P[1] = o.SinTheta, o.CosTheta
	case *RotateZ: // transform.go:275-280
		n.Kind, n.A = rtgpu.KindRotateZ, f.hittable(o.Obj)
		n.P[0], n.P[1] = o.SinTheta, o.CosTheta
	case *Scale: // transform.go:360-365
		n.Kind, n.A = rtgpu.KindScale, f.hittable(o.Obj)
		n.P = [16]float64{o.Factor.X, o.Factor.Y, o.Factor.Z, o.InvFactor.X, o.InvFactor.Y, o.InvFactor.Z}
	case *Volume: // volume.go:9-13
		n.Kind, n.A = rtgpu.KindVolume, f.hittable(o.boundary)
		n.Material = f.material(o.phaseFunction)
		n.P[0] = o.negInvDensity
	default:
		f.unsupported(fmt.Sprintf("hittable %T", h))
	}
	f.scene.Nodes = append(f.scene.Nodes, n)
	i := int32(len(f.scene.Nodes) - 1)
	f.nodes[h] = i
	return i
}

// list emits the objects, then their indices as one contiguous run of the
// child table: returns (first, count).
func (f *gpuFlat) list(objs []Hittable) (int32, int32) {
	idx := make([]int32, len(objs))
	for k, o := range objs {
		idx[k] = f.hittable(o)
	}
	first := int32(len(f.scene.Children))
	f.scene.Children = append(f.scene.Children, idx...)
	return first, int32(len(idx))
}

func (f *gpuFlat) material(m Material) int32 {
	if m == nil {
		f.unsupported("nil material")
		return -1
	}
	if i, ok := f.mats[m]; ok {
		return i
	}
	var d rtgpu.Material
	switch o := m.(type) {
	case *Lambertian: // material.go:33-35
		d.Kind, d.Texture = rtgpu.MatLambertian, f.texture(o.tex)
	case *Metal: // material.go:86-89 (NewMetal already clamped Fuzz)
		d.Kind, d.Albedo, d.Fuzz = rtgpu.MatMetal, v3(o.Albedo), o.Fuzz
	case *Dielectric: // material.go:146-148
		d.Kind, d.RefractionIndex = rtgpu.MatDielectric, o.RefractionIndex
	case *DiffuseLight: // material.go:202-204
		d.Kind, d.Texture = rtgpu.MatDiffuseLight, f.texture(o.tex)
	case *Isotropic: // material.go:243-245
		d.Kind, d.Texture = rtgpu.MatIsotropic, f.texture(o.tex)
	default:
		f.unsupported(fmt.Sprintf("material %T", m))
	}
	f.scene.Materials = append(f.scene.Materials, d)
	i := int32(len(f.scene.Materials) - 1)
	f.mats[m] = i
	return i
}

func (f *gpuFlat) texture(t Texture) int32 {
	if t == nil {
		f.unsupported("nil texture")
		return -1
	}
	if i, ok := f.texs[t]; ok {
		return i
	}
	d := rtgpu.Texture{Even: -1, Odd: -1, Perlin: -1, Image: -1}
	switch o := t.(type) {
	case *SolidColor: // texture.go:9-11
		d.Kind, d.Albedo = rtgpu.TexSolid, v3(o.Albedo)
	case *CheckerTexture: // texture.go:13-17 (the library takes solid sub-textures)
		d.Kind, d.InvScale = rtgpu.TexChecker, o.invScale
		d.Even, d.Odd = f.texture(o.even), f.texture(o.odd)
	case *NoiseTexture: // texture.go:19-22
		d.Kind, d.Scale, d.Perlin = rtgpu.TexNoise, o.scale, f.perlin(o.noise)
	case *ImageTexture: // image_texture.go:5-7
		d.Kind, d.Image = rtgpu.TexImage, f.image(o.image)
	default:
		f.unsupported(fmt.Sprintf("texture %T", t))
	}
	f.scene.Textures = append(f.scene.Textures, d)
	i := int32(len(f.scene.Textures) - 1)
	f.texs[t] = i
	return i
}

func (f *gpuFlat) perlin(p *Perlin) int32 {
	if i, ok := f.perlins[p]; ok {
		return i
	}
	var d rtgpu.Perlin // noise.go:8-13: the tables NewPerlin drew from math/rand
	for k := 0; k < 256; k++ {
		d.RandVec[k] = v3(p.randvec[k])
		d.PermX[k], d.PermY[k], d.PermZ[k] = int32(p.permX[k]), int32(p.permY[k]), int32(p.permZ[k])
	}
	f.scene.Perlins = append(f.scene.Perlins, d)
	i := int32(len(f.scene.Perlins) - 1)
	f.perlins[p] = i
	return i
}

func (f *gpuFlat) image(img *ImageLoader) int32 {
	if i, ok := f.images[img]; ok {
		return i
	}
	f.scene.Images = append(f.scene.Images, imageOf(img))
	i := int32(len(f.scene.Images) - 1)
	f.images[img] = i
	return i
}

// imageOf views ImageLoader.data ([]Color = []Vec3, three packed float64)
// as the flat rgb array rt_image takes; the library copies it at upload.
func imageOf(img *ImageLoader) rtgpu.Image {
	if img == nil || img.data == nil || img.Width() == 0 || img.Height() == 0 {
		return rtgpu.Image{} // image_loader.go:83-96: Width()/Height() == 0 without data
	}
	rgb := unsafe.Slice((*float64)(unsafe.Pointer(&img.data[0])), 3*len(img.data))
	return rtgpu.Image{Width: img.Width(), Height: img.Height(), RGB: rgb}
}

// GPUCameraDesc is the state Camera.Initialize() leaves (camera.go:286-344);
// the fields after FreeCamera feed GetRay's moving / free camera branch
// (camera.go:390-434).
func GPUCameraDesc(c *Camera) rtgpu.CameraDesc {
	return rtgpu.CameraDesc{
		ImageWidth:       int32(c.ImageWidth),
		ImageHeight:      int32(c.ImageHeight),
		SamplesPerPixel:  int32(c.SamplesPerPixel),
		MaxDepth:         int32(c.MaxDepth),
		Center:           v3(c.center),
		Pixel00:          v3(c.pixel00Loc),
		PixelDeltaU:      v3(c.pixelDeltaU),
		PixelDeltaV:      v3(c.pixelDeltaV),
		DefocusAngle:     c.DefocusAngle,
		DefocusDiskU:     v3(c.defocusDiskU),
		DefocusDiskV:     v3(c.defocusDiskV),
		Background:       v3(c.Background),
		UseSkyGradient:   b2i(c.UseSkyGradient),
		PhantomHDRI:      b2i(c.PhantomHDRI),
		CameraMotion:     b2i(c.CameraMotion),
		FreeCamera:       b2i(c.FreeCamera),
		CenterMotionOrig: v3(c.centerMotion.Origin()),
		CenterMotionDir:  v3(c.centerMotion.Direction()),
		LookAtMotionOrig: v3(c.lookAtMotion.Origin()),
		LookAtMotionDir:  v3(c.lookAtMotion.Direction()),
		Vup:              v3(c.Vup),
		Forward:          v3(c.Forward),
		ViewportWidth:    c.viewportWidth,
		ViewportHeight:   c.viewportHeight,
		FocusDist:        c.FocusDist,
		DefocusRadius:    c.FocusDist * math.Tan(DegreesToRadians(c.DefocusAngle/2)), // camera.go:356
	}
}
