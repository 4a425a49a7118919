// Package rtgpu is the cgo binding of librtgpu.so (include/rtgpu.h), the
// MI355X path tracer that replaces the per-pixel loop of rt.BucketRenderer
// (rt/bucket_renderer.go:257-301 -> rt/camera.go:368-518).
//
// COMPILE-UNVERIFIED: the build image of this repository has no Go toolchain.
// The struct layouts below are pinned against include/rtgpu.h by
// tests/test_go_binding.py (gcc offsetof vs. the Go field list parsed from
// this file); everything else is reviewed, not compiled.
//
// Install (see INTEGRATION.md §2): copy this directory to <go-raytracing>/rtgpu
// and link the repository's headers and library next to it:
//
//	ln -s /path/to/repo/include rtgpu/include
//	ln -s /path/to/repo/go-raytracing_amd/lib rtgpu/lib
//
// Package rt never sees a C type: it fills the pointer-free mirror structs
// declared here (Node, Material, Texture, Perlin, CameraDesc, Bucket) and
// this package passes them across the boundary.  The library copies every
// array before rt_scene_upload / rt_render return and keeps no caller
// memory, so the Go memory is pinned only for the duration of one call.
package rtgpu

/*
#cgo CFLAGS: -I${SRCDIR}/include
#cgo LDFLAGS: -L${SRCDIR}/lib -lrtgpu -Wl,-rpath,${SRCDIR}/lib
#include <stdlib.h>
#include "rtgpu.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"runtime"
	"unsafe"
)

// ABIVersion is the RT_ABI_VERSION this binding was written against.
const ABIVersion = 8 // RT_ABI_VERSION

// Hittable kinds (enum rt_hittable_kind).
const (
	KindSphere    int32 = 1  // RT_SPHERE
	KindQuad      int32 = 2  // RT_QUAD
	KindTriangle  int32 = 3  // RT_TRIANGLE
	KindPlane     int32 = 4  // RT_PLANE
	KindList      int32 = 5  // RT_LIST
	KindBVHNode   int32 = 6  // RT_BVH_NODE
	KindBVHLeaf   int32 = 7  // RT_BVH_LEAF
	KindTranslate int32 = 8  // RT_TRANSLATE
	KindRotateX   int32 = 9  // RT_ROTATE_X
	KindRotateY   int32 = 10 // RT_ROTATE_Y
	KindRotateZ   int32 = 11 // RT_ROTATE_Z
	KindScale     int32 = 12 // RT_SCALE
	KindVolume    int32 = 13 // RT_VOLUME
	KindCircle    int32 = 14 // RT_CIRCLE
)

// Material kinds (enum rt_material_kind).
const (
	MatLambertian   int32 = 1 // RT_LAMBERTIAN
	MatMetal        int32 = 2 // RT_METAL
	MatDielectric   int32 = 3 // RT_DIELECTRIC
	MatDiffuseLight int32 = 4 // RT_DIFFUSE_LIGHT
	MatIsotropic    int32 = 5 // RT_ISOTROPIC
)

// Texture kinds (enum rt_texture_kind).
const (
	TexSolid   int32 = 1 // RT_TEX_SOLID
	TexChecker int32 = 2 // RT_TEX_CHECKER
	TexNoise   int32 = 3 // RT_TEX_NOISE
	TexImage   int32 = 4 // RT_TEX_IMAGE
)

// Status codes (enum rt_status).
const (
	StatusOK          = 0  // RT_OK
	StatusInvalid     = -1 // RT_ERR_INVALID
	StatusUnsupported = -2 // RT_ERR_UNSUPPORTED
	StatusHIP         = -3 // RT_ERR_HIP
	StatusOOM         = -4 // RT_ERR_OOM
	StatusNoScene     = -5 // RT_ERR_NO_SCENE
	StatusDevice      = -6 // RT_ERR_DEVICE
)

// Context options (rt_ctx_set_option).
const (
	OptBLASBuilder  int32 = 1 // RT_OPT_BLAS_BUILDER
	OptTLASBuilder  int32 = 2 // RT_OPT_TLAS_BUILDER
	OptNodeFormat   int32 = 3 // RT_OPT_NODE_FORMAT
	OptBatchSlots   int32 = 4 // RT_OPT_BATCH_SLOTS
	OptRefill       int32 = 5 // RT_OPT_REFILL
	OptMaxBlocks    int32 = 6 // RT_OPT_MAX_BLOCKS
	OptStreams      int32 = 7 // RT_OPT_STREAMS
	OptVolumes      int32 = 8 // RT_OPT_VOLUMES
	VolumesLifted   int32 = 0 // RT_VOLUMES_LIFTED
	VolumesInBVH    int32 = 1 // RT_VOLUMES_IN_BVH
	OptBVH4Collapse int32 = 9 // RT_OPT_BVH4_COLLAPSE
	CollapseSAH     int32 = 0 // RT_COLLAPSE_SAH
	CollapseGreedy  int32 = 1 // RT_COLLAPSE_GREEDY
	BuildReference  int32 = 0 // RT_BLAS_REFERENCE
	BuildSAH        int32 = 1 // RT_BLAS_SAH
	BuildDevice     int32 = 2 // RT_BLAS_DEVICE
	NodesFP32       int32 = 0 // RT_NODES_FP32
	NodesQuant8     int32 = 1 // RT_NODES_QUANT8
	NodesWide8      int32 = 2 // RT_NODES_WIDE8
	OptDealing      int32 = 10 // RT_OPT_DEALING
	OptDealFirst    int32 = 11 // RT_OPT_DEAL_FIRST
	OptTail         int32 = 12 // RT_OPT_TAIL
	OptOverlap      int32 = 13 // RT_OPT_OVERLAP
	DealStatic      int32 = 0  // RT_DEAL_STATIC
	DealDynamic     int32 = 1  // RT_DEAL_DYNAMIC
)

// Node mirrors rt_hittable: one node per concrete rt.Hittable.  P holds the
// kind's float64 fields in the order rtgpu.h documents per kind.
//
//rtgpu:mirror rt_hittable
type Node struct {
	Kind     int32       `c:"kind"`
	Material int32       `c:"material"`
	A        int32       `c:"a"`
	B        int32       `c:"b"`
	BBox     [6]float64  `c:"bbox"`
	P        [16]float64 `c:"p"`
}

// Material mirrors rt_material.
//
//rtgpu:mirror rt_material
type Material struct {
	Kind            int32      `c:"kind"`
	Texture         int32      `c:"texture"`
	Albedo          [3]float64 `c:"albedo"`
	Fuzz            float64    `c:"fuzz"`
	RefractionIndex float64    `c:"refraction_index"`
}

// Texture mirrors rt_texture (the 4-byte hole after Odd is C's padding).
//
//rtgpu:mirror rt_texture
type Texture struct {
	Kind     int32      `c:"kind"`
	Even     int32      `c:"even"`
	Odd      int32      `c:"odd"`
	_        int32      `c:"-"`
	Albedo   [3]float64 `c:"albedo"`
	InvScale float64    `c:"inv_scale"`
	Scale    float64    `c:"scale"`
	Perlin   int32      `c:"perlin"`
	Image    int32      `c:"image"`
}

// Perlin mirrors rt_perlin: the tables NewPerlin drew (rt/noise.go:8-13).
//
//rtgpu:mirror rt_perlin
type Perlin struct {
	RandVec [256][3]float64 `c:"randvec"`
	PermX   [256]int32      `c:"perm_x"`
	PermY   [256]int32      `c:"perm_y"`
	PermZ   [256]int32      `c:"perm_z"`
}

// CameraDesc mirrors rt_camera_desc: the state Camera.Initialize leaves
// (rt/camera.go:286-344).
//
//rtgpu:mirror rt_camera_desc
type CameraDesc struct {
	ImageWidth       int32      `c:"image_width"`
	ImageHeight      int32      `c:"image_height"`
	SamplesPerPixel  int32      `c:"samples_per_pixel"`
	MaxDepth         int32      `c:"max_depth"`
	Center           [3]float64 `c:"center"`
	Pixel00          [3]float64 `c:"pixel00"`
	PixelDeltaU      [3]float64 `c:"pixel_delta_u"`
	PixelDeltaV      [3]float64 `c:"pixel_delta_v"`
	DefocusAngle     float64    `c:"defocus_angle"`
	DefocusDiskU     [3]float64 `c:"defocus_disk_u"`
	DefocusDiskV     [3]float64 `c:"defocus_disk_v"`
	Background       [3]float64 `c:"background"`
	UseSkyGradient   int32      `c:"use_sky_gradient"`
	PhantomHDRI      int32      `c:"phantom_hdri"`
	CameraMotion     int32      `c:"camera_motion"`
	FreeCamera       int32      `c:"free_camera"`
	CenterMotionOrig [3]float64 `c:"center_motion_orig"`
	CenterMotionDir  [3]float64 `c:"center_motion_dir"`
	LookAtMotionOrig [3]float64 `c:"look_at_motion_orig"`
	LookAtMotionDir  [3]float64 `c:"look_at_motion_dir"`
	Vup              [3]float64 `c:"vup"`
	Forward          [3]float64 `c:"forward"`
	ViewportWidth    float64    `c:"viewport_width"`
	ViewportHeight   float64    `c:"viewport_height"`
	FocusDist        float64    `c:"focus_dist"`
	DefocusRadius    float64    `c:"defocus_radius"`
}

// Bucket mirrors rt_bucket (rt.Bucket with int32 fields).
//
//rtgpu:mirror rt_bucket
type Bucket struct {
	X      int32 `c:"x"`
	Y      int32 `c:"y"`
	Width  int32 `c:"width"`
	Height int32 `c:"height"`
}

// Stats mirrors rt_stats.
//
//rtgpu:mirror rt_stats
type Stats struct {
	KernelMs float64 `c:"kernel_ms"`
	Samples  uint64  `c:"samples"`
}

// SceneInfo mirrors rt_scene_info.
//
//rtgpu:mirror rt_scene_info
type SceneInfo struct {
	Nodes       int32 `c:"nodes"`
	Leaves      int32 `c:"leaves"`
	Refs        int32 `c:"refs"`
	Spheres     int32 `c:"spheres"`
	Quads       int32 `c:"quads"`
	Triangles   int32 `c:"triangles"`
	Planes      int32 `c:"planes"`
	Instances   int32 `c:"instances"`
	BLASes      int32 `c:"blases"`
	Volumes     int32 `c:"volumes"`
	Materials   int32 `c:"materials"`
	Textures    int32 `c:"textures"`
	Lights      int32 `c:"lights"`
	StackNeeded int32 `c:"stack_needed"`
	TLASDepth   int32 `c:"tlas_depth"`
	BLASDepth   int32 `c:"blas_depth"`
	DeviceBytes int64 `c:"device_bytes"`
	NodeFormat  int32 `c:"node_format"`
	Nodes8      int32 `c:"nodes8"`
}

// Image is an ImageLoader's pixels (rt/image_loader.go:17-24): linear
// float64 rgb, row-major, Width*Height*3 values.  Width == 0 is an
// ImageLoader without data (ImageTexture.Value returns cyan).
type Image struct {
	Width, Height int
	RGB           []float64
}

// Environment is an HDRIEnvironment (rt/hdri.go:13-26).  The library builds
// the importance-sampling tables itself (hdri.go:145-224).
type Environment struct {
	Image              Image
	Rotation           float64 // radians
	ImportanceSampling bool
}

// Scene is the flattened object graph rt_scene_upload takes.
type Scene struct {
	Nodes     []Node
	Children  []int32 // child index table of KindList / KindBVHLeaf nodes
	Root      int32
	Materials []Material
	Textures  []Texture
	Lights    []int32 // Camera.Lights as node indices
	Env       *Environment
	Images    []Image
	Perlins   []Perlin
}

// Error is a non-OK status of an entry point with rt_last_error's message.
type Error struct {
	Status  int
	Message string
}

func (e *Error) Error() string { return fmt.Sprintf("rtgpu: status %d: %s", e.Status, e.Message) }

// IsUnsupported reports whether err is RT_ERR_UNSUPPORTED: a Go type or
// nesting the GPU path does not take; the caller renders on the CPU.
func IsUnsupported(err error) bool {
	var e *Error
	return errors.As(err, &e) && e.Status == StatusUnsupported
}

// Ctx is a context over one or several devices (rt_ctx).  Not safe for
// concurrent use.
type Ctx struct {
	p *C.rt_ctx
}

// DeviceCount is the number of visible HIP devices (rt_device_count).
func DeviceCount() (int, error) {
	var n C.int32_t
	if rc := C.rt_device_count(&n); rc != C.RT_OK {
		return 0, &Error{int(rc), "rt_device_count failed"}
	}
	return int(n), nil
}

// New creates a context after checking the ABI: on HIP device devices[0]
// alone, or over every listed device (rt_ctx_create_multi: each render deals
// its buckets round-robin over them, like bucket_renderer.go:193-213's
// worker pool with one GPU per worker).  No devices: every visible device.
func New(devices ...int) (*Ctx, error) {
	if v := int(C.rt_abi_version()); v != ABIVersion {
		return nil, &Error{StatusInvalid, fmt.Sprintf("librtgpu ABI %d, binding expects %d", v, ABIVersion)}
	}
	if len(devices) == 0 {
		n, err := DeviceCount()
		if err != nil {
			return nil, err
		}
		if n == 0 {
			return nil, &Error{StatusHIP, "no HIP device"}
		}
		for d := 0; d < n; d++ {
			devices = append(devices, d)
		}
	}
	var p *C.rt_ctx
	if len(devices) == 1 {
		if rc := C.rt_ctx_create(C.int(devices[0]), &p); rc != C.RT_OK {
			return nil, &Error{int(rc), "rt_ctx_create failed"}
		}
		return &Ctx{p: p}, nil
	}
	list := (*C.int32_t)(C.calloc(C.size_t(len(devices)), C.sizeof_int32_t))
	defer C.free(unsafe.Pointer(list))
	ids := unsafe.Slice(list, len(devices))
	for i, d := range devices {
		ids[i] = C.int32_t(d)
	}
	if rc := C.rt_ctx_create_multi(list, C.int32_t(len(devices)), &p); rc != C.RT_OK {
		return nil, &Error{int(rc), "rt_ctx_create_multi failed"}
	}
	return &Ctx{p: p}, nil
}

// NumDevices is the number of devices the context renders on.
func (c *Ctx) NumDevices() int { return int(C.rt_ctx_num_devices(c.p)) }

// LastDealing reports the last multi-device render's split: the tiles each
// device rendered and the runs it claimed (rt_last_dealing).
func (c *Ctx) LastDealing() (tiles, runs []int32, err error) {
	n := c.NumDevices()
	tiles, runs = make([]int32, n), make([]int32, n)
	if n == 0 {
		return tiles, runs, nil
	}
	err = c.check(C.rt_last_dealing(c.p, (*C.int32_t)(unsafe.Pointer(&tiles[0])),
		(*C.int32_t)(unsafe.Pointer(&runs[0])), C.int32_t(n)))
	return tiles, runs, err
}

// Close releases the context and its device memory.
func (c *Ctx) Close() {
	if c.p != nil {
		C.rt_ctx_destroy(c.p)
		c.p = nil
	}
}

func (c *Ctx) check(rc C.int) error {
	if rc == C.RT_OK {
		return nil
	}
	return &Error{int(rc), C.GoString(C.rt_last_error(c.p))}
}

// SetOption sets a context option (OptBLASBuilder / OptTLASBuilder /
// OptNodeFormat / OptVolumes / OptBVH4Collapse, or a schedule option: OptBatchSlots, OptRefill,
// OptMaxBlocks, OptStreams, OptDealing, OptDealFirst, which never change
// the image).  The scene
// options take effect at the next Upload, the schedule options at the next
// render.
func (c *Ctx) SetOption(key, value int32) error {
	return c.check(C.rt_ctx_set_option(c.p, C.int32_t(key), C.int32_t(value)))
}

// SetMeshBuilder chooses how mesh BVHs are laid out on the device
// (BuildReference / BuildSAH / BuildDevice).
func (c *Ctx) SetMeshBuilder(b int32) error { return c.SetOption(OptBLASBuilder, b) }

// Upload flattens and copies the scene to the device.  The descriptor and
// its small C-side arrays (rt_image, rt_environment) hold Go pointers that
// are pinned for the call only: the library copies everything before
// returning (rtgpu.h: "C never retains caller memory").
func (c *Ctx) Upload(s *Scene) error {
	if len(s.Nodes) == 0 {
		return &Error{StatusInvalid, "empty scene"}
	}
	var pin runtime.Pinner
	defer pin.Unpin()

	d := (*C.rt_scene_desc)(C.calloc(1, C.sizeof_rt_scene_desc))
	defer C.free(unsafe.Pointer(d))

	pin.Pin(&s.Nodes[0])
	d.hittables = (*C.rt_hittable)(unsafe.Pointer(&s.Nodes[0]))
	d.num_hittables = C.int32_t(len(s.Nodes))
	if len(s.Children) > 0 {
		pin.Pin(&s.Children[0])
		d.children = (*C.int32_t)(unsafe.Pointer(&s.Children[0]))
	}
	d.num_children = C.int32_t(len(s.Children))
	d.root = C.int32_t(s.Root)
	if len(s.Materials) > 0 {
		pin.Pin(&s.Materials[0])
		d.materials = (*C.rt_material)(unsafe.Pointer(&s.Materials[0]))
	}
	d.num_materials = C.int32_t(len(s.Materials))
	if len(s.Textures) > 0 {
		pin.Pin(&s.Textures[0])
		d.textures = (*C.rt_texture)(unsafe.Pointer(&s.Textures[0]))
	}
	d.num_textures = C.int32_t(len(s.Textures))
	if len(s.Lights) > 0 {
		pin.Pin(&s.Lights[0])
		d.lights = (*C.int32_t)(unsafe.Pointer(&s.Lights[0]))
	}
	d.num_lights = C.int32_t(len(s.Lights))
	if len(s.Perlins) > 0 {
		pin.Pin(&s.Perlins[0])
		d.perlins = (*C.rt_perlin)(unsafe.Pointer(&s.Perlins[0]))
	}
	d.num_perlins = C.int32_t(len(s.Perlins))

	if n := len(s.Images); n > 0 {
		imgs := unsafe.Slice((*C.rt_image)(C.calloc(C.size_t(n), C.sizeof_rt_image)), n)
		defer C.free(unsafe.Pointer(&imgs[0]))
		for i := range s.Images {
			imgs[i].width, imgs[i].height, imgs[i].rgb = imageArgs(&pin, &s.Images[i])
		}
		d.images = &imgs[0]
		d.num_images = C.int32_t(n)
	}
	if s.Env != nil {
		env := (*C.rt_environment)(C.calloc(1, C.sizeof_rt_environment))
		defer C.free(unsafe.Pointer(env))
		env.width, env.height, env.rgb = imageArgs(&pin, &s.Env.Image)
		env.rotation = C.double(s.Env.Rotation)
		if s.Env.ImportanceSampling {
			env.use_importance_sampling = 1
		}
		d.environment = env
	}
	return c.check(C.rt_scene_upload(c.p, d))
}

func imageArgs(pin *runtime.Pinner, im *Image) (C.int32_t, C.int32_t, *C.double) {
	if im.Width <= 0 || im.Height <= 0 || len(im.RGB) < im.Width*im.Height*3 {
		return 0, 0, nil // ImageLoader without data
	}
	pin.Pin(&im.RGB[0])
	return C.int32_t(im.Width), C.int32_t(im.Height), (*C.double)(unsafe.Pointer(&im.RGB[0]))
}

// Info returns the sizes of the flattened device scene.
func (c *Ctx) Info() (SceneInfo, error) {
	var info SceneInfo
	err := c.check(C.rt_scene_get_info(c.p, (*C.rt_scene_info)(unsafe.Pointer(&info))))
	return info, err
}

// RenderParams is one rt_render call: samplesForPass / depthForPass of
// bucket_renderer.go:175-191 over a set of buckets.
type RenderParams struct {
	SamplesPerPixel int
	MaxDepth        int
	SampleOffset    int
	Seed            uint32
	Buckets         []Bucket // nil: the whole image
	Accumulate      bool     // false: overwrite the buckets' pixels
}

// Render renders into accum (Width*Height*3 float32, the per-pixel sum of
// sample radiance, linear) and blocks until done.
func (c *Ctx) Render(cam *CameraDesc, p RenderParams, accum []float32) (Stats, error) {
	var st Stats
	if len(accum) < int(cam.ImageWidth)*int(cam.ImageHeight)*3 {
		return st, &Error{StatusInvalid, "accum buffer smaller than width*height*3"}
	}
	var pin runtime.Pinner
	defer pin.Unpin()
	prm := (*C.rt_render_params)(C.calloc(1, C.sizeof_rt_render_params))
	defer C.free(unsafe.Pointer(prm))
	prm.samples_per_pixel = C.int32_t(p.SamplesPerPixel)
	prm.max_depth = C.int32_t(p.MaxDepth)
	prm.sample_offset = C.int32_t(p.SampleOffset)
	prm.seed = C.uint32_t(p.Seed)
	if len(p.Buckets) > 0 {
		pin.Pin(&p.Buckets[0])
		prm.buckets = (*C.rt_bucket)(unsafe.Pointer(&p.Buckets[0]))
		prm.num_buckets = C.int32_t(len(p.Buckets))
	}
	if p.Accumulate {
		prm.accumulate = 1
	}
	rc := C.rt_render(c.p, (*C.rt_camera_desc)(unsafe.Pointer(cam)), prm,
		(*C.float)(unsafe.Pointer(&accum[0])), (*C.rt_stats)(unsafe.Pointer(&st)))
	return st, c.check(rc)
}

// RenderRGBA is one progressive pass as renderBucketWithQuality does it
// (bucket_renderer.go:257-301): the buckets are rendered into the context's
// device-resident sums and quantised on the device (:276-285); only the
// RGBA8 framebuffer (width*height*4 bytes) comes back.  Pixels outside the
// buckets keep their previous value (rt_render_rgba8).
func (c *Ctx) RenderRGBA(cam *CameraDesc, p RenderParams, rgba []byte) (Stats, error) {
	var st Stats
	if len(rgba) < int(cam.ImageWidth)*int(cam.ImageHeight)*4 {
		return st, &Error{StatusInvalid, "rgba buffer smaller than width*height*4"}
	}
	var pin runtime.Pinner
	defer pin.Unpin()
	prm := (*C.rt_render_params)(C.calloc(1, C.sizeof_rt_render_params))
	defer C.free(unsafe.Pointer(prm))
	prm.samples_per_pixel = C.int32_t(p.SamplesPerPixel)
	prm.max_depth = C.int32_t(p.MaxDepth)
	prm.sample_offset = C.int32_t(p.SampleOffset)
	prm.seed = C.uint32_t(p.Seed)
	if len(p.Buckets) > 0 {
		pin.Pin(&p.Buckets[0])
		prm.buckets = (*C.rt_bucket)(unsafe.Pointer(&p.Buckets[0]))
		prm.num_buckets = C.int32_t(len(p.Buckets))
	}
	if p.Accumulate {
		prm.accumulate = 1
	}
	rc := C.rt_render_rgba8(c.p, (*C.rt_camera_desc)(unsafe.Pointer(cam)), prm,
		(*C.uint8_t)(unsafe.Pointer(&rgba[0])), (*C.rt_stats)(unsafe.Pointer(&st)))
	return st, c.check(rc)
}

// Sync waits for every render enqueued on the context and reports a
// device-side error of any of them.
func (c *Ctx) Sync() error { return c.check(C.rt_sync(c.p)) }

// Tonemap quantises an accumulated sum to RGBA8 exactly as
// bucket_renderer.go:276-285 does (1/spp, LinearToGamma, clamp, 256x).
func (c *Ctx) Tonemap(accum []float32, width, height, spp int, rgba []byte) error {
	if len(accum) < width*height*3 || len(rgba) < width*height*4 {
		return &Error{StatusInvalid, "tonemap buffer too small"}
	}
	return c.check(C.rt_tonemap_rgba8(c.p, (*C.float)(unsafe.Pointer(&accum[0])), C.int32_t(width),
		C.int32_t(height), C.int32_t(spp), (*C.uint8_t)(unsafe.Pointer(&rgba[0]))))
}

// Layout checks: each mirror is exactly as large as its C struct.
var (
	_ [unsafe.Sizeof(Node{}) - uintptr(C.sizeof_rt_hittable)]byte
	_ [uintptr(C.sizeof_rt_hittable) - unsafe.Sizeof(Node{})]byte
	_ [unsafe.Sizeof(Material{}) - uintptr(C.sizeof_rt_material)]byte
	_ [uintptr(C.sizeof_rt_material) - unsafe.Sizeof(Material{})]byte
	_ [unsafe.Sizeof(Texture{}) - uintptr(C.sizeof_rt_texture)]byte
	_ [uintptr(C.sizeof_rt_texture) - unsafe.Sizeof(Texture{})]byte
	_ [unsafe.Sizeof(Perlin{}) - uintptr(C.sizeof_rt_perlin)]byte
	_ [uintptr(C.sizeof_rt_perlin) - unsafe.Sizeof(Perlin{})]byte
	_ [unsafe.Sizeof(CameraDesc{}) - uintptr(C.sizeof_rt_camera_desc)]byte
	_ [uintptr(C.sizeof_rt_camera_desc) - unsafe.Sizeof(CameraDesc{})]byte
	_ [unsafe.Sizeof(Bucket{}) - uintptr(C.sizeof_rt_bucket)]byte
	_ [uintptr(C.sizeof_rt_bucket) - unsafe.Sizeof(Bucket{})]byte
	_ [unsafe.Sizeof(Stats{}) - uintptr(C.sizeof_rt_stats)]byte
	_ [uintptr(C.sizeof_rt_stats) - unsafe.Sizeof(Stats{})]byte
	_ [unsafe.Sizeof(SceneInfo{}) - uintptr(C.sizeof_rt_scene_info)]byte
	_ [uintptr(C.sizeof_rt_scene_info) - unsafe.Sizeof(SceneInfo{})]byte
)
