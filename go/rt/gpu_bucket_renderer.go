// gpu_bucket_renderer.go — NewGPUBucketRenderer: BucketRenderer's three
// progressive passes (bucket_renderer.go:127-213) with each pass rendered by
// librtgpu.so on an MI355X instead of numWorkers goroutines.
//
// COMPILE-UNVERIFIED: no Go toolchain in this repository's build image.  Copy
// to rt/ of byvfx/go-raytracing next to gpu_flatten.go; main.go:86 then reads
//
//	renderer := rt.NewGPUBucketRenderer(camera, bvh, bucketSize, numWorkers)
//
// and ebiten.RunGame(renderer) is unchanged.  The type embeds the CPU
// renderer, so Draw / Layout / SaveImage / IsCompleted / GetRenderDuration
// and the stats overlay are the reference's own code; only Update differs.
// The same schedule is implemented in C++ by librtscene.so (rts_renderer_*),
// which tests/test_gpu_parity.py::test_bucket_renderer_three_passes checks
// against the CPU oracle.
package rt

import (
	"fmt"
	"log"
	"os"
	"time"

	"go-raytracing/rtgpu"
)

// GPUBucketRenderer is a BucketRenderer whose passes run on the GPU.  When
// the scene holds something the GPU path does not take (rtgpu.IsUnsupported)
// or no device is present, gpu is nil and every method is the CPU
// renderer's.
type GPUBucketRenderer struct {
	*BucketRenderer
	gpu     *rtgpu.Ctx
	cam     rtgpu.CameraDesc
	buckets []rtgpu.Bucket // r.buckets (centre-out order of generateBuckets)
	rgba    []byte         // tonemapped frame of the pass in flight
	seed    uint32
	err     error // first GPU error (under BucketRenderer.mu); the render stops there
}

// NewGPUBucketRenderer has NewBucketRenderer's signature
// (bucket_renderer.go:54-74).  Its worker pool is every visible GPU (as
// main.go:84 sizes the CPU pool with runtime.NumCPU()); numWorkers only
// matters for the CPU fallback.
func NewGPUBucketRenderer(camera *Camera, world Hittable, bucketSize int, numWorkers int) *GPUBucketRenderer {
	g := &GPUBucketRenderer{BucketRenderer: NewBucketRenderer(camera, world, bucketSize, numWorkers), seed: 1}
	if err := g.initGPU(camera, world); err != nil {
		fmt.Fprintf(os.Stderr, "GPU renderer unavailable (%v); rendering on the CPU\n", err)
		if g.gpu != nil {
			g.gpu.Close()
			g.gpu = nil
		}
	}
	return g
}

func (g *GPUBucketRenderer) initGPU(camera *Camera, world Hittable) error {
	camera.Initialize() // the state GetRay reads (camera.go:286-344); idempotent
	scene, err := FlattenForGPU(world, camera)
	if err != nil {
		return err
	}
	// every visible device; if that context cannot be made (a device without
	// peer access to device 0) or a device fails the upload (out of memory),
	// device 0 alone before giving up on the GPU
	if g.gpu, err = rtgpu.New(); err == nil {
		if err = g.gpu.Upload(scene); err != nil {
			g.gpu.Close()
			g.gpu = nil
		}
	}
	if g.gpu == nil {
		// say why the other devices are not used: an out-of-memory or
		// peer-access failure would otherwise only show up as lower speed
		log.Printf("rt: GPU renderer on all devices failed (%v); using device 0 only", err)
		if g.gpu, err = rtgpu.New(0); err != nil {
			return err
		}
		if err = g.gpu.Upload(scene); err != nil {
			return err
		}
	}
	// RTGPU_DEALING=dynamic: the devices claim runs of tiles as they finish
	// (the reference's bucket channel, bucket_renderer.go:193-213) instead of
	// the static round-robin split; for devices that differ in speed
	if os.Getenv("RTGPU_DEALING") == "dynamic" && g.gpu.NumDevices() > 1 {
		if err = g.gpu.SetOption(rtgpu.OptDealing, rtgpu.DealDynamic); err != nil {
			return err
		}
	}
	g.cam = GPUCameraDesc(camera)
	g.buckets = make([]rtgpu.Bucket, len(g.BucketRenderer.buckets))
	for i, b := range g.BucketRenderer.buckets {
		g.buckets[i] = rtgpu.Bucket{X: int32(b.X), Y: int32(b.Y), Width: int32(b.Width), Height: int32(b.Height)}
	}
	g.rgba = make([]byte, 4*camera.ImageWidth*camera.ImageHeight)
	return nil
}

// Close releases the device context (the CPU renderer has nothing to free).
func (g *GPUBucketRenderer) Close() {
	if g.gpu != nil {
		g.gpu.Close()
		g.gpu = nil
	}
}

// Update is BucketRenderer.Update (bucket_renderer.go:127-165) with the pass
// body swapped for gpuPass.
func (g *GPUBucketRenderer) Update() error {
	if g.gpu == nil {
		return g.BucketRenderer.Update()
	}
	r := g.BucketRenderer
	if r.completed {
		return nil
	}
	r.mu.Lock()
	if !r.renderStarted {
		r.renderStarted = true
		r.mu.Unlock()
		go g.gpuPass()
	} else {
		r.mu.Unlock()
	}
	if r.passComplete.Load() && r.currentPass < r.totalPasses {
		r.passComplete.Store(false)
		r.completedCount.Store(0)
		r.currentPass++
		gerr := g.passErr()
		if r.currentPass < r.totalPasses && gerr == nil {
			go g.gpuPass()
		} else {
			r.completed = true
			r.renderEnd = time.Now()
			if gerr != nil {
				fmt.Fprintf(os.Stderr, "GPU render failed: %v\n", gerr)
			}
			r.drawStatsToFramebuffer()
			_ = r.SaveImage("image.png")
			PrintRenderStats(r.renderEnd.Sub(r.renderStart), r.camera.ImageWidth, r.camera.ImageHeight)
			g.Close()
		}
	}
	return nil
}

// passQuality is renderPass's schedule (bucket_renderer.go:175-191).
func passQuality(pass int, c *Camera) (spp, depth int) {
	switch pass {
	case 0:
		return 1, 3
	case 1:
		return max(1, c.SamplesPerPixel/4), max(3, c.MaxDepth/2)
	default:
		return c.SamplesPerPixel, c.MaxDepth
	}
}

// passErr is the first GPU error so far; gpuPass writes it under r.mu on its
// goroutine, Update reads it on the game loop's.
func (g *GPUBucketRenderer) passErr() error {
	g.BucketRenderer.mu.Lock()
	defer g.BucketRenderer.mu.Unlock()
	return g.err
}

// passChunk is the device work per rt_render_rgba8 call of a pass: long
// enough that a call's fixed cost (its last kernels' tails, the RGBA8 copy)
// stays a few per cent, short enough that the progress bar moves several
// times a second.
const passChunk = 150 * time.Millisecond

// gpuPass renders the current pass over every device (each call deals its
// buckets round-robin over the context's GPUs and overwrites their sums, as
// renderBucketWithQuality writes every bucket pixel each pass), quantised on
// the device with bucket_renderer.go:276-285's formula (rt_render_rgba8:
// only the RGBA8 frame crosses PCIe).  It goes in calls of about passChunk
// of work (the first 64 buckets, later ones sized from the previous call's
// rate); after each call it copies that call's buckets into the framebuffer
// under r.mu and advances completedCount by them, as renderBucketWithQuality
// does bucket by bucket, so the window's progress bar moves during a pass.
func (g *GPUBucketRenderer) gpuPass() {
	r := g.BucketRenderer
	spp, depth := passQuality(r.currentPass, r.camera)
	w := r.camera.ImageWidth
	seed := g.seed + uint32(r.currentPass)*0x9E3779B9 // one RNG stream per pass
	n := 64
	for i := 0; i < len(g.buckets); {
		chunk := g.buckets[i:min(i+n, len(g.buckets))]
		t0 := time.Now()
		_, err := g.gpu.RenderRGBA(&g.cam, rtgpu.RenderParams{SamplesPerPixel: spp, MaxDepth: depth, Seed: seed,
			Buckets: chunk}, g.rgba)
		el := time.Since(t0)
		r.mu.Lock()
		if err != nil {
			g.err = err
			r.mu.Unlock()
			break
		}
		for _, b := range chunk {
			for y := int(b.Y); y < int(b.Y+b.Height); y++ {
				row := (y*w + int(b.X)) * 4
				copy(r.framebuffer.Pix[row:row+int(b.Width)*4], g.rgba[row:row+int(b.Width)*4])
			}
		}
		r.mu.Unlock()
		r.completedCount.Add(int32(len(chunk)))
		i += len(chunk)
		if el > 0 {
			n = min(max(int(float64(len(chunk))*float64(passChunk)/float64(el)), 16), len(g.buckets))
		}
	}
	r.passComplete.Store(true)
}
