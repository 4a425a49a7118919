"""GPU (HIP, via the C-ABI) vs CPU oracle parity.  Marked gpu.

Tolerances (stated, BASELINE.json north_star):
  * first-bounce closest-hit ids (top-level object, primitive) and hit t:
    bit-exact vs the oracle's fp32 mirror mode, every scene (fog included: the
    free-flight log is libm-free on both sides, tests/test_detlog.py); every
    later bounce and every NEE shadow ray: tests/test_gpu_paths.py.  The one
    residual class is grazing hits within fp32 rounding of a primitive's box,
    where the BVH topology decides which box culls the hit: about 1 in 10^8
    path rays on C4 (1 of 95.9 M); tests/test_gpu_grazing.py replays the
    recorded case and bounds the rate at <= 1 per 10^7 over a full-width
    scan;
  * radiance vs the fp32 mirror (same counter RNG keys, so every path is the
    same path, tests/test_gpu_paths.py): image mean over pixels of the squared
    RGB error of the per-pixel average radiance <= FP32_MSE = 1e-10, and at
    most FP32_OFF = 1e-3 of the pixels (HDRI scenes: FP32_OFF_HDRI = 1e-2)
    off by more than 1e-5 relative.  What remains is the order of the adds
    (the GPU adds beta * emission bounce by bounce, the recursion returns
    Le + att * L) and, with an HDRI, the last-ulp differences of ocml's and
    glibc's atan2f / asinf / sinf / cosf in the environment lookups.
    Measured (round 4): mse <= 3.9e-16, max |d| <= 4.7e-7, no pixel off;
    HDRI scenes mse 6.9e-12, max |d| 1.0e-4, 0.27-0.52 % of the pixels off;
  * radiance vs the oracle's float64 mode (the Go arithmetic, camera.go:443-518
    in float64) on the BASELINE configs: the same image-mean squared error
    <= 1e-4 at the spp stated per config in FP64_CASES, and the image-mean
    relative bias within 2e-3;
  * RGBA8 quantisation: bit-exact given the same float sums.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FP32_MSE = 1e-10
FP32_OFF, FP32_OFF_HDRI = 1e-3, 1e-2


def fp32_bar(name, gpu_sum, ref_sum, spp):
    """(mse, share of pixels off by > 1e-5 relative); asserts the fp32 bar."""
    a, b = gpu_sum.astype(np.float64) / spp, ref_sum / spp
    mse = float(np.mean((a - b) ** 2))
    px_err = np.max(np.abs(a - b), axis=2)
    off = float(np.mean(px_err > 1e-5 * np.maximum(1.0, np.max(np.abs(b), axis=2))))
    print(f"fp32 parity {name}: mse {mse:.3e} max |d| {px_err.max():.3e} pixels off by >1e-5 rel {off:.2e}")
    assert mse <= FP32_MSE, f"{name}: mse {mse:.3e}"
    assert off <= (FP32_OFF_HDRI if name.startswith("hdri") else FP32_OFF), f"{name}: {off:.3e} of the pixels off"
    return mse, off

LUCY = dict(lucy_rings=60, lucy_cols=80)
SCENES = [
    ("simple", dict(width=96)),
    ("random", dict(width=96)),
    ("cornell", dict(width=64)),
    ("cornell-smoke", dict(width=64)),
    ("cornell-lucy", dict(width=64, **LUCY)),
    ("hdri-test", dict(width=96)),
    ("hdri-nee", dict(width=96)),
    ("quads", dict(width=64)),
    ("primitives", dict(width=96)),
    ("perlin", dict(width=96)),
    ("earth", dict(width=96)),
    ("checkered-spheres", dict(width=96)),
    ("glossy-metal", dict(width=96)),
    ("cornell-glossy", dict(width=64)),
    ("cornell-rotations", dict(width=64)),
]


def _scene(g, name, kw):
    return g.Scene(name, **kw)


@pytest.mark.parametrize("name,kw", SCENES, ids=[s[0] for s in SCENES])
def test_primary_hits_bit_exact(g, O, ctx, name, kw):
    s = _scene(g, name, kw)
    cam = s.camera
    ctx.upload(s.desc)
    for sample in (0, 3):
        tg, pg, t_g = ctx.primary_hits(cam, 1234, sample)
        to, po, t_o = O.primary_hits(s.desc, cam, 1234, sample, fp32=True)
        mism = np.flatnonzero((tg != to) | (pg != po))
        assert mism.size == 0, f"{name}: {mism.size} mismatches, first {mism[:5]}"
        hit = tg >= 0
        assert np.array_equal(t_g[hit], t_o[hit].astype(np.float32)), f"{name}: hit t differs"
        assert (tg >= 0).any()


@pytest.mark.parametrize("collapse", ["sah", "greedy"])
@pytest.mark.parametrize("builder", ["reference", "sah", "device"])
@pytest.mark.parametrize("name", ["cornell-lucy", "random", "cornell-smoke"])
def test_bvh_builders_same_hits(g, O, builder, name, collapse):
    """The SAH BVHs (mesh BLAS, world), the device-built LBVH mesh BLAS and the
    reference topology, each collapsed to BVH4 nodes either way
    (RT_OPT_BVH4_COLLAPSE), give the same first hits (ids and t) as the
    oracle, which walks the caller's graph."""
    s = _scene(g, name, dict(width=64, **LUCY) if name == "cornell-lucy" else dict(width=64))
    cam = s.camera
    c = g.Context(0)
    try:
        c.set_blas_builder(builder)
        c.set_tlas_builder("sah" if builder == "device" else builder)
        c.set_collapse(collapse)
        c.upload(s.desc)
        tg, pg, t_g = c.primary_hits(cam, 99, 1)
        to, po, t_o = O.primary_hits(s.desc, cam, 99, 1, fp32=True)
        assert np.array_equal(tg, to) and np.array_equal(pg, po)
        hit = tg >= 0
        assert np.array_equal(t_g[hit], t_o[hit].astype(np.float32))
    finally:
        c.close()


@pytest.mark.parametrize("name,kw", SCENES, ids=[s[0] for s in SCENES])
def test_radiance_parity_fp32(g, O, ctx, name, kw):
    s = _scene(g, name, kw)
    cam = s.camera
    spp = 8
    ctx.upload(s.desc)
    p = g.make_params(spp, cam.max_depth, seed=77)
    gpu, _ = ctx.render(cam, p)
    ref = O.render(s.desc, cam, p, fp32=True)
    assert np.isfinite(gpu).all()
    fp32_bar(name, gpu, ref, spp)
    assert gpu.mean() > 0


@pytest.mark.parametrize("name,kw", SCENES, ids=[s[0] for s in SCENES])
def test_quant8_nodes_parity(g, O, name, kw):
    """RT_NODES_QUANT8 (64-B quantised nodes, node_quant.h): first hits
    bit-exact against the oracle (the boxes only cull) and the same radiance
    bar as the fp32 nodes; cornell-rotations keeps its fp32 nodes."""
    s = _scene(g, name, kw)
    cam = s.camera
    c = g.Context(0)
    try:
        c.set_node_format("quant8")
        c.upload(s.desc)
        tg, pg, t_g = c.primary_hits(cam, 1234, 3)
        to, po, t_o = O.primary_hits(s.desc, cam, 1234, 3, fp32=True)
        assert np.array_equal(tg, to) and np.array_equal(pg, po), f"{name}: hit ids differ"
        hit = tg >= 0
        assert np.array_equal(t_g[hit], t_o[hit].astype(np.float32)), f"{name}: hit t differs"
        spp = 8
        p = g.make_params(spp, cam.max_depth, seed=77)
        gpu, _ = c.render(cam, p)
        ref = O.render(s.desc, cam, p, fp32=True)
        assert np.isfinite(gpu).all()
        fp32_bar(name, gpu, ref, spp)
    finally:
        c.close()


# BASELINE configs (C1 SimpleScene, C2 RandomScene, C3 CornellBoxScene, C4
# CornellBoxLucy with the full 280K-triangle mesh, C5 HDRITestScene) at reduced
# resolution, plus the fog and RotateX/Z variants: (scene, kwargs, spp).  The
# fp32-vs-float64 error is dominated by paths whose branch (a dielectric
# reflect/refract draw, a grazing hit, a rejection-sampling loop) flips between
# the two precisions; it falls as 1/spp.  HDRITestScene needs 128 spp: its
# flipped paths carry HDRI radiance up to 77.75 (measured 5.7e-4 at 16 spp,
# 3e-5..7e-5 at 64, 1.8e-5..3.9e-5 at 128 over seeds 5-7).
FP64_CASES = [
    ("simple", dict(width=96), 64),
    ("random", dict(width=96), 64),
    ("cornell", dict(width=64), 64),
    ("cornell-smoke", dict(width=64), 64),
    ("cornell-lucy", dict(width=64), 64),
    ("hdri-test", dict(width=96), 128),
    ("cornell-rotations", dict(width=64), 64),
]


@pytest.mark.parametrize("name,kw,spp", FP64_CASES, ids=[c[0] for c in FP64_CASES])
def test_radiance_vs_fp64_reference(g, O, ctx, name, kw, spp):
    """fp32 GPU vs the float64 restatement of the Go arithmetic, same RNG keys:
    per-pixel L2 <= 1e-4 (image mean) and image-mean relative bias <= 2e-3."""
    s = _scene(g, name, kw)
    cam = s.camera
    ctx.upload(s.desc)
    p = g.make_params(spp, cam.max_depth, seed=5)
    gpu, _ = ctx.render(cam, p)
    ref = O.render(s.desc, cam, p, fp32=False, threads=16)
    a = gpu.astype(np.float64) / spp
    b = ref / spp
    mse = float(np.mean((a - b) ** 2))
    bias = float((a.mean() - b.mean()) / max(b.mean(), 1e-6))
    print(f"fp64 tolerance {name} {cam.image_width}x{cam.image_height} {spp}spp: mse {mse:.3e} rel_bias {bias:+.2e}")
    assert mse <= 1e-4, f"{name}: mse {mse:.3e}"
    assert abs(bias) <= 2e-3, f"{name}: relative bias {bias:+.3e}"


def test_tonemap_bit_exact(g, O, ctx):
    rng = np.random.default_rng(0)
    acc = (rng.random((37, 53, 3)) * 3.0).astype(np.float32)
    acc[0, 0] = [0.0, -1.0, np.nan]
    acc[0, 1] = [1e9, 0.998001 * 4, 0.25 * 4]
    for spp in (1, 4, 7):
        assert np.array_equal(ctx.tonemap(acc, spp), O.tonemap(acc, spp))


def test_deterministic_and_bucket_split(g, ctx):
    s = g.Scene("cornell", width=64)
    cam = s.camera
    ctx.upload(s.desc)
    p = g.make_params(6, 5, seed=9)
    a, _ = ctx.render(cam, p)
    b, _ = ctx.render(cam, p)
    assert np.array_equal(a, b)
    bk = g.generate_buckets(cam.image_width, cam.image_height, 32)
    acc = np.zeros_like(a)
    for half in (bk[: len(bk) // 2], bk[len(bk) // 2:]):
        ctx.render(cam, g.make_params(6, 5, seed=9, buckets=half), acc)
    np.testing.assert_allclose(acc, a, rtol=2e-6, atol=1e-6)


def test_accumulate_sample_offset(g, ctx):
    s = g.Scene("simple", width=64)
    cam = s.camera
    ctx.upload(s.desc)
    full, _ = ctx.render(cam, g.make_params(8, 10, seed=3))
    acc, _ = ctx.render(cam, g.make_params(4, 10, seed=3))
    ctx.render(cam, g.make_params(4, 10, seed=3, sample_offset=4, accumulate=True), acc)
    np.testing.assert_allclose(acc, full, rtol=1e-5, atol=1e-5)


def test_overwrite_only_bucket_pixels(g, ctx):
    s = g.Scene("simple", width=64)
    cam = s.camera
    ctx.upload(s.desc)
    acc = np.full((cam.image_height, cam.image_width, 3), -7.0, np.float32)
    ctx.render(cam, g.make_params(2, 10, seed=3, buckets=[(0, 0, 16, 8)]), acc)
    assert (acc[:8, :16] != -7.0).all()
    assert (acc[8:] == -7.0).all() and (acc[:, 16:] == -7.0).all()


def test_count_work(g, ctx):
    s = g.Scene("cornell", width=48)
    cam = s.camera
    ctx.upload(s.desc)
    w = ctx.count_work(cam, g.make_params(4, 5, seed=1))
    n = cam.image_width * cam.image_height * 4
    assert w["samples"] == n
    assert w["rays"] >= n and w["node_visits"] > 0 and w["quad_tests"] > 0 and w["volume_tests"] > 0
    assert w["shadow_rays"] > 0


@pytest.mark.parametrize("name", ["cornell", "hdri-test"])
def test_bucket_renderer_three_passes(g, O, tmp_path, name):
    """The progressive 3-pass schedule (bucket_renderer.go:175-191): pass k
    renders (1 spp, depth 3), (max(1, spp/4), max(3, depth/2)), (spp, depth)
    and OVERWRITES the framebuffer (renderBucketWithQuality :257-301).  Each
    pass's accumulation matches the oracle's render of that pass's
    spp/depth/seed over the centre-out buckets, its RGBA8 framebuffer is the
    reference quantisation (:276-285) of that accumulation, bit for bit, and
    SaveImage's PNG decodes back to the final framebuffer."""
    from tests.pngdec import read_png
    s = g.Scene(name, width=64, spp=8)
    cam = s.camera
    seed = 1
    r = g.BucketRenderer(s, 32, 8, 0, seed=seed)
    assert not r.is_completed()
    spp_full, depth_full = cam.samples_per_pixel, cam.max_depth
    schedule = [(1, 3), (max(1, spp_full // 4), max(3, depth_full // 2)), (spp_full, depth_full)]
    buckets = g.generate_buckets(cam.image_width, cam.image_height, 32)
    for k, (spp, depth) in enumerate(schedule):
        r.render_pass(k)
        assert r.is_completed() == (k == 2)
        acc, fb = r.accum(), r.framebuffer()
        pseed = (seed + k * 0x9E3779B9) & 0xFFFFFFFF
        ref = O.render(s.desc, cam, g.make_params(spp, depth, seed=pseed, buckets=buckets), fp32=True)
        mse, _ = fp32_bar(f"{name} pass {k}", acc, ref, spp)
        assert np.array_equal(fb, O.tonemap(acc, spp)), f"pass {k}: framebuffer is not the quantised accumulation"
        same = float(np.mean(fb == O.tonemap(ref.astype(np.float32), spp)))
        print(f"{name} pass {k} ({spp} spp, depth {depth}): mse {mse:.2e}, RGBA8 bytes equal to the oracle's {same:.5f}")
        assert same >= 0.99, f"pass {k}: only {same:.4f} of the RGBA8 bytes match the oracle"
        assert (fb[..., 3] == 255).all()
    out = tmp_path / "image.png"
    r.save_image(str(out))
    assert np.array_equal(read_png(str(out)), r.framebuffer())


@pytest.mark.parametrize("rings,cols", [(60, 80), (0, 0)])
def test_device_bvh_build(g, O, rings, cols):
    """RT_BLAS_DEVICE: the mesh BLAS (small mesh, and the full 280K-triangle
    Lucy stand-in) is built on the GPU at upload (build.hip).  First hits are
    bit-exact against the oracle, the radiance matches the SAH-built scene's
    bit for bit (same hits, same shading), and the device nodes are counted."""
    s = g.Scene("cornell-lucy", width=64, lucy_rings=rings, lucy_cols=cols)
    cam = s.camera
    dev, host = g.Context(0), g.Context(0)
    try:
        dev.set_blas_builder("device")
        dev.upload(s.desc)
        host.upload(s.desc)
        assert dev.last_build_ms() > 0.0 and host.last_build_ms() == 0.0
        di, hi = dev.info(), host.info()
        assert di.triangles == hi.triangles and di.nodes > 0 and 0 < di.stack_needed <= 64
        tg, pg, t_g = dev.primary_hits(cam, 7, 2)
        to, po, t_o = O.primary_hits(s.desc, cam, 7, 2, fp32=True)
        assert np.array_equal(tg, to) and np.array_equal(pg, po)
        hit = tg >= 0
        assert np.array_equal(t_g[hit], t_o[hit].astype(np.float32))
        p = g.make_params(4, cam.max_depth, seed=3)
        a, _ = dev.render(cam, p)
        b, _ = host.render(cam, p)
        assert np.array_equal(a, b)
    finally:
        dev.close()
        host.close()
