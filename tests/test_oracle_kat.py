"""Known-answer tests pinning the CPU oracle to the Go formulas (the reference
ships no tests/golden vectors: SURVEY.md §4, §8(c)).  Each expected value is
derived by hand from the cited Go code."""
import math

import numpy as np
import pytest

from tests.scene_builder import Builder, pinhole

EPS = 0.0  # zero pixel deltas: sub-pixel jitter cannot move the ray (RNG still keyed per pixel)


def lowbias32(x):
    x &= 0xFFFFFFFF
    x ^= x >> 16
    x = (x * 0x7FEB352D) & 0xFFFFFFFF
    x ^= x >> 15
    x = (x * 0x846CA68B) & 0xFFFFFFFF
    x ^= x >> 16
    return x


def test_rng_known_answers(O):
    for seed, pix, smp, ctr in [(0, 0, 0, 0), (1, 2, 3, 4), (0xDEADBEEF, 12345, 499, (3 << 16) | (1 << 12) | 7)]:
        k = lowbias32(seed ^ 0xA511E9B3)
        k = lowbias32(k ^ pix)
        k = lowbias32((k + smp * 0x9E3779B9) & 0xFFFFFFFF)
        h = lowbias32(k ^ lowbias32(ctr ^ 0x632BE5AB))
        assert O.rng_uniform(seed, pix, smp, ctr) == (h >> 8) * 2.0 ** -24


def _one_ray_cam(g, direction=(0, 0, -1), origin=(0, 0, 0), w=1, h=1, **kw):
    p00 = tuple(o + d for o, d in zip(origin, direction))
    return pinhole(g, w, h, origin, p00, (EPS, 0, 0), (0, -EPS, 0), **kw)


def _hit(g, O, b, root, cam, fp32):
    d = b.desc(root)
    top, prim, t = O.primary_hits(d, cam, 7, 0, fp32=fp32)
    return int(top[0]), int(prim[0]), float(t[0])


@pytest.mark.parametrize("fp32", [False, True])
def test_sphere_roots_open_interval(g, O, fp32):
    b = Builder(g)
    m = b.lambertian((0.5, 0.5, 0.5))
    s1 = b.sphere((0, 0, -5), 1.0, m)                  # sphere.go:63-94: t = 4
    root = b.listing([s1])
    assert _hit(g, O, b, root, _one_ray_cam(g), fp32)[1:] == (s1, pytest.approx(4.0))
    b = Builder(g)
    m = b.lambertian((0.5, 0.5, 0.5))
    s2 = b.sphere((0, 0, 0), 2.0, m)                   # origin inside: root1 < tmin -> root2 = 2
    root = b.listing([s2])
    assert _hit(g, O, b, root, _one_ray_cam(g), fp32)[1:] == (s2, pytest.approx(2.0))


@pytest.mark.parametrize("fp32", [False, True])
def test_quad_and_triangle_closed_edges(g, O, fp32):
    b = Builder(g)
    m = b.lambertian((0.5, 0.5, 0.5))
    q = b.quad((0, 0, -3), (1, 0, 0), (0, 1, 0), m)    # ray hits the corner: alpha = beta = 0 (Contains)
    assert _hit(g, O, b, b.listing([q]), _one_ray_cam(g), fp32)[1:] == (q, pytest.approx(3.0))
    b = Builder(g)
    m = b.lambertian((0.5, 0.5, 0.5))
    t = b.triangle((0, 0, -2), (1, 0, -2), (0, 1, -2), m)   # vertex hit: u = v = 0
    assert _hit(g, O, b, b.listing([t]), _one_ray_cam(g), fp32)[1:] == (t, pytest.approx(2.0))


def test_plane_parallel_and_open(g, O):
    b = Builder(g)
    m = b.lambertian((0.5, 0.5, 0.5))
    p = b.plane((0, -1, 0), (0, 1, 0), m)
    assert _hit(g, O, b, b.listing([p]), _one_ray_cam(g), False)[1] == -1     # |n.d| < 1e-8
    b = Builder(g)
    m = b.lambertian((0.5, 0.5, 0.5))
    p = b.plane((0, 0, -0.0005), (0, 0, 1), m)          # t = 0.0005 < 0.001: outside (0.001, inf)
    assert _hit(g, O, b, b.listing([p]), _one_ray_cam(g), False)[1] == -1


@pytest.mark.parametrize("fp32", [False, True])
def test_aabb_nan_slab_keeps_bounds(g, O, fp32):
    """aabb.go:59-116: d.x == 0 with the origin on the slab plane gives
    0*inf = NaN, which never updates the interval -> the box is hit."""
    b = Builder(g)
    m = b.lambertian((0.5, 0.5, 0.5))
    q = b.quad((0, -1, -3), (1, 0, 0), (0, 2, 0), m)    # x in [0,1]; ray x = 0 exactly
    node = b.leaf_node([q])
    top, prim, t = _hit(g, O, b, node, _one_ray_cam(g, direction=(0, 0, -1), origin=(0, 0, 0)), fp32)
    assert prim == q and t == pytest.approx(3.0)


@pytest.mark.parametrize("fp32", [False, True])
def test_tie_rule_list_order(g, O, fp32):
    """HittableList.Hit narrows to closestSoFar: at equal t a later
    closed-interval quad replaces the earlier one (Contains), a later
    identical sphere does not (Surrounds)."""
    b = Builder(g)
    m = b.lambertian((0.5, 0.5, 0.5))
    q1 = b.quad((-1, -1, -3), (2, 0, 0), (0, 2, 0), m)
    q2 = b.quad((-1, -1, -3), (2, 0, 0), (0, 2, 0), m)
    assert _hit(g, O, b, b.listing([q1, q2]), _one_ray_cam(g), fp32)[1] == q2
    b = Builder(g)
    m = b.lambertian((0.5, 0.5, 0.5))
    s1 = b.sphere((0, 0, -5), 1.0, m)
    s2 = b.sphere((0, 0, -5), 1.0, m)
    assert _hit(g, O, b, b.listing([s1, s2]), _one_ray_cam(g), fp32)[1] == s1


def _render1(g, O, b, root, cam, spp=4, depth=5, fp32=False):
    d = b.desc(root)
    return O.render(d, cam, g.make_params(spp, depth, seed=3), fp32=fp32)[0, 0] / spp


@pytest.mark.parametrize("fp32", [False, True])
def test_sky_gradient_and_background(g, O, fp32):
    b = Builder(g)
    m = b.lambertian((0.5, 0.5, 0.5))
    far = b.sphere((0, -100, 0), 1.0, m)
    cam = _one_ray_cam(g, direction=(0, 1, 0), sky=True)   # camera.go:520-526: a = 1 -> (0.5,0.7,1)
    np.testing.assert_allclose(_render1(g, O, b, b.listing([far]), cam, fp32=fp32), [0.5, 0.7, 1.0], rtol=1e-6)
    cam = _one_ray_cam(g, direction=(0, 1, 0), bg=(0.25, 0.5, 0.75))
    np.testing.assert_allclose(_render1(g, O, b, b.listing([far]), cam, fp32=fp32), [0.25, 0.5, 0.75], rtol=1e-6)


@pytest.mark.parametrize("fp32", [False, True])
def test_mirror_metal_reflects_sky(g, O, fp32):
    """Metal fuzz 0 (material.go:113-119): reflected (0,0,1) -> sky a = 0.5 ->
    (0.75, 0.85, 1.0), times the albedo."""
    b = Builder(g)
    mm = b.mat(g.RT_METAL, albedo=(0.5, 0.25, 1.0), fuzz=0.0)
    q = b.quad((-1, -1, -3), (2, 0, 0), (0, 2, 0), mm)
    got = _render1(g, O, b, b.listing([q]), _one_ray_cam(g, sky=True), fp32=fp32)
    np.testing.assert_allclose(got, [0.5 * 0.75, 0.25 * 0.85, 1.0], rtol=1e-6)


@pytest.mark.parametrize("fp32", [False, True])
def test_depth_semantics(g, O, fp32):
    """rayColorInternal (camera.go:443-518): a diffuse surface at depth 1
    returns Le + att*L(depth 0) = 0; an emitter seen directly returns Le."""
    b = Builder(g)
    m = b.lambertian((0.9, 0.9, 0.9))
    q = b.quad((-1, -1, -3), (2, 0, 0), (0, 2, 0), m)
    assert (_render1(g, O, b, b.listing([q]), _one_ray_cam(g, sky=True), depth=1, fp32=fp32) == 0).all()
    b = Builder(g)
    lm = b.light((3.0, 2.0, 1.0))
    q = b.quad((-1, -1, -3), (2, 0, 0), (0, 2, 0), lm)
    np.testing.assert_allclose(_render1(g, O, b, b.listing([q]), _one_ray_cam(g), depth=1, fp32=fp32), [3, 2, 1])


def _go_mod2(n):  # Go's % truncates toward zero
    return int(math.fmod(n, 2))


@pytest.mark.parametrize("fp32", [False, True])
@pytest.mark.parametrize("x,y", [(-0.5, 0.5), (-1.5, 0.5), (0.5, -0.5), (-2.5, -1.5), (1.5, 2.5)])
def test_checker_parity_negative_coords(g, O, fp32, x, y):
    """CheckerTexture.Value (texture.go:47-65) seen through an emitter."""
    b = Builder(g)
    tex = b.checker(1.0, (1.0, 0.0, 0.0), (0.0, 0.0, 1.0))
    lm = b.mat(g.RT_DIFFUSE_LIGHT, tex)
    q = b.quad((-10, -10, -3), (20, 0, 0), (0, 20, 0), lm)
    got = _render1(g, O, b, b.listing([q]), _one_ray_cam(g, direction=(x, y, -3)), depth=1, fp32=fp32)
    s = math.floor(x + 1e-4) + math.floor(y + 1e-4) + math.floor(-3 + 1e-4)
    expect = [1.0, 0.0, 0.0] if _go_mod2(s) == 0 else [0.0, 0.0, 1.0]
    np.testing.assert_allclose(got, expect)


def test_tonemap_known_answers(O):
    """bucket_renderer.go:276-285 with LinearToGamma (utils.go:85-90)."""
    acc = np.array([[[0.25 * 4, 1.0 * 4, -2.0], [np.nan, 0.0, 4 * 0.998001], [4 * 0.49, 4 * 0.0001, 1e30]]],
                   np.float32)
    out = O.tonemap(acc, 4)
    assert out[0, 0].tolist() == [128, 255, 0, 255]
    assert out[0, 1, :3].tolist() == [0, 0, int(256 * min(math.sqrt(np.float32(4 * 0.998001) / 4), 0.999))]
    assert out[0, 2, :3].tolist() == [int(256 * math.sqrt(np.float32(4 * 0.49) / 4)),
                                      int(256 * math.sqrt(np.float32(4 * 0.0001) / 4)), 255]


@pytest.mark.parametrize("ntests", [1, 2])
def test_volume_leaf_wrapper_tested_twice(g, O, ntests):
    """Volume.Hit draws a fresh free-flight length per call (volume.go:66);
    the BVH leaf wrapper BVHNode{leaf, leaf} (bvh.go:141) calls its leaf twice
    per traversal, so a volume in a BVH leaf scatters with probability
    1-exp(-2*rho*L) instead of 1-exp(-rho*L)."""
    b = Builder(g)
    wm = b.lambertian((0.5, 0.5, 0.5))
    faces = [b.quad((-1, -1, -2), (2, 0, 0), (0, 2, 0), wm), b.quad((-1, -1, -4), (2, 0, 0), (0, 2, 0), wm)]
    boundary = b.listing(faces)                         # slab z in [-4,-2]: L = 2 along -z
    iso = b.mat(g.RT_ISOTROPIC, b.solid((1, 1, 1)))
    rho = 0.25
    vol = b.volume(boundary, rho, iso)
    back = b.quad((-5, -5, -10), (10, 0, 0), (0, 10, 0), wm)
    root = b.leaf_node([vol, back]) if ntests == 2 else b.listing([vol, back])
    d = b.desc(root)
    cam = pinhole(g, 128, 128, (0, 0, 0), (0, 0, -1), (EPS, 0, 0), (0, -EPS, 0))
    top, prim, t = O.primary_hits(d, cam, 99, 0, fp32=False)
    frac = float(np.mean(prim == vol))
    expect = 1 - math.exp(-ntests * rho * 2.0)
    assert abs(frac - expect) < 4 * math.sqrt(expect * (1 - expect) / top.size)


def test_phantom_hdri_only_at_camera_max_depth(g, O):
    """camera.go:456-458: primary misses are black only when depth ==
    Camera.MaxDepth (so BucketRenderer's 1-spp preview pass at depth 3 shows
    the HDRI)."""
    s = g.Scene("hdri-test", width=48)
    cam = s.camera
    top, prim, _ = O.primary_hits(s.desc, cam, 1, 0, fp32=False)
    sky = np.flatnonzero(top.reshape(cam.image_height, cam.image_width)[0] < 0)
    assert sky.size > 0
    full = O.render(s.desc, cam, g.make_params(1, cam.max_depth, seed=1), fp32=False)
    prev = O.render(s.desc, cam, g.make_params(1, 3, seed=1), fp32=False)
    assert (full[0, sky] == 0).all()
    assert (prev[0, sky] > 0).all()


def test_fp32_mirror_close_to_fp64(g, O):
    s = g.Scene("cornell", width=48)
    cam = s.camera
    p = g.make_params(16, 5, seed=2)
    a = O.render(s.desc, cam, p, fp32=False) / 16
    b = O.render(s.desc, cam, p, fp32=True) / 16
    assert abs(a.mean() - b.mean()) < 0.02 * a.mean()
    assert float(np.mean((a - b) ** 2)) < 5e-3


# ---- NEE, instance transforms, volumes (tests/kat_cases.py) ---------------
from tests import kat_cases as K  # noqa: E402


@pytest.mark.parametrize("fp32", [False, True])
def test_area_light_nee_closed_form(g, O, fp32):
    """sampleAreaLight (camera.go:610-678): cosines, pdfL, balance weight,
    x number of lights, per-component clamp at 20 (red clamps)."""
    b, d, cam = K.area_light_scene(g)
    got = O.render(d, cam, g.make_params(4, 1, seed=K.SEED), fp32=fp32)[0]
    want = K.area_light_expected(spp=4)
    assert (want[:, 0] == 80.0).any() and (want[:, 0] < 80.0).any() and (want[:, 1] < 20).all()   # red clamps
    np.testing.assert_allclose(got, want, rtol=2e-5 if fp32 else 1e-12, atol=1e-9)


@pytest.mark.parametrize("fp32", [False, True])
def test_instance_chain_point_and_normal(g, O, fp32):
    """Translate(RotateY(Scale(quad))): t = 1 in every space, the bounce-1 ray
    starts at the world hit point and leaves along N + RandomUnitVector with
    N renormalised by Scale and rotated back (transform.go:113-191, 360-444)."""
    b, d, cam, top, q = K.instance_scene(g)
    t_top, t_prim, t_t, ray, _ = O.path_records(d, cam, K.SEED, 0, 2, fp32=fp32, threads=2)
    assert (t_top[0] == top).all() and (t_prim[0] == q).all()
    tol = 2e-6 if fp32 else 1e-12
    np.testing.assert_allclose(t_t[0], 1.0, rtol=tol)
    P = K.instance_world_point()
    N = K.instance_expected_normal()
    assert abs(np.linalg.norm(N) - 1) < 1e-12 and N[1] < 0
    for pix in range(cam.image_width):
        assert t_top[1, pix] != -2
        np.testing.assert_allclose(ray[1, pix, :3], P, rtol=tol * 4, atol=tol * 4)
        n_got = ray[1, pix, 3:] - K.random_unit_vector(K.SEED, pix, 0, 0)
        np.testing.assert_allclose(n_got, N, rtol=0, atol=tol * 8)


@pytest.mark.parametrize("fp32", [False, True])
def test_volume_hit_fixed_draw(g, O, fp32):
    """Volume.Hit (volume.go:34-79): t1 = 2, t2 = 4, the free flight
    -ln(U)/rho from the pixel's draw; a longer flight passes to the wall."""
    b, d, cam, vol, back = K.volume_scene(g)
    top, prim, t = O.primary_hits(d, cam, K.SEED, 0, fp32=fp32)
    ids, ts = K.volume_expected()
    want = np.array([vol if i == "vol" else back for i in ids])
    assert np.array_equal(prim, want)
    assert 0.2 < (want == vol).mean() < 0.8
    np.testing.assert_allclose(t, ts, rtol=2e-6 if fp32 else 1e-12)


@pytest.mark.parametrize("name,kw", [("cornell", dict(width=48)), ("hdri-nee", dict(width=48)),
                                     ("cornell-smoke", dict(width=48))])
def test_path_records_consistent(g, O, name, kw):
    """The oracle's per-bounce recorder: bounce 0 is primary_hits, a path that
    ended stays ended, a visible shadow ray is a traced one."""
    s = g.Scene(name, **kw)
    cam = s.camera
    top, prim, t, ray, nee = O.path_records(s.desc, cam, 5, 1, 4, fp32=True, threads=4)
    pt, pp, ptt = O.primary_hits(s.desc, cam, 5, 1, fp32=True)
    assert np.array_equal(top[0], pt) and np.array_equal(prim[0], pp) and np.array_equal(t[0], ptt)
    for k in range(1, 4):
        assert not ((top[k - 1] == -2) & (top[k] != -2)).any()
        assert not ((top[k - 1] == -1) & (top[k] != -2)).any()      # a miss ends the path
    assert ((nee >> 2) & ~nee & 3 == 0).all()
    assert ((nee >> 2) & 3).any()
