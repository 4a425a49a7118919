"""GetRay's slow path: camera motion blur and the free camera
(camera.go:390-434, SetMotion :204-209, EnableFreeCamera :226-232).

CPU: the oracle's slow path reproduces the fast path bit for bit in fp64
when the camera does not move (zero centerMotion / lookAtMotion velocity) or
when the free camera looks along LookAt-LookFrom: the reference computes the
same basis and pixel grid with the same operations in Initialize (:286-344)
and GetRay (:390-434).  A moving camera changes the image.
GPU: first hits bit-exact and fp32 radiance parity against the oracle for
moving and free cameras, with and without the defocus disk (RandomScene)."""
import numpy as np
import pytest

CASES = [
    ("simple", dict(width=64, motion=((0.3, 0.2, 2.5), (0.1, 0.0, -1.0)))),
    ("random", dict(width=96, motion=((13.5, 2.3, 3.2), (0.0, 0.1, 0.0)))),      # defocus 0.6
    ("quads", dict(width=64, free_forward=(0.1, 0.05, -1.0))),
    ("random", dict(width=96, free_forward=(-12.0, -2.2, -3.0))),
    ("cornell-lucy", dict(width=48, lucy_rings=30, lucy_cols=40,
                          motion=((300.0, 278.0, -800.0), (278.0, 260.0, 0.0)))),
]
IDS = ["simple-motion", "random-motion", "quads-free", "random-free", "lucy-motion"]


def _unit(v):
    v = np.asarray(v, np.float64)
    return v / np.sqrt(v @ v)


@pytest.mark.parametrize("name,width", [("simple", 48), ("random", 64)])
def test_static_slow_path_equals_fast_path_fp64(g, O, name, width):
    s0 = g.Scene(name, width=width)
    cam0 = s0.camera
    lf = list(cam0.center_motion_orig)
    la = list(cam0.look_at_motion_orig)
    s1 = g.Scene(name, width=width, motion=(lf, la))     # CameraMotion with zero velocity
    assert s1.camera.camera_motion == 1
    assert list(s1.camera.center_motion_dir) == [0.0, 0.0, 0.0]
    fwd = (np.asarray(la) - np.asarray(lf))
    s2 = g.Scene(name, width=width, free_forward=fwd)     # FreeCamera along LookAt - LookFrom
    assert s2.camera.free_camera == 1
    assert np.allclose(list(s2.camera.forward), _unit(fwd), atol=0)
    p = g.make_params(2, 4, seed=9)
    ref = O.render(s0.desc, cam0, p, fp32=False, threads=4)
    assert np.array_equal(O.render(s1.desc, s1.camera, p, fp32=False, threads=4), ref)
    assert np.array_equal(O.render(s2.desc, s2.camera, p, fp32=False, threads=4), ref)


def test_motion_changes_image_and_hits(g, O):
    s0 = g.Scene("simple", width=48)
    s1 = g.Scene("simple", width=48, motion=((0.5, 0.3, 2.5), (0.2, 0.0, -1.0)))
    c = s1.camera
    assert list(c.center_motion_dir) == pytest.approx([0.5, 0.3, 0.5])
    assert list(c.look_at_motion_dir) == pytest.approx([0.2, 0.0, 0.0])
    t0, _, _ = O.primary_hits(s0.desc, s0.camera, 3, 0, fp32=False)
    t1, _, _ = O.primary_hits(s1.desc, s1.camera, 3, 0, fp32=False)
    assert (t0 != t1).any()


@pytest.mark.gpu
def test_invalid_moving_camera_rejected(g, ctx):
    """A moving camera without the cached viewport is an invalid argument
    (no CPU fallback, no silent static render)."""
    s = g.Scene("simple", width=32)
    cam = s.camera
    cam.camera_motion = 1
    cam.viewport_width = 0.0
    ctx.upload(s.desc)
    with pytest.raises(g.RTError) as e:
        ctx.render(cam, g.make_params(1, 3))
    assert e.value.code == -1


@pytest.mark.gpu
@pytest.mark.parametrize("name,kw", CASES, ids=IDS)
def test_moving_camera_hits_bit_exact(g, O, ctx, name, kw):
    s = g.Scene(name, **kw)
    cam = s.camera
    ctx.upload(s.desc)
    for sample in (0, 5):
        tg, pg, t_g = ctx.primary_hits(cam, 4321, sample)
        to, po, t_o = O.primary_hits(s.desc, cam, 4321, sample, fp32=True)
        mism = np.flatnonzero((tg != to) | (pg != po))
        assert mism.size == 0, f"{mism.size} mismatches, first {mism[:5]}"
        same = tg >= 0
        assert np.array_equal(t_g[same], t_o[same].astype(np.float32))
        assert same.any()


@pytest.mark.gpu
@pytest.mark.parametrize("name,kw", CASES, ids=IDS)
def test_moving_camera_radiance_parity(g, O, ctx, name, kw):
    s = g.Scene(name, **kw)
    cam = s.camera
    spp = 8
    ctx.upload(s.desc)
    p = g.make_params(spp, min(cam.max_depth, 10), seed=31)
    gpu, _ = ctx.render(cam, p)
    ref = O.render(s.desc, cam, p, fp32=True)
    from tests.test_gpu_parity import fp32_bar
    fp32_bar(name, gpu, ref, spp)
    assert gpu.mean() > 0
