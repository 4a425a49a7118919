"""The hand-derived known answers of tests/kat_cases.py (sampleAreaLight, a
Scale -> RotateY -> Translate instance, Volume.Hit with a fixed draw) through
the GPU, via the C-ABI: the production render for the NEE radiance, the
production k_extend's records (rt_extend_hits) for hits, hit points and
normals.  fp32 tolerances: the kernels compute in fp32."""
import numpy as np
import pytest

from tests import kat_cases as K

pytestmark = pytest.mark.gpu


def test_gpu_area_light_nee_closed_form(g, ctx):
    b, d, cam = K.area_light_scene(g)
    ctx.upload(d)
    got, _ = ctx.render(cam, g.make_params(4, 1, seed=K.SEED))
    np.testing.assert_allclose(got[0].astype(np.float64), K.area_light_expected(spp=4), rtol=2e-5, atol=1e-6)


def test_gpu_instance_chain_point_and_normal(g, ctx):
    b, d, cam, top, q = K.instance_scene(g)
    ctx.upload(d)
    t_top, t_prim, t_t, _ = ctx.extend_hits(cam, K.SEED, 0, 0)
    assert (t_top == top).all() and (t_prim == q).all()
    np.testing.assert_allclose(t_t, 1.0, rtol=2e-6)
    _, _, _, ray = ctx.extend_hits(cam, K.SEED, 0, 1)
    P, N = K.instance_world_point(), K.instance_expected_normal()
    for pix in range(cam.image_width):
        np.testing.assert_allclose(ray[pix, :3], P, atol=1e-5)
        np.testing.assert_allclose(ray[pix, 3:] - K.random_unit_vector(K.SEED, pix, 0, 0), N, atol=1e-5)


def test_gpu_volume_hit_fixed_draw(g, ctx):
    b, d, cam, vol, back = K.volume_scene(g)
    ctx.upload(d)
    ids, ts = K.volume_expected()
    want = np.array([vol if i == "vol" else back for i in ids])
    for probe in ("primary", "extend"):
        if probe == "primary":
            top, prim, t = ctx.primary_hits(cam, K.SEED, 0)
        else:
            top, prim, t, _ = ctx.extend_hits(cam, K.SEED, 0, 0)
        assert np.array_equal(prim, want), probe
        np.testing.assert_allclose(t, ts, rtol=2e-6)
