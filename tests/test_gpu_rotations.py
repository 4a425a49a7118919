"""Sibling RotateX objects whose hits leave their bounding boxes.
Marked gpu.

RotateX / RotateZ (transform.go:194-353) rotate the ray one way in Hit and
the bbox corners the other way, so an object can report a hit outside its
own bbox and outside its parent BVHNode's.  BVHNode.Hit (bvh.go:219-239)
tests its own box once, then calls the left child over [tmin, tmax] and the
right child over [tmin, closest hit of the left] with no box test.  Here a
BVHNode holds two such objects: the left one's quad lies at z = -3, the
right one's at z = -2.5 over half the window, while both report a bbox at
z = -9.  A camera ray down -z enters the parent's box at t = 9, hits the left
quad at t = 3 and the right quad at t = 2.5: the reference keeps the right
one.  The device must too (flatten.cpp tlas_item: such a node stays a BVH4
node of its own, its rotated children in unbounded slots, visited in DFS
order).  Checked against the oracle's fp32 mirror of the reference's
recursion: first hits bit-exact, radiance to the fp32 bar."""
import math

import numpy as np
import pytest

from tests.scene_builder import Builder, pinhole
from tests.test_gpu_parity import fp32_bar

pytestmark = pytest.mark.gpu


def rot90_x(b, y_obj, x0, x1, mat):
    """Translate(RotateX(quad at y = y_obj, 90 degrees)) whose quad lies at
    world z = -3 - (y_obj + 3) ... (true z = -y_obj + tz) and whose reported
    bbox sits at z = y_obj + tz = -9."""
    q = b.quad((x0, y_obj, -1.0), (x1 - x0, 0.0, 0.0), (0.0, 0.0, 2.0), mat)
    r = b.rotate_x(q, math.sin(math.radians(90.0)), math.cos(math.radians(90.0)))
    tz = -9.0 - y_obj
    return b.translate(r, (0.0, 0.0, tz))


def sibling_scene(g):
    b = Builder(g)
    red, green, grey = b.lambertian((0.8, 0.2, 0.2)), b.lambertian((0.2, 0.8, 0.2)), b.lambertian((0.5, 0.5, 0.5))
    left = rot90_x(b, -3.0, -1.0, 1.0, red)      # true z = -3, bbox z = -9
    right = rot90_x(b, -3.25, 0.0, 1.0, green)   # true z = -2.5 (x >= 0 only), bbox z = -9
    pair = b.bvh_node(left, right)
    back = b.quad((-30.0, -30.0, -20.0), (60.0, 0.0, 0.0), (0.0, 60.0, 0.0), grey)
    root = b.bvh_node(pair, back)
    d = b.desc(root)
    w, h = 48, 32
    cam = pinhole(g, w, h, (0, 0, 0), (-0.6 + 0.0125, 0.4 - 0.0125, -1.0), (0.025, 0, 0), (0, -0.025, 0),
                  max_depth=3, sky=True)
    return d, cam


def test_right_sibling_hit_outside_the_parent_box(g, O, ctx):
    d, cam = sibling_scene(g)
    ctx.upload(d)
    tg, pg, t_g = ctx.primary_hits(cam, 3, 0)
    to, po, t_o = O.primary_hits(d, cam, 3, 0, fp32=True)
    assert np.array_equal(tg, to) and np.array_equal(pg, po)
    hit = tg >= 0
    assert np.array_equal(t_g[hit], t_o[hit].astype(np.float32))
    # the case itself: rays through x > 0 within the quads take the right
    # object's quad at t = 2.5 (the oracle's recursion does), the others the
    # left one's at t = 3
    ts = np.round(t_g[hit].astype(np.float64), 3)
    assert np.any(np.isclose(ts, 2.5, atol=0.05)) and np.any(np.isclose(ts, 3.0, atol=0.1))
    spp = 4
    got, _ = ctx.render(cam, g.make_params(spp, cam.max_depth, seed=3))
    ref = O.render(d, cam, g.make_params(spp, cam.max_depth, seed=3), fp32=True)
    fp32_bar("sibling-rotations", got, ref, spp)
