"""Deep traversal stacks (the kernels' 128-entry bound, wavefront.h
kStackMax, probe.hip's 128-entry LDS variant).  Marked gpu.

A RotateX object (transform.go:201-237) keeps the world BVH in the
reference's own topology and traversal order (flatten.cpp dfs_order: two
stack words per entry), so a hand-built BVHNode chain (bvh.go) whose
subtree is always the left child makes every ray that crosses it push the
chain's quads one level after the other: the stack grows with the chain
depth and runs through the LDS ring into the global spill.  The quads all
cover the same window at distinct depths, so each such ray hits every
quad's box and the closest one is in the middle of the chain.  Checked
against the oracle's fp32 mirror: first hits bit-exact, radiance to the
fp32 bar of tests/test_gpu_parity.py.  A chain twice as deep exceeds the
bound and the upload fails with RT_ERR_UNSUPPORTED."""
import math

import numpy as np
import pytest

from tests.scene_builder import Builder, pinhole
from tests.test_gpu_parity import fp32_bar

pytestmark = pytest.mark.gpu


def chain_scene(g, depth):
    b = Builder(g)
    mats = [b.lambertian((0.2 + 0.6 * (i % 5) / 4, 0.5, 0.8 - 0.6 * (i % 3) / 2)) for i in range(6)]
    quads = []
    for i in range(depth):
        z = -5.0 - 0.05 * ((7 * i + depth // 2) % depth)   # distinct depths, the nearest mid-chain
        quads.append(b.quad((-3.5, -1.4, z), (7.0, 0.0, 0.0), (0.0, 2.8, 0.0), mats[i % 6]))
    cur = quads[-1]
    for q in reversed(quads[:-1]):
        cur = b.bvh_node(cur, q)                      # subtree left: visited first, the quad pushed
    s, c = math.sin(math.radians(30.0)), math.cos(math.radians(30.0))
    tilted = b.rotate_x(b.quad((3.6, -1.0, -4.0), (0.8, 0.0, 0.0), (0.0, 2.0, 0.0), mats[1]), s, c)
    root = b.bvh_node(cur, tilted)
    d = b.desc(root)
    w, h = 64, 24
    cam = pinhole(g, w, h, (0, 0, 0), (-4.0 + 0.0625, 1.5 - 0.0625, -4.0), (0.125, 0, 0), (0, -0.125, 0),
                  max_depth=4, sky=True)
    return b, d, cam


def test_deep_chain_beyond_64_entries(g, O, ctx):
    b, d, cam = chain_scene(g, 40)
    ctx.upload(d)
    info = ctx.info()
    assert 64 < info.stack_needed <= 128, info.stack_needed
    tg, pg, t_g = ctx.primary_hits(cam, 5, 0)
    to, po, t_o = O.primary_hits(d, cam, 5, 0, fp32=True)
    assert np.array_equal(tg, to) and np.array_equal(pg, po)
    hit = tg >= 0
    assert hit.sum() > cam.image_width * cam.image_height // 3
    assert np.array_equal(t_g[hit], t_o[hit].astype(np.float32))
    spp = 4
    got, _ = ctx.render(cam, g.make_params(spp, cam.max_depth, seed=5))
    ref = O.render(d, cam, g.make_params(spp, cam.max_depth, seed=5), fp32=True)
    fp32_bar("deep-chain", got, ref, spp)


def test_chain_beyond_the_bound_is_unsupported(g, ctx):
    b, d, cam = chain_scene(g, 96)
    with pytest.raises(g.RTError) as ei:
        ctx.upload(d)
    assert ei.value.code == -2   # RT_ERR_UNSUPPORTED (include/rtgpu.h)
