"""Schedule independence of the closest hit on the headline config (C4).

north_star: integer hit-index work bit-exact.  The production closest-hit
kernel (k_extend) is persistent: which rays share a wave, and when, depends on
the batch size, the claim-pool refill threshold and the grid size.  The
traversal is built so that none of that changes a hit (DESIGN.md §3
"Determinism": a non-speculative phase 1 and a widened box cull), so:

  * the whole frame is bit-identical under three different schedules;
  * the first-bounce hit records written by the production k_extend are
    identical under those schedules and equal, id for id and t for t, to the
    CPU oracle's fp32 mode (which walks the caller's reference BVH in Go's
    DFS order, bvh.go:219-239);
  * the radiance matches the fp32 oracle within the fp32 bar (test_gpu_parity.fp32_bar).

CornellBoxLucy with the full 280K-triangle mesh at 320x180, 16 spp.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 21
SPP = 16


@pytest.fixture(scope="module")
def lucy(g):
    s = g.Scene("cornell-lucy", width=320, aspect=16.0 / 9.0)
    assert s.camera.image_height == 180
    return s


def _schedules(npix):
    # (batch slots, refill, max persistent blocks, streams): automatic (two
    # twin streams); three batches per frame with waves that claim only when
    # every lane idles on a small grid, one stream; many small batches
    # claiming as soon as one lane idles, two streams; the pixels split over
    # three and four streams
    return [(0, 0, 0, 0), (npix * 6, 64, 37, 1), (npix * 2, 1, 600, 2), (npix * 4, 4, 0, 3), (0, 0, 0, 4)]


def test_c4_full_mesh_schedule_independent(g, O, lucy):
    cam = lucy.camera
    npix = cam.image_width * cam.image_height
    c = g.Context(0)
    try:
        c.upload(lucy.desc)
        assert c.info().triangles >= 280000
        p = g.make_params(SPP, cam.max_depth, seed=SEED)
        frames, hits = [], []
        for slots, refill, blocks, streams in _schedules(npix):
            c.set_schedule(slots, refill, blocks, streams)
            f, _ = c.render(cam, p)
            frames.append(f)
            hits.append([c.extend_first_hits(cam, SEED, k) for k in (0, 7)])
        for k in range(1, len(frames)):
            assert np.array_equal(frames[0], frames[k]), f"schedule {k}: frame differs"
            for (ta, pa, da), (tb, pb, db) in zip(hits[0], hits[k]):
                assert np.array_equal(ta, tb) and np.array_equal(pa, pb) and np.array_equal(da, db)
        # production hits == oracle fp32 (ids and t), every pixel
        for sample, (tg, pg, t_g) in zip((0, 7), hits[0]):
            to, po, t_o = O.primary_hits(lucy.desc, cam, SEED, sample, fp32=True)
            mism = np.flatnonzero((tg != to) | (pg != po))
            assert mism.size == 0, f"sample {sample}: {mism.size} hit-id mismatches, first {mism[:5]}"
            hit = tg >= 0
            assert hit.mean() > 0.3
            assert np.array_equal(t_g[hit], t_o[hit].astype(np.float32)), f"sample {sample}: hit t differs"
        # the probe kernel (whole-ray traversal) agrees with the production kernel
        tp, pp, _ = c.primary_hits(cam, SEED, 0)
        assert np.array_equal(tp, hits[0][0][0]) and np.array_equal(pp, hits[0][0][1])
        ref = O.render(lucy.desc, cam, p, fp32=True, threads=16)
        from tests.test_gpu_parity import fp32_bar
        mse, _ = fp32_bar("C4 320x180 16spp full mesh, 5 schedules bit-identical", frames[0], ref, SPP)
    finally:
        c.close()


@pytest.mark.parametrize("name,kw", [("cornell", dict(width=64)), ("random", dict(width=96)),
                                     ("hdri-test", dict(width=96))])
def test_other_configs_schedule_independent(g, name, kw):
    """C3 (fog: volumes in closest-hit and shadow traversal), C2, C5."""
    s = g.Scene(name, **kw)
    cam = s.camera
    npix = cam.image_width * cam.image_height
    c = g.Context(0)
    try:
        c.upload(s.desc)
        p = g.make_params(8, cam.max_depth, seed=SEED)
        frames = []
        for slots, refill, blocks, streams in _schedules(npix):
            c.set_schedule(slots, refill, blocks, streams)
            frames.append(c.render(cam, p)[0])
        for k in range(1, len(frames)):
            assert np.array_equal(frames[0], frames[k]), f"{name}: schedule {k} frame differs"
    finally:
        c.close()


@pytest.mark.parametrize("streams", [3, 4])
def test_many_streams_fresh_context(g, streams):
    """Three / four twins on a fresh context whose batch buffers are sized
    exactly for this render (no larger earlier batch, one batch per frame):
    every twin's queue counters and NEE job words lie inside the allocation
    (api.cpp render_wave checks the slices before launching) and the frame
    equals the one-stream frame bit for bit."""
    s = g.Scene("cornell", width=96)
    cam = s.camera
    npix = cam.image_width * cam.image_height
    spp = 8
    p = g.make_params(spp, cam.max_depth, seed=SEED)
    frames = []
    for st in (streams, 1):
        c = g.Context(0)
        try:
            c.upload(s.desc)
            c.set_schedule(npix * spp, 0, 0, st)
            frames.append(c.render(cam, p)[0])
        finally:
            c.close()
    assert np.array_equal(frames[0], frames[1])


def test_schedule_option_validation(g, ctx):
    with pytest.raises(g.RTError):
        ctx.set_option(g.RT_OPT_REFILL, 65)
    with pytest.raises(g.RTError):
        ctx.set_option(g.RT_OPT_BATCH_SLOTS, -1)
    with pytest.raises(g.RTError):
        ctx.set_option(g.RT_OPT_STREAMS, 5)
    ctx.set_schedule(0, 0, 0, 0)
