"""Multi-device contexts behind the C-ABI (rt_ctx_create_multi).

The reference renders with a pool of workers over buckets
(bucket_renderer.go:193-213, main.go:83-86); the drop-in's pool is one GPU
per worker: rt_render deals the buckets round-robin over the context's
devices and each device writes its own pixels into the primary's frame.  On
the one-GPU box the device list repeats device 0 (two or three contexts on the
same GPU, concurrent streams), which exercises the same dealing, threading,
stream joins and combine as an 8-GPU node.  Each pixel has exactly one owner
and the RNG is keyed by global pixel id, so every frame must be bit-identical
to the one-device frame.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lucy(g):
    return g.Scene("cornell-lucy", width=96, aspect=16.0 / 9.0, lucy_rings=60, lucy_cols=80)


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_multi_device_frame_equals_one_device(g, lucy, devices):
    cam = lucy.camera
    p = g.make_params(6, cam.max_depth, seed=13)
    one = g.Context(0)
    multi = g.Context(devices=devices)
    try:
        assert multi.num_devices == len(devices) and one.num_devices == 1
        one.upload(lucy.desc)
        multi.upload(lucy.desc)
        a, _ = one.render(cam, p)
        b, st = multi.render(cam, p)
        assert np.array_equal(a, b)
        assert st.samples == cam.image_width * cam.image_height * 6
        # a bucket subset overwrites only its pixels; the rest keep the caller's values
        bk = g.generate_buckets(cam.image_width, cam.image_height, 32)[:5]
        fill = np.full_like(a, -3.0)
        multi.render(cam, g.make_params(6, cam.max_depth, seed=13, buckets=bk), fill)
        mask = np.zeros(a.shape[:2], bool)
        for x, y, w, h in bk:
            mask[y:y + h, x:x + w] = True
        assert np.array_equal(fill[mask], a[mask]) and (fill[~mask] == -3.0).all()
        # progressive accumulation across calls (sample_offset, accumulate)
        acc, _ = multi.render(cam, g.make_params(3, cam.max_depth, seed=13))
        multi.render(cam, g.make_params(3, cam.max_depth, seed=13, sample_offset=3, accumulate=True), acc)
        np.testing.assert_allclose(acc, a, rtol=1e-5, atol=1e-5)
    finally:
        multi.close()
        one.close()


def test_multi_device_render_device_async(g, lucy):
    """rt_render_device on the caller's stream: every device's share joins it."""
    import torch
    cam = lucy.camera
    p = g.make_params(4, cam.max_depth, seed=17)
    one = g.Context(0)
    multi = g.Context(devices=[0, 0])
    try:
        one.upload(lucy.desc)
        multi.upload(lucy.desc)
        ref, _ = one.render(cam, p)
        dev = torch.device("cuda", 0)
        buf = torch.full((cam.image_height * cam.image_width * 3,), 5.0, dtype=torch.float32, device=dev)
        torch.cuda.synchronize(dev)
        s = torch.cuda.Stream(dev)   # a real stream (the null stream would select the context's own)
        with torch.cuda.stream(s):
            buf.zero_()   # enqueued on the caller's stream before the render
            multi.render_device(cam, p, buf.data_ptr(), s.cuda_stream)
            out = buf.cpu().numpy().reshape(ref.shape)   # stream-ordered after the joins
        assert np.array_equal(out, ref)
        multi.sync()
        assert multi.last_render_kernel_ms() > 0.0
    finally:
        multi.close()
        one.close()


def test_multi_device_options_and_count(g):
    assert g.device_count() >= 1
    with pytest.raises(g.RTError):
        g.Context(devices=[0, 10_000])
    c = g.Context(devices=[0, 0])
    try:
        c.set_schedule(0, 32, 0)
        with pytest.raises(g.RTError):
            c.set_option(g.RT_OPT_REFILL, 99)
    finally:
        c.close()


@pytest.mark.parametrize("devices,first", [([0, 0, 0], 0), ([0, 0], 10), ([0, 0, 0, 0], 100)])
def test_dynamic_dealing_frame_equals_one_device(g, lucy, devices, first):
    """RT_DEAL_DYNAMIC (bucket_renderer.go:193-213's channel): every device
    claims runs of tiles from one counter until none are left.  Whatever the
    split, the frame is bit-identical to one device's and to the static
    split's, every tile is rendered exactly once, and the runs shrink as the
    list drains (more runs than devices when the first run is a small share)."""
    import torch
    cam = lucy.camera
    p = g.make_params(6, cam.max_depth, seed=13)
    one = g.Context(0)
    multi = g.Context(devices=devices)
    try:
        one.upload(lucy.desc)
        multi.upload(lucy.desc)
        a, _ = one.render(cam, p)
        multi.set_dealing("static")
        s, _ = multi.render(cam, p)
        st_tiles, st_runs = multi.last_dealing()
        assert np.array_equal(a, s)
        multi.set_dealing("dynamic", first)
        b, _ = multi.render(cam, p)
        tiles, runs = multi.last_dealing()
        assert np.array_equal(a, b)
        assert sum(tiles) == sum(st_tiles) > 0 and st_runs == [1] * len(devices)
        assert all((t > 0) == (r > 0) for t, r in zip(tiles, runs))
        if first == 10:
            assert sum(runs) > len(devices)
        # the asynchronous entry point on a caller stream: same frame
        dev = torch.device("cuda", 0)
        buf = torch.full((cam.image_height * cam.image_width * 3,), 5.0, dtype=torch.float32, device=dev)
        torch.cuda.synchronize(dev)
        cs = torch.cuda.Stream(dev)
        with torch.cuda.stream(cs):
            buf.zero_()
            multi.render_device(cam, p, buf.data_ptr(), cs.cuda_stream)
            out = buf.cpu().numpy().reshape(a.shape)
        assert np.array_equal(out, a)
        assert multi.last_render_kernel_ms() > 0.0
        with pytest.raises(g.RTError):
            multi.set_option(g.RT_OPT_DEALING, 7)
    finally:
        multi.close()
        one.close()
