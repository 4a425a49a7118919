"""C-ABI behaviour on the GPU beyond parity (rtgpu.h): the asynchronous
rt_render_device path and its error reporting, and scene refusals.  Marked gpu."""
import numpy as np
import pytest

from tests.scene_builder import Builder

pytestmark = pytest.mark.gpu


def test_render_device_equals_render_and_sync(g, ctx):
    """rt_render_device (the bench / multi-GPU path) renders the same frame as
    rt_render; rt_sync waits for it and reports no device error."""
    import torch
    s = g.Scene("cornell", width=64)
    cam = s.camera
    ctx.upload(s.desc)
    p = g.make_params(4, 5, seed=21)
    host, _ = ctx.render(cam, p)
    buf = torch.zeros(cam.image_height * cam.image_width * 3, dtype=torch.float32, device="cuda:0")
    stream = torch.cuda.current_stream()
    for _ in range(3):   # several renders in flight before the check
        buf.zero_()
        ctx.render_device(cam, p, buf.data_ptr(), stream.cuda_stream)
    ctx.sync()
    assert ctx.last_render_kernel_ms() > 0.0
    torch.cuda.synchronize()
    assert np.array_equal(buf.cpu().numpy().reshape(host.shape), host)


def _mesh_bvh(g, b, tris):
    """A BVHNode tree over triangles: median split, leaves of <= 4 wrapped as
    BVHNode{leaf, leaf} (bvh.go:120-217 shape)."""
    if len(tris) <= 4:
        return b.leaf_node(tris)
    m = len(tris) // 2
    lo, hi = _mesh_bvh(g, b, tris[:m]), _mesh_bvh(g, b, tris[m:])
    bb = [min(b.h[lo].bbox[0], b.h[hi].bbox[0]), max(b.h[lo].bbox[1], b.h[hi].bbox[1]),
          min(b.h[lo].bbox[2], b.h[hi].bbox[2]), max(b.h[lo].bbox[3], b.h[hi].bbox[3]),
          min(b.h[lo].bbox[4], b.h[hi].bbox[4]), max(b.h[lo].bbox[5], b.h[hi].bbox[5])]
    return b._add(g.RT_BVH_NODE, -1, lo, hi, bb, [])


@pytest.mark.parametrize("builder", ["reference", "sah", "device"])
def test_volume_with_mesh_boundary_refused(g, builder):
    """Volume.Hit over a BVH boundary is outside the device path: every BLAS
    builder refuses it with RT_ERR_UNSUPPORTED (the Go caller keeps its CPU
    renderer), including the device builder, whose placeholder root used to
    slip past the check."""
    b = Builder(g)
    m = b.lambertian((0.5, 0.5, 0.5))
    tris = []
    for i in range(12):           # a closed-ish fan of 48 triangles
        for k in range(4):
            x = float(i)
            tris.append(b.triangle((x, 0, k), (x + 1, 0, k), (x, 1, k + 0.5), m))
    mesh = _mesh_bvh(g, b, tris)
    iso = b.mat(g.RT_ISOTROPIC, b.solid((1, 1, 1)))
    vol = b.volume(mesh, 0.1, iso)
    root = b.listing([vol, b.sphere((0, 0, -5), 1.0, m)])
    c = g.Context(0)
    try:
        c.set_blas_builder(builder)
        with pytest.raises(g.RTError) as ei:
            c.upload(b.desc(root))
        assert ei.value.code == -2, str(ei.value)
    finally:
        c.close()


def test_node_format_option(g):
    """RT_OPT_NODE_FORMAT: only RT_NODES_FP32 / RT_NODES_QUANT8 / RT_NODES_WIDE8 are accepted;
    a quantised upload renders the same frame as the fp32 one on a scene
    whose hits sit well inside the boxes' margins (CornellBox, 4 spp), and a
    RotateX/Z scene silently keeps its fp32 nodes: its quant8 upload holds no
    quantised node array (the same device bytes as its fp32 upload), while
    CornellBox's holds one more array (64 B per node)."""
    c = g.Context(0)
    try:
        with pytest.raises(g.RTError):
            c.set_option(g.RT_OPT_NODE_FORMAT, 7)
        frames, nbytes, nodes = {}, {}, {}
        used = {}
        for fmt in ("fp32", "quant8", "wide8"):
            c.set_node_format(fmt)
            for name in ("cornell", "cornell-rotations"):
                s = g.Scene(name, width=48)
                c.upload(s.desc)
                info = c.info()
                nbytes[fmt, name], nodes[name] = info.device_bytes, info.nodes
                used[fmt, name] = info.node_format
                frames[fmt, name], _ = c.render(s.camera, g.make_params(4, 5, seed=3))
        for name in ("cornell", "cornell-rotations"):
            assert np.array_equal(frames["fp32", name], frames["quant8", name]), name
            assert np.array_equal(frames["fp32", name], frames["wide8", name]), name
        # the 8-wide format is taken by CornellBox, not by the RotateX/Z scene
        assert used["wide8", "cornell"] == g.RT_NODES_WIDE8 and used["wide8", "cornell-rotations"] == g.RT_NODES_FP32
        assert used["quant8", "cornell"] == g.RT_NODES_QUANT8 and used["fp32", "cornell"] == g.RT_NODES_FP32
        assert nbytes["quant8", "cornell-rotations"] == nbytes["fp32", "cornell-rotations"]
        assert nbytes["quant8", "cornell"] >= nbytes["fp32", "cornell"] + 64 * nodes["cornell"]
    finally:
        c.close()


def test_render_rgba8_pass(g, O):
    """rt_render_rgba8 (one progressive pass, bucket_renderer.go:257-301): the
    device framebuffer is the reference quantisation (:276-285) of the device
    sums, bit for bit; the sums equal rt_render's; a later call over a bucket
    subset rewrites only those buckets' RGBA8 pixels; one and two devices agree."""
    s = g.Scene("cornell", width=64)
    cam = s.camera
    for devices in (None, [0, 0]):
        c = g.Context(0, devices=devices)
        try:
            c.upload(s.desc)
            p = g.make_params(4, 5, seed=31)
            rgba, st = c.render_rgba8(cam, p)
            sums = c.frame_sums(cam)
            ref, _ = c.render(cam, p)
            assert np.array_equal(sums, ref)
            assert np.array_equal(rgba, O.tonemap(sums, 4))
            assert st.samples == cam.image_width * cam.image_height * 4
            bk = g.generate_buckets(cam.image_width, cam.image_height, 32)[:1]
            rgba2, _ = c.render_rgba8(cam, g.make_params(1, 3, seed=7, buckets=bk))
            x, y, w, h = bk[0]
            mask = np.zeros(rgba.shape[:2], bool)
            mask[y:y + h, x:x + w] = True
            assert np.array_equal(rgba2[~mask], rgba[~mask])
            assert np.array_equal(rgba2[mask], O.tonemap(c.frame_sums(cam), 1)[mask])
        finally:
            c.close()


def test_kernel_times_pair_twin_launches(g, ctx):
    """rt_last_kernel_times: with twin streams the two halves' launches of a
    kernel and bounce count as one launch (their union interval), so both
    schedules report one extend / shade / shadow launch per bounce; the
    twins field names the schedule, and the frames are bit-identical."""
    s = g.Scene("cornell", width=64)
    cam = s.camera
    ctx.upload(s.desc)
    p = g.make_params(8, 5, seed=5)
    frames, times = {}, {}
    try:
        ctx.set_kernel_timing(True)
        for streams in (1, 2, 4):
            ctx.set_option(g.RT_OPT_STREAMS, streams)
            frames[streams], _ = ctx.render(cam, p)
            times[streams] = ctx.last_kernel_times()
    finally:
        ctx.set_option(g.RT_OPT_STREAMS, 0)
        ctx.set_kernel_timing(False)
    assert np.array_equal(frames[1], frames[2]) and np.array_equal(frames[1], frames[4])
    for streams, t in times.items():
        assert t["twins"] == streams
        for k in ("extend", "shade", "shadow"):
            assert t[f"{k}_launches"] == 5, (streams, k, t)
            assert t[f"{k}_ms"] > 0.0


@pytest.mark.parametrize("name", ["cornell", "cornell-smoke"])
def test_lifted_volumes_equal_volumes_in_bvh(g, ctx, name):
    """RT_OPT_VOLUMES: volumes lifted out of the world BVH and tested by
    k_shade's volume variant (closest hit by the tie rule, NEE shadow rays
    cleared when a volume occludes them) render the same frame, bit for bit,
    as volumes tested inside the traversal; unknown values are refused."""
    s = g.Scene(name, width=64)
    p = g.make_params(8, 5, seed=29)
    frames = {}
    try:
        with pytest.raises(g.RTError):
            ctx.set_option(g.RT_OPT_VOLUMES, 2)
        for mode in (g.RT_VOLUMES_IN_BVH, g.RT_VOLUMES_LIFTED):
            ctx.set_option(g.RT_OPT_VOLUMES, mode)
            ctx.upload(s.desc)
            frames[mode], _ = ctx.render(s.camera, p)
    finally:
        ctx.set_option(g.RT_OPT_VOLUMES, g.RT_VOLUMES_LIFTED)
    assert np.isfinite(frames[g.RT_VOLUMES_LIFTED]).all()
    assert np.array_equal(frames[g.RT_VOLUMES_IN_BVH], frames[g.RT_VOLUMES_LIFTED])


@pytest.mark.parametrize("name", ["cornell-lucy", "cornell", "random"])
def test_collapse_option_same_frame(g, ctx, name):
    """RT_OPT_BVH4_COLLAPSE: the SAH-optimal collapse (default) uploads fewer
    BVH4 nodes than the greedy one (or as many) and renders the same frame,
    bit for bit (the closest hit does not depend on the node topology);
    unknown values are refused."""
    s = g.Scene(name, width=64, **(dict(lucy_rings=60, lucy_cols=80) if name == "cornell-lucy" else {}))
    p = g.make_params(8, 5, seed=31)
    frames, nodes = {}, {}
    try:
        with pytest.raises(g.RTError):
            ctx.set_option(g.RT_OPT_BVH4_COLLAPSE, 2)
        for mode in (g.RT_COLLAPSE_GREEDY, g.RT_COLLAPSE_SAH):
            ctx.set_option(g.RT_OPT_BVH4_COLLAPSE, mode)
            ctx.upload(s.desc)
            nodes[mode] = ctx.info().nodes
            frames[mode], _ = ctx.render(s.camera, p)
    finally:
        ctx.set_option(g.RT_OPT_BVH4_COLLAPSE, g.RT_COLLAPSE_SAH)
    assert nodes[g.RT_COLLAPSE_SAH] <= nodes[g.RT_COLLAPSE_GREEDY]
    assert np.isfinite(frames[g.RT_COLLAPSE_SAH]).all()
    assert np.array_equal(frames[g.RT_COLLAPSE_GREEDY], frames[g.RT_COLLAPSE_SAH])


@pytest.mark.parametrize("name,kw,nodes", [("random", dict(width=160), "fp32"), ("hdri-test", dict(width=160), "fp32"),
                                           ("random", dict(width=160), "wide8"),
                                           ("cornell", dict(width=64), "fp32")])
def test_tail_kernel_same_frame(g, name, kw, nodes):
    """RT_OPT_TAIL: the long-tail kernel (k_tail) that carries the last paths
    of a deep render without lights to their ends renders the same frame, bit
    for bit, as every bounce through the per-bounce kernels, at every hand-off
    size (2 = almost never, 2^30 = at the first check) and with both twin
    counts; a scene with lights (cornell) never hands off.  Negative values
    are refused."""
    s = g.Scene(name, **kw)
    cam = s.camera
    p = g.make_params(16, cam.max_depth, seed=7)
    c = g.Context(0)
    try:
        with pytest.raises(g.RTError):
            c.set_option(g.RT_OPT_TAIL, -1)
        c.set_node_format(nodes)
        c.upload(s.desc)
        frames = {}
        for tail in (1, 2, 1 << 14, 1 << 30):
            for streams in (1, 2):
                c.set_tail(tail)
                c.set_schedule(streams=streams)
                frames[tail, streams], _ = c.render(cam, p)
        ref = frames[1, 1]
        assert np.isfinite(ref).all() and ref.sum() > 0
        for k, f in frames.items():
            assert np.array_equal(f, ref), k
    finally:
        c.close()


@pytest.mark.parametrize("name,kw,nodes,spp", [("cornell-lucy", dict(width=320, aspect=16.0 / 9.0), "fp32", 8),
                                               ("cornell", dict(width=96), "fp32", 16),
                                               ("hdri-nee", dict(width=96), "fp32", 8),
                                               ("cornell-smoke", dict(width=96), "quant8", 8),
                                               ("cornell-lucy", dict(width=160, aspect=16.0 / 9.0), "wide8", 8)])
def test_bounce_overlap_same_frame(g, name, kw, nodes, spp):
    """RT_OPT_OVERLAP: bounce b's k_shadow / k_nee_apply on a second stream
    per part beside bounce b + 1's k_extend (parity sets of the NEE counters,
    a spill area per stream) renders the same frame, bit for bit, as the
    serial schedule, with one to three parts and several batches per frame
    (the host emulation runs the most separated order under ASan,
    tests/test_flatten_host.py::test_bounce_overlap_bit_identical).  Values
    outside 0..2 are refused."""
    s = g.Scene(name, **kw)
    cam = s.camera
    p = g.make_params(spp, cam.max_depth, seed=13)
    c = g.Context(0)
    try:
        for bad in (-1, 3):
            with pytest.raises(g.RTError):
                c.set_option(g.RT_OPT_OVERLAP, bad)
        c.set_node_format(nodes)
        c.upload(s.desc)
        frames = {}
        for overlap in (1, 2):
            for streams in (1, 2, 3):
                for slots in (0, 3 * cam.image_width * cam.image_height):   # one batch / several batches
                    c.set_overlap(overlap)
                    c.set_schedule(streams=streams, batch_slots=slots)
                    frames[overlap, streams, slots], _ = c.render(cam, p)
        ref = frames[1, 1, 0]
        assert np.isfinite(ref).all() and ref.sum() > 0
        for k, f in frames.items():
            assert np.array_equal(f, ref), k
    finally:
        c.close()


def test_measured_read_bandwidth(g, ctx):
    """rt_measure_read_bandwidth: the roofline's measured HBM read peak (a
    coalesced stream over 1 GiB, larger than the Infinity Cache) lies between
    a quarter of the 8 TB/s spec and the spec; bad arguments are refused."""
    gbs = ctx.measure_read_bandwidth(1 << 30, 4)
    print(f"measured stream-read peak {gbs:.0f} GB/s")
    assert 2000.0 < gbs <= 8000.0
    with pytest.raises(g.RTError):
        ctx.measure_read_bandwidth(1024, 4)


def test_batch_slots_follow_free_memory(g):
    """The automatic batch size (85 % of the free HBM, api.cpp rt_render):
    with all but about 3 GB of the device held by another allocation, a
    frame whose one-batch size (37.7 M slots, 8.7 GB) does not fit renders in
    several batches, and the frame is the one rendered in a single batch once
    the memory is back."""
    import torch
    s = g.Scene("cornell", width=96)
    cam = s.camera
    p = g.make_params(4096, cam.max_depth, seed=5)
    c = g.Context(0)
    try:
        c.upload(s.desc)
        free, _ = torch.cuda.mem_get_info(0)
        hold = torch.empty(max(0, free - (3 << 30)), dtype=torch.uint8, device="cuda:0")
        try:
            tight, _ = c.render(cam, p)
            left, _ = torch.cuda.mem_get_info(0)
            assert left < (3 << 30)
        finally:
            del hold
            torch.cuda.empty_cache()
        c.set_schedule(batch_slots=cam.image_width * cam.image_height * 4096)
        whole, _ = c.render(cam, p)
        assert np.isfinite(whole).all() and whole.sum() > 0
        assert np.array_equal(tight, whole)
    finally:
        c.close()
