"""Host-side rt mirror: scene builders (scenes.go), NewBVHNode (bvh.go) vs the
oracle's restatement, loaders (image_loader.go, obj_loader.go)."""
import os

import numpy as np
import pytest

RT_SPHERE, RT_QUAD, RT_TRIANGLE, RT_PLANE, RT_LIST, RT_BVH_NODE, RT_BVH_LEAF = 1, 2, 3, 4, 5, 6, 7
RT_TRANSLATE, RT_ROTATE_Y, RT_SCALE, RT_VOLUME = 8, 10, 12, 13


def test_random_scene_counts(g):
    s = g.Scene("random")
    h = s.hittables()
    nsph = int((h["kind"] == RT_SPHERE).sum())
    # scenes.go:52-65 grid of 400 candidates, ~10% dropped (chooseMat >= 0.9)
    # and a few too close to (4,0.2,0): SURVEY.md §0.7 range 334-374 + 3 big.
    assert 334 + 3 <= nsph <= 374 + 3
    assert int((h["kind"] == RT_PLANE).sum()) == 1
    cam = s.camera
    assert (cam.image_width, cam.image_height, cam.samples_per_pixel, cam.max_depth) == (1200, 675, 500, 50)
    assert cam.defocus_angle == 0.6 and cam.use_sky_gradient == 1
    moving = h[(h["kind"] == RT_SPHERE) & (np.abs(h["p"][:, 4]) > 0)]
    assert len(moving) > 80 and (moving["p"][:, 4] < 0.5).all()


def test_random_scene_seeded(g):
    a = g.Scene("random", seed=1).hittables()
    b = g.Scene("random", seed=1).hittables()
    c = g.Scene("random", seed=2).hittables()
    assert np.array_equal(a["p"], b["p"])
    assert a.shape != c.shape or not np.array_equal(a["p"], c["p"])


def test_cornell_structure(g):
    s = g.Scene("cornell")
    h = s.hittables()
    k = h["kind"]
    assert int((k == RT_QUAD).sum()) == 6 + 12 + 6     # walls+light, 2 boxes, fog boundary
    assert int((k == RT_VOLUME).sum()) == 1
    vol = h[k == RT_VOLUME][0]
    assert vol["p"][0] == pytest.approx(-1000.0)         # -1/0.001
    assert int((k == RT_ROTATE_Y).sum()) == 2 and int((k == RT_TRANSLATE).sum()) == 2
    cam = s.camera
    assert (cam.image_width, cam.image_height, cam.max_depth) == (600, 600, 5)
    assert s.desc.contents.num_lights == 1
    # light quad Q=(213,554,227), u=(130,0,0), v=(0,0,105): normal (0,-1,0)?? cross(u,v)=(0,-13650,0)
    li = s.desc.contents.lights[0]
    assert list(h[li]["p"][12:15]) == [0.0, -1.0, 0.0]
    assert h[li]["p"][15] == pytest.approx(-554.0)


def test_lucy_synthetic_bounds_and_size(g):
    s = g.Scene("cornell-lucy")
    h = s.hittables()
    tri = h[h["kind"] == RT_TRIANGLE]
    assert len(tri) == 280000
    v = tri["p"][:, :9].reshape(-1, 3)
    np.testing.assert_allclose(v.min(0), [-465, -0.025, -267], atol=1e-9)
    np.testing.assert_allclose(v.max(0), [465, 1597, 267], atol=1e-9)
    assert int((h["kind"] == RT_SCALE).sum()) == 10     # 10 instances share one BLAS
    assert int((h["kind"] == RT_ROTATE_Y).sum()) == 8    # rot 0 skipped twice (transform.go:34)
    n = np.cross(v[1::3] - v[0::3], v[2::3] - v[0::3])
    assert (np.linalg.norm(n, axis=1) > 0).all()         # no degenerate triangles


def _bvh_encoding(h, ch, node):
    """Preorder encoding of the graph BVH like oracle_build_bvh: -1 internal,
    leaf = count + indices into the object list."""
    out = []

    def rec(i):
        e = h[i]
        if e["kind"] == RT_BVH_NODE and e["a"] != e["b"]:
            out.append(-1)
            rec(e["a"])
            rec(e["b"])
        else:
            leaf = h[e["a"]]
            kids = ch[leaf["a"]: leaf["a"] + leaf["b"]]
            out.append(len(kids))
            out.extend(int(k) for k in kids)

    rec(node)
    return out


@pytest.mark.parametrize("name,kw", [("cornell", {}), ("random", {}), ("cornell-lucy", dict(lucy_rings=40, lucy_cols=50))])
def test_world_bvh_matches_oracle_builder(g, O, name, kw):
    s = g.Scene(name, **kw)
    h, ch = s.hittables(), s.children()
    objs = s.world_objects()
    enc = _bvh_encoding(h, ch, s.desc.contents.root)
    boxes = h["bbox"][objs]
    ref = O.build_bvh(boxes)
    mapped = [x if i == 0 else x for i, x in enumerate(ref)]
    # map oracle leaf indices (positions in the object list) to hittable ids
    out, i = [], 0
    while i < len(ref):
        if ref[i] == -1:
            out.append(-1)
            i += 1
        else:
            n = ref[i]
            out.append(n)
            out.extend(int(objs[j]) for j in ref[i + 1: i + 1 + n])
            i += 1 + n
    assert enc == out


def test_mesh_blas_matches_oracle_builder(g, O):
    s = g.Scene("cornell-lucy", lucy_rings=30, lucy_cols=40)
    h, ch = s.hittables(), s.children()
    # the shared mesh BVH: child of the Scale wrappers
    mesh_root = int(h[h["kind"] == RT_SCALE][0]["a"])
    enc = _bvh_encoding(h, ch, mesh_root)
    tris = np.flatnonzero(h["kind"] == RT_TRIANGLE)   # emitted in leaf order; rebuild from bboxes
    # order of the triangles as given to NewBVHNode = synthetic generation order,
    # recover it from the leaf contents sorted by hittable index
    order = np.sort(tris)
    ref = O.build_bvh(h["bbox"][order])
    out, i = [], 0
    while i < len(ref):
        if ref[i] == -1:
            out.append(-1)
            i += 1
        else:
            n = ref[i]
            out.append(n)
            out.extend(int(order[j]) for j in ref[i + 1: i + 1 + n])
            i += 1 + n
    assert enc == out


def test_hdr_loader_matches_oracle_and_reference_stats(g, O):
    path = os.path.join(g.ASSET_DIR, "hdri", "abandoned_hall_01_1k.hdr")
    a = g.load_hdr(path)
    b = O.load_hdr(path)
    assert a.shape == (512, 1024, 3)
    assert np.array_equal(a, b)
    # max radiance 77.75, totalPower (hdri.go:189) ~ 293971.37
    assert a.max() == pytest.approx(77.75)
    assert O.hdri_total_power(a) == pytest.approx(293971.37, abs=0.01)


def test_hdr_rle_and_flat_known_answers(g, O, tmp_path):
    """RGBE decode (m+0.5)*2^(e-136), e==0 -> 0 (image_loader.go:364-383), for
    both scanline encodings (readHDRScanline / readRLEScanline)."""
    W, H = 8, 2
    px = [(128, 64, 32, 129), (0, 0, 0, 0), (255, 255, 255, 136), (1, 2, 3, 100)] * 2
    flat = b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n-Y 2 +X 8\n" + bytes(sum((list(p) for p in px), [])) * 2
    f1 = tmp_path / "flat.hdr"
    f1.write_bytes(flat)
    rle = bytearray(b"#?RADIANCE\n\n-Y 2 +X 8\n")
    for _ in range(H):
        rle += bytes([2, 2, 0, W])
        for c in range(4):
            comp = [p[c] for p in px]
            rle += bytes([8]) + bytes(comp)               # one raw run
    f2 = tmp_path / "rle.hdr"
    f2.write_bytes(bytes(rle))
    expect = np.zeros((H, W, 3))
    for x, p in enumerate(px):
        if p[3]:
            expect[:, x] = [(v + 0.5) * 2.0 ** (p[3] - 136) for v in p[:3]]
    for f in (f1, f2):
        assert np.array_equal(g.load_hdr(str(f)), expect)
        assert np.array_equal(O.load_hdr(str(f)), expect)


def test_obj_loader_roundtrip(g, tmp_path):
    path = str(tmp_path / "m.obj")
    assert g.rtscene().rts_write_synthetic_lucy_obj(path.encode(), 10, 12) == 0
    assert g.rtscene().rts_obj_triangle_count(path.encode()) == 2 * 10 * 12
    # fan triangulation + negative indices (obj_loader.go:62-97)
    q = tmp_path / "quad.obj"
    q.write_text("# c\nv 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nf 1/1/1 2 3 4\nf -4 -3 -2\n")
    assert g.rtscene().rts_obj_triangle_count(str(q).encode()) == 3
    bad = tmp_path / "bad.obj"
    bad.write_text("v 0 0 0\nf 1 2 3\n")
    assert g.rtscene().rts_obj_triangle_count(str(bad).encode()) < 0


def test_unknown_scene_errors(g):
    with pytest.raises(g.RTError):
        g.Scene("no-such-scene")
