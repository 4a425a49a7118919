"""Integer hit work past the camera ray (north_star: "integer hit-index work
bit-exact").

rt_extend_hits reads back the hit records the production closest-hit kernel
(k_extend) wrote at bounce k, with the incoming ray it traced;
rt_shadow_visibility reads the NEE shadow jobs of bounce k and what the
any-hit kernel (k_shadow) found.  The fp32 oracle records the same per bounce
while it walks the caller's reference BVH recursively (rayColorInternal
camera.go:443-518: world.Hit at :449, sampleHDRILight's shadow ray :582,
sampleAreaLight's :639).

For every path whose incoming ray is bit-identical on both sides, the hit ids
and t must be equal, and so must the NEE rays traced and their visibility
(a lifted volume occluding a shadow ray is resolved in shading: the GPU then
has no such ray, the oracle an occluded one; the volume scenes therefore also
run with RT_VOLUMES_IN_BVH, where every shadow ray is traced and the traced
flags must match exactly).  Paths whose rays differ ("diverged": an earlier
bounce rounded differently) are counted and reported and bounded, never
compared.

Depth: every bounce the reference recurses through, up to the scene's
MaxDepth (camera.go:443-518) — RandomScene's 50 (scenes.go:72-73) and
HDRITestScene's 20 (scenes.go:444-445) — or until no path is alive on either
side.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 29
LIFTED, IN_BVH = 0, 1
# (id, scene, constructor kwargs, samples probed, max share of diverged
# paths, bounces probed (0: the scene's MaxDepth), volume placement)
CASES = [
    ("cornell-lucy", "cornell-lucy", dict(width=320, aspect=16.0 / 9.0), (0, 5), 2e-3, 0, LIFTED, "fp32"),  # C4, 280K mesh
    ("cornell", "cornell", dict(width=128), (0, 5), 2e-3, 0, LIFTED, "fp32"),              # C3, fog + area light
    ("cornell-in-bvh", "cornell", dict(width=96), (0,), 2e-3, 0, IN_BVH, "fp32"),          # C3, fog in the BVH
    ("random", "random", dict(width=192), (0, 5), 2e-3, 0, LIFTED, "fp32"),                # C2 to MaxDepth 50
    ("hdri-test", "hdri-test", dict(width=192), (0, 3), 2e-2, 0, LIFTED, "fp32"),          # C5 to MaxDepth 20
    ("cornell-smoke", "cornell-smoke", dict(width=96), (0,), 2e-3, 0, LIFTED, "fp32"),     # two lifted volumes
    ("cornell-smoke-in-bvh", "cornell-smoke", dict(width=96), (0,), 2e-3, 0, IN_BVH, "fp32"),
    ("cornell-rotations", "cornell-rotations", dict(width=96), (0,), 2e-3, 0, LIFTED, "fp32"),  # RotateX/Z, Scale
    ("hdri-nee", "hdri-nee", dict(width=96), (0,), 2e-2, 0, LIFTED, "fp32"),               # HDRI IS + area light
    # the 8-wide node format (RT_NODES_WIDE8) through the production kernels
    ("cornell-lucy-wide8", "cornell-lucy", dict(width=320, aspect=16.0 / 9.0), (0,), 2e-3, 0, LIFTED, "wide8"),
    ("random-wide8", "random", dict(width=192), (0,), 2e-3, 0, LIFTED, "wide8"),
    ("hdri-test-wide8", "hdri-test", dict(width=192), (0,), 2e-2, 0, LIFTED, "wide8"),
    ("cornell-wide8", "cornell", dict(width=96), (0,), 2e-3, 0, LIFTED, "wide8"),
]


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def compare_paths(g, O, name, kw, samples, bounces=0, volumes=LIFTED, nodes="fp32"):
    """Per bounce and sample: (alive paths, compared, diverged, id/t mismatches,
    NEE mismatches).  Raises nothing; the caller asserts."""
    s = g.Scene(name, **kw)
    cam = s.camera
    nb = bounces or cam.max_depth
    c = g.Context(0)
    rows = []
    try:
        c.set_option(g.RT_OPT_VOLUMES, g.RT_VOLUMES_IN_BVH if volumes == IN_BVH else g.RT_VOLUMES_LIFTED)
        c.set_node_format(nodes)
        c.upload(s.desc)
        assert c.info().node_format == {"fp32": g.RT_NODES_FP32, "wide8": g.RT_NODES_WIDE8}[nodes]
        lifted = c.info().volumes > 0
        for sample in samples:
            ot, op, ott, oray, onee = O.path_records(s.desc, cam, SEED, sample, nb, fp32=True, threads=16)
            for b in range(nb):
                if not np.any(ot[b] != -2):   # no path left on the oracle's side: the GPU must agree
                    gt = c.extend_hits(cam, SEED, sample, b)[0]
                    rows.append(dict(sample=sample, bounce=b, alive=int(np.sum(gt != -2)), compared=0,
                                     diverged=int(np.sum(gt != -2)), hit_mismatch=0, nee_mismatch=0, shadow_rays=0,
                                     first_bad=[]))
                    break
                gt, gp, gtt, gray = c.extend_hits(cam, SEED, sample, b)
                gnee = c.shadow_visibility(cam, SEED, sample, b)
                alive_g, alive_o = gt != -2, ot[b] != -2
                same_ray = alive_g & alive_o & np.all(_bits(gray) == _bits(oray[b]), axis=1)
                div = (alive_g | alive_o) & ~same_ray
                hit_bad = same_ray & ((gt != ot[b]) | (gp != op[b]) | (_bits(gtt) != _bits(ott[b])))
                ok = same_ray & ~hit_bad
                gf, gv = gnee & 3, (gnee >> 2) & 3
                of, ov = onee[b] & 3, (onee[b] >> 2) & 3
                nee_bad = ok & (((gv & ~gf) != 0) | (gv != ov) | ((gf & ~of) != 0))
                if not lifted:
                    nee_bad |= ok & (gf != of)
                bad = np.flatnonzero(hit_bad | nee_bad)[:4]
                rows.append(dict(sample=sample, bounce=b, alive=int(np.sum(alive_g | alive_o)),
                                 compared=int(np.sum(same_ray)), diverged=int(np.sum(div)),
                                 hit_mismatch=int(np.sum(hit_bad)), nee_mismatch=int(np.sum(nee_bad)),
                                 shadow_rays=int(np.sum(((gf & 1) != 0).astype(int) + ((gf & 2) != 0))),
                                 first_bad=[(int(p), (int(gt[p]), int(gp[p]), float(gtt[p]), int(gnee[p])),
                                             (int(ot[b][p]), int(op[b][p]), float(ott[b][p]), int(onee[b][p])))
                                            for p in bad]))
    finally:
        c.close()
    return rows


@pytest.mark.parametrize("cid,name,kw,samples,max_div,bounces,volumes,nodes", CASES, ids=[c[0] for c in CASES])
def test_bounce_hits_and_shadow_rays_bit_exact(g, O, cid, name, kw, samples, max_div, bounces, volumes, nodes):
    rows = compare_paths(g, O, name, kw, samples, bounces, volumes, nodes)
    for r in rows:
        print(f"{cid} sample {r['sample']} bounce {r['bounce']}: alive {r['alive']} compared {r['compared']} "
              f"diverged {r['diverged']} shadow rays {r['shadow_rays']} hit mismatches {r['hit_mismatch']} "
              f"NEE mismatches {r['nee_mismatch']}")
    assert sum(r["compared"] for r in rows if r["bounce"] > 0) > 0
    deepest = max(r["bounce"] for r in rows if r["compared"] > 0)
    print(f"{cid}: deepest compared bounce {deepest}, paths compared {sum(r['compared'] for r in rows)}, "
          f"diverged {sum(r['diverged'] for r in rows)}")
    for r in rows:
        assert r["hit_mismatch"] == 0 and r["nee_mismatch"] == 0, f"{name}: {r}"
        assert r["diverged"] <= max_div * max(r["alive"], 1), f"{name}: too many diverged paths {r}"
