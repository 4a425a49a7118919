#!/usr/bin/env python3
"""Frame and per-ray diff of two node formats on the GPU (diagnostic).

Renders one scene with two node formats (RT_OPT_NODE_FORMAT) and reports the
pixels whose float3 sums differ; for those pixels it then reads the
production k_extend hit records (rt_extend_hits) of every sample and bounce
in both formats and prints the first records that differ, with the ray.

usage: tools/format_diff.py [scene] [width] [spp] [fmtA] [fmtB] [seed]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import __graft_entry__ as ge
    g = ge.load_package()
    scene = sys.argv[1] if len(sys.argv) > 1 else "cornell-lucy"
    width = int(sys.argv[2]) if len(sys.argv) > 2 else 1200
    spp = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    fa = sys.argv[4] if len(sys.argv) > 4 else "fp32"
    fb = sys.argv[5] if len(sys.argv) > 5 else "wide8"
    seed = int(sys.argv[6]) if len(sys.argv) > 6 else 1
    s = g.Scene(scene, width=width, aspect=16.0 / 9.0)
    cam = s.camera
    ctx = {}
    frames = {}
    for f in (fa, fb):
        c = g.Context(0)
        c.set_node_format(f)
        c.upload(s.desc)
        print(f, "node format in use:", c.info().node_format, "nodes8:", c.info().nodes8, flush=True)
        frames[f], _ = c.render(cam, g.make_params(spp, cam.max_depth, seed=seed))
        ctx[f] = c
    a, b = frames[fa].reshape(-1, 3), frames[fb].reshape(-1, 3)
    bad = np.flatnonzero(np.any(a != b, axis=1))
    print(f"{scene} {cam.image_width}x{cam.image_height} {spp} spp: {len(bad)} pixels differ; sums "
          f"{a.astype(np.float64).sum()!r} / {b.astype(np.float64).sum()!r}", flush=True)
    # the samples of the first differing pixels that differ: one-pixel
    # renders of one sample each (sample_offset), then the hit records of
    # every bounce of that sample in both formats
    W = cam.image_width
    for p in bad[:3]:
        x, y = int(p % W), int(p // W)
        hits = []
        for smp in range(spp):
            one = {}
            for f in (fa, fb):
                fr, _ = ctx[f].render(cam, g.make_params(1, cam.max_depth, seed=seed, sample_offset=smp,
                                                         buckets=[(x, y, 1, 1)]))
                one[f] = fr.reshape(-1, 3)[p]
            if np.any(one[fa] != one[fb]):
                hits.append(smp)
                print(f"pixel ({x},{y}) sample {smp}: {one[fa].tolist()} vs {one[fb].tolist()}", flush=True)
        for smp in hits[:2]:
            for bounce in range(cam.max_depth):
                ta, pa, tta, raya = ctx[fa].extend_hits(cam, seed, smp, bounce)
                tb, pb, ttb, rayb = ctx[fb].extend_hits(cam, seed, smp, bounce)
                na = ctx[fa].shadow_visibility(cam, seed, smp, bounce)
                nb = ctx[fb].shadow_visibility(cam, seed, smp, bounce)
                print(f"  bounce {bounce}: ray {raya[p].tolist()} / {rayb[p].tolist()}\n"
                      f"    {fa}: top {ta[p]} prim {pa[p]} t {tta[p]!r} nee {na[p]}\n"
                      f"    {fb}: top {tb[p]} prim {pb[p]} t {ttb[p]!r} nee {nb[p]}", flush=True)
    for c in ctx.values():
        c.close()


if __name__ == "__main__":
    main()
