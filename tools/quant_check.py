"""Quantised-node A/B on the GPU (node_quant.h).

Renders one BASELINE scene twice on the GPU — traversing the quantised
DNodeQ boxes (RT_NODES_QUANT8) and the fp32 DNode4 boxes (RT_NODES_FP32, the
default) — and lists the pixels whose sums differ; each format also renders
the frame again to show whether it depends on the wave schedule.  Boxes only cull, so a difference
can only come from a box test that rejected a ray whose primitive hit lies at
the box's edge.  Each differing pixel is then rendered alone by the fp64
oracle (the reference's arithmetic, no fp32 box rounding) and by the fp32
oracle, and the script reports which GPU image each one is closer to.

    python tools/quant_check.py [--scene cornell-lucy] [--width 1200] [--spp 500]
Writes a JSON summary to stdout.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cornell-lucy")
    ap.add_argument("--width", type=int, default=1200)
    ap.add_argument("--aspect", type=float, default=16.0 / 9.0)
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--max-pixels", type=int, default=40)
    ap.add_argument("--repeats", type=int, default=2)
    args = ap.parse_args()
    import __graft_entry__ as ge
    g = ge.load_package()
    from oracle import oracle_py as O

    scene = g.Scene(args.scene, width=args.width, aspect=args.aspect, spp=args.spp)
    cam = scene.camera
    W, H = cam.image_width, cam.image_height
    spp, depth = cam.samples_per_pixel, cam.max_depth
    params = g.make_params(spp, depth, seed=args.seed)
    imgs, sums, work = {}, {}, {}
    for mode in ("quantised", "exact"):
        ctx = g.Context(0)
        ctx.set_tlas_builder("sah")
        ctx.set_blas_builder("sah")
        ctx.set_node_format("quant8" if mode == "quantised" else "fp32")
        ctx.upload(scene.desc)
        acc, _ = ctx.render(cam, params)
        imgs[mode] = np.asarray(acc, np.float64).reshape(H, W, 3)
        # repeat renders: the frame must not depend on the wave schedule
        sums[mode] = [float(imgs[mode].sum())] + [float(np.asarray(ctx.render(cam, params)[0], np.float64).sum())
                                                  for _ in range(args.repeats)]
        work[mode] = ctx.count_work(cam, params)
        ctx.close()
    q, e = imgs["quantised"], imgs["exact"]
    diff = np.any(q != e, axis=2)
    ys, xs = np.nonzero(diff)
    out = {"scene": args.scene, "width": W, "height": H, "spp": spp, "depth": depth,
           "frame_sum_quantised": float(q.sum()), "frame_sum_exact": float(e.sum()),
           "differing_pixels": int(diff.sum()), "repeat_sums": sums,
           "work": {m: {k: int(v) for k, v in w.items()} for m, w in work.items()}, "pixels": []}
    closer = {"quantised": 0, "exact": 0, "tie": 0}
    for y, x in list(zip(ys.tolist(), xs.tolist()))[: args.max_pixels]:
        bp = g.make_params(spp, depth, seed=args.seed, buckets=[(x, y, 1, 1)])
        r64 = O.render(scene.desc, cam, bp, fp32=False)[y, x]
        r32 = O.render(scene.desc, cam, bp, fp32=True)[y, x]
        dq = float(np.abs(q[y, x] - r64).sum() / spp)
        de = float(np.abs(e[y, x] - r64).sum() / spp)
        who = "quantised" if dq < de else "exact" if de < dq else "tie"
        closer[who] += 1
        out["pixels"].append({"x": x, "y": y, "quantised": (q[y, x] / spp).round(6).tolist(),
                              "exact": (e[y, x] / spp).round(6).tolist(),
                              "oracle_fp64": (r64 / spp).round(6).tolist(),
                              "oracle_fp32": (r32 / spp).round(6).tolist(),
                              "err_quantised": round(dq, 7), "err_exact": round(de, 7), "closer": who})
    out["closer_to_fp64"] = closer
    print(json.dumps(out))


if __name__ == "__main__":
    main()
