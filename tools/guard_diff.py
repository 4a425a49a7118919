#!/usr/bin/env python3
"""Host-side analysis of tools/guard_diag.py's renders: per depth, each
library's image-mean relative bias against the CPU oracle (fp32 mirror and
fp64 restatement) on the same scene / seed / spp, run-to-run equality, and
the pixels where two libraries differ.

  python3 tools/guard_diff.py gpurun_out/guard lib_guard lib_head lib
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import __graft_entry__ as ge
    from oracle import oracle_py as O
    g = ge.load_package()
    d0 = sys.argv[1]
    libs = sys.argv[2:]
    scene = os.environ.get("DIAG_SCENE", "cornell")
    s = g.Scene(scene, width=64)
    cam = s.camera
    spp = 64
    for d in (1, 2, 3, 5):
        p = g.make_params(spp, d, seed=5)
        r32 = O.render(s.desc, cam, p, fp32=True, threads=8) / spp
        r64 = O.render(s.desc, cam, p, fp32=False, threads=8) / spp
        line = [f"depth {d}: oracle fp32 mean {r32.mean():.6f} fp64 {r64.mean():.6f}"]
        imgs = {}
        for lib in libs:
            a = np.load(os.path.join(d0, f"{lib}_d{d}_r0.npy")).astype(np.float64) / spp
            b = np.load(os.path.join(d0, f"{lib}_d{d}_r1.npy")).astype(np.float64) / spp
            imgs[lib] = a
            same = np.array_equal(a, b)
            line.append(f"  {lib}: bias32 {(a.mean() - r32.mean()) / r32.mean():+.2e} "
                        f"bias64 {(a.mean() - r64.mean()) / r64.mean():+.2e} "
                        f"mse32 {np.mean((a - r32) ** 2):.2e} rerun-identical {same}")
        print("\n".join(line))
        if len(libs) >= 2:
            a, b = imgs[libs[0]], imgs[libs[1]]
            diff = np.abs(a - b).sum(axis=2)
            ys, xs = np.nonzero(diff > 0)
            print(f"  {libs[0]} vs {libs[1]}: {ys.size} pixels differ; first {list(zip(ys[:8], xs[:8]))}")
    for lib in libs:
        h = os.path.join(d0, f"{lib}_hits.npy")
        if os.path.exists(h):
            top, prim, t = np.load(h)
            to, po, tt = O.primary_hits(s.desc, cam, 5, 0, fp32=True)
            print(f"{lib}: primary-hit mismatches vs oracle {int(np.sum((top != to) | (prim != po)))}")


if __name__ == "__main__":
    main()
