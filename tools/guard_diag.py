#!/usr/bin/env python3
"""Diagnostic: CornellBoxScene renders of the library in
RTGPU_LIB_DIR at several path depths, saved as .npy for a host-side diff
against the production build and the CPU oracle (tools/guard_diff.py).

  RTGPU_LIB_DIR=lib_guard python3 tools/guard_diag.py gpurun_out/guard/guard
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import __graft_entry__ as ge
    g = ge.load_package()
    prefix = sys.argv[1]
    os.makedirs(os.path.dirname(prefix), exist_ok=True)
    scene = os.environ.get("DIAG_SCENE", "cornell")
    s = g.Scene(scene, width=64)
    cam = s.camera
    ctx = g.Context(0)
    ctx.upload(s.desc)
    for d in (1, 2, 3, 5):
        for rep in range(2):
            acc, _ = ctx.render(cam, g.make_params(64, d, seed=5))
            np.save(f"{prefix}_d{d}_r{rep}.npy", acc)
            print(f"{prefix} depth {d} rep {rep}: mean {acc.mean() / 64:.6f}", flush=True)
    top, prim, t = ctx.primary_hits(cam, 5, 0)
    np.save(f"{prefix}_hits.npy", np.stack([top, prim, t.view(np.int32)]))
    ctx.close()


if __name__ == "__main__":
    main()
