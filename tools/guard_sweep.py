#!/usr/bin/env python3
"""RTG_GUARD diagnostic sweep: renders with the
guard build (every device index checked, canaries after every scratch
buffer) over the twin counts and scenes whose stores the guard covers, each
on a fresh context whose batch buffers are sized exactly for the render.
The library prints any bad index or damaged canary to stderr after each
render; this script prints one line per render and the frame checksum.

  make -C go-raytracing_amd/csrc EXTRA="-DRTG_GUARD -DRTG_DIAG_RING=8" OUT=../lib_guard
  RTGPU_LIB_DIR=lib_guard python3 tools/guard_sweep.py
  RTGPU_LIB_DIR=lib_guard RTGPU_GUARD_OLD_WQ=1 python3 tools/guard_sweep.py   # round-3 queue sizing
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CASES = [("cornell", dict(width=96), 8), ("cornell-smoke", dict(width=64), 8),
         ("cornell-lucy", dict(width=96, lucy_rings=60, lucy_cols=80), 8), ("hdri-nee", dict(width=96), 8),
         ("random", dict(width=96), 4)]


def full_nee_scene(g):
    """Every camera ray of tests/kat_cases.py's area-light scene (64 x 1)
    hits a Lambertian floor under the lights: every path writes a NEE job,
    so the job words of every twin run to the end of its slots."""
    from tests import kat_cases as K
    b, d, cam = K.area_light_scene(g)
    return b, d, cam


def main():
    import __graft_entry__ as ge
    g = ge.load_package()
    cases = list(CASES) + [("full-nee", None, 4)]
    for name, kw, spp in cases:
        if kw is None:
            keep, desc, cam = full_nee_scene(g)
            s = type("S", (), {"desc": desc, "camera": cam})()
        else:
            s = g.Scene(name, **kw)
        cam = s.camera
        npix = cam.image_width * cam.image_height
        for streams in (1, 2, 3, 4):
            c = g.Context(0)
            try:
                c.upload(s.desc)
                c.set_schedule(npix * spp, 0, 0, streams)
                acc, _ = c.render(cam, g.make_params(spp, cam.max_depth, seed=5))
                sys.stderr.flush()
                print(f"{name} {cam.image_width}x{cam.image_height} {spp}spp streams {streams}: "
                      f"sum {float(acc.astype(np.float64).sum()):.9g}", flush=True)
            finally:
                c.close()


if __name__ == "__main__":
    main()
