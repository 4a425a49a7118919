"""Diagnostic: the multi-device test's sequence (one-device and [0,0,0]
contexts created, uploaded, rendered) repeated N times in one process for
the library in RTGPU_LIB_DIR; prints how many repetitions gave a multi-device
frame different from the one-device frame, and where."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

g = ge.load_package()
s = g.Scene("cornell-lucy", width=96, aspect=16.0 / 9.0, lucy_rings=60, lucy_cols=80)
cam = s.camera
p = g.make_params(6, cam.max_depth, seed=13)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
bad = 0
for r in range(reps):
    for devs in ([0, 0], [0, 0, 0]):
        one = g.Context(0)
        multi = g.Context(devices=devs)
        one.upload(s.desc)
        multi.upload(s.desc)
        a, _ = one.render(cam, p)
        b, _ = multi.render(cam, p)
        d = (a != b).any(axis=2)
        if d.any():
            bad += 1
            ys, xs = np.nonzero(d)
            zero_b = int((b[d] == 0).all(axis=-1).sum())
            print(f"rep {r} {devs}: {int(d.sum())} pixels differ (of {d.size}), {zero_b} of them zero in multi, "
                  f"max |diff| {float(np.abs(a - b).max()):.4g}, rows {ys.min()}-{ys.max()} cols {xs.min()}-{xs.max()}",
                  flush=True)
        multi.close()
        one.close()
print(f"{bad} mismatching renders of {2 * reps}")
