#!/usr/bin/env python3
"""Rare-event scan of the integer hit parity (diagnostic).

For whole frames at full resolution, compares every path ray of every
bounce that the production k_extend traced (rt_extend_hits) with the fp32
oracle's recursion (oracle_path_records) — the per-bounce probe of
tests/test_gpu_paths.py at the bench's size and over several samples, to
measure how often the two disagree.  Reports per sample and bounce the rays
compared, diverged and mismatched, and the first mismatches (ray, both hits).

usage: tools/oracle_ray_scan.py [scene] [width] [first_sample] [samples] [nodes] [threads] [blas]
(blas: "sah" (default) or "reference": the caller's own BVH topology, which
the oracle walks)
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import __graft_entry__ as ge
    g = ge.load_package()
    from oracle import oracle_py as O
    scene = sys.argv[1] if len(sys.argv) > 1 else "cornell-lucy"
    width = int(sys.argv[2]) if len(sys.argv) > 2 else 1200
    s0 = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    ns = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    nodes = sys.argv[5] if len(sys.argv) > 5 else "fp32"
    threads = int(sys.argv[6]) if len(sys.argv) > 6 else 16
    blas = sys.argv[7] if len(sys.argv) > 7 else "sah"
    seed = 1
    s = g.Scene(scene, width=width, aspect=16.0 / 9.0)
    cam = s.camera
    nb = cam.max_depth
    c = g.Context(0)
    c.set_node_format(nodes)
    c.set_blas_builder(blas)
    c.set_tlas_builder("sah" if blas == "sah" else "reference")
    c.upload(s.desc)
    tot = dict(compared=0, diverged=0, mismatched=0)
    bits = lambda a: np.ascontiguousarray(a, np.float32).view(np.uint32)
    for smp in range(s0, s0 + ns):
        t0 = time.time()
        ot, op, ott, oray, _ = O.path_records(s.desc, cam, seed, smp, nb, fp32=True, threads=threads)
        for b in range(nb):
            gt, gp, gtt, gray = c.extend_hits(cam, seed, smp, b)
            ag, ao = gt != -2, ot[b] != -2
            same = ag & ao & np.all(bits(gray) == bits(oray[b]), axis=1)
            div = (ag | ao) & ~same
            bad = np.flatnonzero(same & ((gt != ot[b]) | (gp != op[b]) | (bits(gtt) != bits(ott[b]))))
            tot["compared"] += int(same.sum())
            tot["diverged"] += int(div.sum())
            tot["mismatched"] += len(bad)
            print(f"sample {smp} bounce {b}: compared {int(same.sum())} diverged {int(div.sum())} mismatched {len(bad)}",
                  flush=True)
            for p in bad[:3]:
                print(f"  pixel {p} ray {gray[p].tolist()}: gpu top {gt[p]} prim {gp[p]} t {gtt[p]!r} | oracle top "
                      f"{ot[b][p]} prim {op[b][p]} t {np.float32(ott[b][p])!r}", flush=True)
        print(f"sample {smp}: {time.time() - t0:.1f} s", flush=True)
    c.close()
    print(f"{scene} {cam.image_width}x{cam.image_height} nodes {nodes} blas {blas}, samples {s0}..{s0 + ns - 1}, bounces 0..{nb - 1}: "
          f"{tot}", flush=True)


if __name__ == "__main__":
    main()
