#!/usr/bin/env python3
"""Per-launch kernel time against render size (C4, one stream): renders the
first of n round-robin shards (n = 1, 2, 4, 8, 16) at the given depths and
prints each kernel's launch time times n, so a cost proportional to the rays
stays flat and a fixed per-launch cost grows with n.

  RTGPU_STREAMS=1 python3 tools/shard_scan.py [depth ...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import __graft_entry__ as ge
    g = ge.load_package()
    depths = [int(x) for x in sys.argv[1:]] or [1, 5]
    s = g.Scene("cornell-lucy", width=1200, aspect=16.0 / 9.0, spp=500)
    cam = s.camera
    ctx = g.Context(0)
    ctx.upload(s.desc)
    ctx.set_schedule(0, 0, 0, int(os.environ.get("RTGPU_STREAMS", "1")))
    ctx.set_kernel_timing(True)
    # SCAN_GRAIN: the dealt unit (16 = 16x16 tiles of the 32x32 buckets, the
    # bench's; 32 / 64 / 128 = whole buckets of that size)
    grain = int(os.environ.get("SCAN_GRAIN", "16"))
    bk = g.generate_buckets(cam.image_width, cam.image_height, 32 if grain == 16 else grain)
    tile = 16 if grain == 16 else 0
    for depth in depths:
        for n in (1, 2, 4, 8, 16):
            p = g.make_params(500, depth, seed=1, buckets=g.shard_buckets(bk, 0, n, tile))
            best = None
            for _ in range(2):
                ctx.render(cam, p)
                kt = ctx.last_kernel_times()
                total = ctx.last_render_kernel_ms()
                if best is None or total < best[0]:
                    best = (total, kt)
            total, kt = best
            print(f"grain {grain} depth {depth} shard 1/{n:<2d}: render {total:8.2f} ms (x n {total * n:8.2f}) | "
                  f"extend {kt['extend_ms'] * n:8.2f} shade {kt['shade_ms'] * n:8.2f} shadow {kt['shadow_ms'] * n:8.2f}"
                  f" (x n; {kt['extend_launches']} / {kt['shade_launches']} / {kt['shadow_launches']} launches)", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
