#!/usr/bin/env python3
"""Which part of a small render's extra cost is fixed per launch and which
grows with the shard's shape: per-launch times of CornellBoxLucy renders of
the same work cut different ways (run under `rocprofv3 --kernel-trace`,
RTGPU_STREAMS=1 for per-kernel attribution):

  full   the frame, 500 spp
  rr8    1/8 of the 32x32 buckets dealt round-robin (bench.py's shard)
  blk8   1/8 of the buckets as one contiguous band of rows
  spp8   every pixel at 500/8 spp (the same sample count as a 1/8 shard)
  rr2 / rr4 / rr16 / rr32  the round-robin shards of other sizes

  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sa -o kt -- python3 tools/shard_anat.py
  python3 tools/shard_anat.py --analyze gpurun_out/sa
"""
import csv
import glob
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ORDER = ["warm", "full", "rr8", "blk8", "spp8", "rr2", "rr4", "rr16", "rr32"]


def render():
    import __graft_entry__ as ge
    g = ge.load_package()
    s = g.Scene("cornell-lucy", width=1200, aspect=16.0 / 9.0, spp=500)
    cam = s.camera
    ctx = g.Context(0)
    ctx.upload(s.desc)
    ctx.set_schedule(0, 0, 0, int(os.environ.get("RTGPU_STREAMS", "1")))
    bk = g.generate_buckets(cam.image_width, cam.image_height, 32)
    rows = sorted(bk, key=lambda b: (b[1], b[0]))
    depth = cam.max_depth
    cases = {
        "warm": g.make_params(500, depth, seed=1),
        "full": g.make_params(500, depth, seed=1),
        "rr8": g.make_params(500, depth, seed=1, buckets=g.shard_buckets(bk, 0, 8)),
        "blk8": g.make_params(500, depth, seed=1, buckets=rows[3 * len(rows) // 8:4 * len(rows) // 8]),
        "spp8": g.make_params(500 // 8, depth, seed=1),
        "rr2": g.make_params(500, depth, seed=1, buckets=g.shard_buckets(bk, 0, 2)),
        "rr4": g.make_params(500, depth, seed=1, buckets=g.shard_buckets(bk, 0, 4)),
        "rr16": g.make_params(500, depth, seed=1, buckets=g.shard_buckets(bk, 0, 16)),
        "rr32": g.make_params(500, depth, seed=1, buckets=g.shard_buckets(bk, 0, 32)),
    }
    for name in ORDER:
        t = time.perf_counter()
        ctx.render(cam, cases[name])
        print(f"{name}: {(time.perf_counter() - t) * 1e3:.2f} ms", flush=True)
        time.sleep(0.05)   # a gap that separates the renders in the trace
    ctx.close()


def analyze(root):
    rows = []
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "").split("(")[0].split("<")[0].replace("void ", "").replace("rtg::", "")
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    rows.sort()
    groups, cur = [], []
    for r in rows:
        if cur and r[0] - cur[-1][1] > 20_000_000:
            groups.append(cur)
            cur = []
        cur.append(r)
    groups.append(cur)
    renders = [grp for grp in groups if any(k == "k_extend" for _, _, k in grp)]
    base = None
    for name, grp in zip(ORDER, renders):
        span = (grp[-1][1] - grp[0][0]) / 1e6
        per = {}
        for s, e, k in grp:
            if k.startswith("k_"):
                per.setdefault(k, []).append((e - s) / 1e6)
        if name == "full":
            base = per
        line = f"{name:5s} span {span:8.2f} ms |"
        for k in ("k_extend", "k_shade", "k_shadow", "k_nee_apply"):
            line += f" {k[2:]} " + " ".join(f"{v:6.2f}" for v in per.get(k, []))
        print(line)
        if base is not None and name not in ("warm", "full"):
            frac = {"rr8": 8, "blk8": 8, "spp8": 8, "rr2": 2, "rr4": 4, "rr16": 16, "rr32": 32}[name]
            ex = " ".join(f"{a - b / frac:+.2f}" for a, b in zip(per.get("k_extend", []), base["k_extend"]))
            sh = " ".join(f"{a - b / frac:+.2f}" for a, b in zip(per.get("k_shadow", []), base["k_shadow"]))
            print(f"      vs full/{frac}: extend {ex} | shadow {sh}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyze":
        analyze(sys.argv[2])
    else:
        render()
