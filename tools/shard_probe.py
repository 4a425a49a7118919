#!/usr/bin/env python3
"""Per-launch anatomy of a full CornellBoxLucy frame vs one 1/8 round-robin
shard of it (run under `rocprofv3 --kernel-trace`): which kernels carry the
per-render overhead that makes 8 shards cost more than one frame.

  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sp -o kt -- python3 tools/shard_probe.py
  python3 tools/shard_probe.py --analyze gpurun_out/sp
"""
import csv
import glob
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def render():
    import __graft_entry__ as ge
    g = ge.load_package()
    streams = int(os.environ.get("RTGPU_STREAMS", "1"))
    s = g.Scene("cornell-lucy", width=1200, aspect=16.0 / 9.0, spp=500)
    cam = s.camera
    ctx = g.Context(0)
    ctx.upload(s.desc)
    ctx.set_schedule(0, 0, 0, streams)
    bk = g.generate_buckets(cam.image_width, cam.image_height, 32)
    full = g.make_params(500, cam.max_depth, seed=1)
    shard = g.make_params(500, cam.max_depth, seed=1, buckets=g.shard_buckets(bk, 0, 8))
    for name, p in (("warm", full), ("full", full), ("shard", shard), ("shard", shard)):
        t = time.perf_counter()
        ctx.render(cam, p)
        print(f"{name}: {(time.perf_counter() - t) * 1e3:.2f} ms", flush=True)
        time.sleep(0.05)   # a gap that separates the renders in the trace
    ctx.close()


def analyze(root):
    rows = []
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            k = name.split("(")[0].split("<")[0].replace("void ", "").replace("rtg::", "")
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    rows.sort()
    # renders = groups separated by > 20 ms gaps
    groups, cur = [], []
    for r in rows:
        if cur and r[0] - cur[-1][1] > 20_000_000:
            groups.append(cur)
            cur = []
        cur.append(r)
    groups.append(cur)
    for gi, grp in enumerate(groups):
        span = (grp[-1][1] - grp[0][0]) / 1e6
        busy = sum((e - s) for s, e, _ in grp) / 1e6
        print(f"render {gi}: {len(grp)} launches, span {span:.2f} ms, sum of durations {busy:.2f} ms")
        per = {}
        for s, e, k in grp:
            c = per.setdefault(k, [0, 0.0])
            c[0] += 1
            c[1] += (e - s) / 1e6
        print("   " + ", ".join(f"{k} {n}x {ms:.2f}" for k, (n, ms) in sorted(per.items(), key=lambda kv: -kv[1][1])))
        if os.environ.get("SP_LAUNCHES"):
            for s, e, k in grp:
                if k.startswith("k_"):
                    print(f"   {k:14s} {(e - s) / 1e6:8.3f} ms  at {(s - grp[0][0]) / 1e6:8.3f}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyze":
        analyze(sys.argv[2])
    else:
        render()
