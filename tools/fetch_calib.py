#!/usr/bin/env python3
"""Turn tools/fetch_calib.sh's counter passes into the FETCH_SIZE calibration
(profiles/r06_fetch_calib.txt / .json).

For each microkernel pattern (tools/fetch_calib/fetch_calib.hip: every 128-B
line of a table missed exactly once per launch): FETCH_SIZE bytes, L2 read
requests to the fabric (TCC_EA0_RDREQ, of which 32-B ones and 128-B
"bubble" ones), L2 misses, per missed line.  The stream / line8 patterns read
whole lines (known: 128 B per line), so bytes / FETCH_SIZE there is the
factor of a whole-line fill; a pattern whose requests per missed line and
request sizes match it moves the same bytes per line.  Then the production
kernels' requests per L2 miss on the bench workload, for the same inference.

usage: tools/fetch_calib.py gpurun_out/calib
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    """{dispatch_id: {counter: value}, names by dispatch id}"""
    vals = defaultdict(dict)
    names = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            did = int(row["Dispatch_Id"])
            vals[did][row["Counter_Name"]] = vals[did].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
            names[did] = row.get("Kernel_Name", "")
    return vals, names


def micro(out):
    res = defaultdict(lambda: defaultdict(list))
    lines = json.load(open(os.path.join(out, "order.json")))["lines"]
    for p in ("fetch", "req", "bubble", "write"):
        d = os.path.join(out, p)
        if not os.path.isdir(d):
            continue
        vals, names = load(d)
        for did in sorted(vals):
            n = names[did]
            for pat in ("stream", "line8", "row16", "node7"):
                if f"k_{pat}(" in n or n.startswith(f"k_{pat}"):
                    for c, v in vals[did].items():
                        res[pat][c].append(v)
    rows = {}
    for pat, cs in res.items():
        r = {}
        for c, v in cs.items():
            v = sorted(v)[len(v) // 2]   # median over the repetitions
            r[c] = v
        per = {}
        if "FETCH_SIZE" in r:
            per["fetch_size_bytes_per_line"] = round(r["FETCH_SIZE"] * 1024 / lines, 2)
        for c, k in (("TCC_EA0_RDREQ_sum", "rdreq_per_line"), ("TCC_EA0_RDREQ_32B_sum", "rdreq32_per_line"),
                     ("TCC_BUBBLE_sum", "rdreq128_per_line"), ("TCC_MISS_sum", "l2_miss_per_line"),
                     ("TCC_HIT_sum", "l2_hit_per_line")):
            if c in r:
                per[k] = round(r[c] / lines, 3)
        rows[pat] = per
    return lines, rows


def production(out):
    fam = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(lambda: defaultdict(int))
    for p in ("bench_req", "bench_bubble", "bench_fetch"):
        d = os.path.join(out, p)
        if not os.path.isdir(d):
            continue
        vals, names = load(d)
        for did, cs in vals.items():
            n = names[did]
            for k in ("k_extend", "k_shadow", "k_shade", "k_nee_apply"):
                if f"rtg::{k}<" in n or f"{k}<" in n or f"rtg::{k}(" in n:
                    for c, v in cs.items():
                        fam[k][c] += v
                        cnt[k][c] += 1
    rows = {}
    for k, cs in fam.items():
        r = {c: v / max(cnt[k][c], 1) for c, v in cs.items()}   # per dispatch
        e = {"dispatches": max(cnt[k].values())}
        m = r.get("TCC_MISS_sum")
        if "TCC_EA0_RDREQ_sum" in r and m:
            e["rdreq_per_l2_miss"] = round(r["TCC_EA0_RDREQ_sum"] / m, 3)
        if "TCC_EA0_RDREQ_32B_sum" in r and r.get("TCC_EA0_RDREQ_sum"):
            e["rdreq32_share"] = round(r["TCC_EA0_RDREQ_32B_sum"] / r["TCC_EA0_RDREQ_sum"], 4)
        if "TCC_BUBBLE_sum" in r and r.get("TCC_EA0_RDREQ_sum"):
            e["rdreq128_share"] = round(r["TCC_BUBBLE_sum"] / r["TCC_EA0_RDREQ_sum"], 4)
        if "FETCH_SIZE" in r and r.get("TCC_EA0_RDREQ_sum"):
            e["fetch_size_bytes_per_rdreq"] = round(r["FETCH_SIZE"] * 1024 / r["TCC_EA0_RDREQ_sum"], 2)
        if m and "FETCH_SIZE" in r:
            e["fetch_size_bytes_per_l2_miss"] = round(r["FETCH_SIZE"] * 1024 / m, 2)
        e.update({c: r[c] for c in sorted(r)})
        rows[k] = e
    return rows


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/calib"
    lines, m = micro(out)
    p = production(out)
    res = {"lines_per_launch": lines, "line_bytes": 128, "patterns": m, "production": p}
    # factor: bytes of a whole-line fill per FETCH_SIZE byte (stream and line8 read 128 B per line)
    whole = [m[k]["fetch_size_bytes_per_line"] for k in ("stream", "line8") if "fetch_size_bytes_per_line" in m.get(k, {})]
    if whole:
        res["whole_line_factor"] = round(128.0 / (sum(whole) / len(whole)), 3)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
