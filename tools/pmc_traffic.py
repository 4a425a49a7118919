"""rocprofv3 outputs of tools/profile_round.sh -> per-kernel stats + HBM traffic.

Writes profiles/pmc_<scene>_<W>x<H>.json:
  kernels.<extend|shade|shadow>.{fetch_bytes_per_launch, write_bytes_per_launch,
  hbm_bytes_per_launch, dispatches}
FETCH_SIZE / WRITE_SIZE are in KiB (rocprofv3 derived counters).  Per
MI355X_MICROARCH.md (HBM section) FETCH_SIZE counts 64 B per 128-B request
on gfx950 for wide streaming reads, so it is doubled; the same factor holds
for the traversal's scattered 16-B rows and node steps (one whole-line
request per missed line: tools/fetch_calib.sh, profiles/r06_fetch_calib.json,
bench.py FETCH_FACTOR).
Also copies the kernel-trace stats CSV to profiles/<tag>_kernel_stats.csv.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
tag = sys.argv[2] if len(sys.argv) > 2 else "r01"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def family(name):
    for k in ("k_extend", "k_shade", "k_shadow", "k_nee_apply", "k_accum", "k_finalize"):
        if f"rtg::{k}<" in name or f"rtg::{k}(" in name:
            return k[2:]
    return None


vals = defaultdict(lambda: defaultdict(float))
disp = defaultdict(lambda: defaultdict(set))
for counter in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(os.path.join(root, counter, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            fam = family(r.get("Kernel_Name", ""))
            if fam is None or r["Counter_Name"] != counter:
                continue
            vals[fam][counter] += float(r["Counter_Value"])
            disp[fam][counter].add(r.get("Dispatch_Id"))
bench = {}
try:
    bench = json.load(open(os.path.join(root, "kt_bench.json")))
except Exception:
    pass
cfg = bench.get("config", {})
out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), bench.py --steps 1 --warmup 0 (default workload: the timed steps' per-launch batches)",
       "scene": cfg.get("scene", "cornell-lucy"), "width": cfg.get("width"), "height": cfg.get("height"),
       # the frame this code renders: bench.py marks the traffic stale when it changes
       "frame_sum": cfg.get("frame_sum"),
       "kernels": {}}
for fam, v in vals.items():
    n = max(len(disp[fam]["FETCH_SIZE"]), 1)
    nw = max(len(disp[fam]["WRITE_SIZE"]), 1)
    fetch = v["FETCH_SIZE"] * 1024 * 2 / n
    write = v["WRITE_SIZE"] * 1024 / nw
    out["kernels"][fam] = {"dispatches": n, "fetch_bytes_per_launch": int(fetch),
                           "write_bytes_per_launch": int(write), "hbm_bytes_per_launch": int(fetch + write)}
name = f"pmc_{out['scene']}_{out['width']}x{out['height']}.json"
os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "profiles", name), "w"), indent=1)
print(json.dumps(out, indent=1))
for f in glob.glob(os.path.join(root, "kt", "**", "*kernel_stats.csv"), recursive=True):
    shutil.copy(f, os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
    print("copied", f)
