"""Aggregate rocprofv3 --pmc CSVs per kernel (sum over dispatches)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
agg = defaultdict(lambda: defaultdict(float))
calls = defaultdict(set)
for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "?")
        k = k.split("(")[0].replace("void ", "")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[k].add((f, r.get("Dispatch_Id")))
for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    print(f"== {k}  dispatches~{len(calls[k]) // max(1, len({c[0] for c in calls[k]}))}")
    for c in sorted(v):
        print(f"   {c:32s} {v[c]:.6g}")
    wc = v.get("SQ_WAVE_CYCLES", 0)
    if wc:
        print(f"   -> wait_any {v.get('SQ_WAIT_ANY',0)/wc:.3f} wait_inst {v.get('SQ_WAIT_INST_ANY',0)/wc:.3f} "
              f"active {v.get('SQ_ACTIVE_INST_ANY',0)/wc:.3f}")
    if v.get("SQ_ACTIVE_INST_VALU"):
        print(f"   -> VALU lane util {v.get('SQ_THREAD_CYCLES_VALU',0)/(64*v['SQ_ACTIVE_INST_VALU']):.3f}")
    h, m = v.get("TCC_HIT_sum", 0), v.get("TCC_MISS_sum", 0)
    if h + m:
        print(f"   -> L2 hit {h/(h+m):.3f}")
    if v.get("TCP_TCC_READ_REQ_sum"):
        print(f"   -> avg L2 read latency {v.get('TCP_TCC_READ_REQ_LATENCY_sum',0)/v['TCP_TCC_READ_REQ_sum']:.1f} cyc")
