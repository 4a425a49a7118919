#!/bin/bash
# WRITE_SIZE / FETCH_SIZE per kernel of the bench workload (one step, one
# stream) for each library variant: tools/pmc_ab.sh lib_a lib_b ...
# [SCENE_ARGS=...]; prints bytes per launch per kernel family.
set -o pipefail
export TMPDIR=/tmp
for lib in "$@"; do
  for c in WRITE_SIZE FETCH_SIZE; do
    RTGPU_LIB_DIR=$lib RTGPU_STREAMS=1 timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmcab_${lib}_$c -o p -- \
      python3 bench.py --pmc-child $SCENE_ARGS > /dev/null 2> gpurun_out/pmcab_${lib}_$c.err || exit 1
  done
  python3 - "$lib" <<'PY'
import csv, glob, sys
from collections import defaultdict
lib = sys.argv[1]
for c in ("WRITE_SIZE", "FETCH_SIZE"):
    v = defaultdict(float); d = defaultdict(set)
    for f in glob.glob(f"gpurun_out/pmcab_{lib}_{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            for k in ("k_extend", "k_shadow", "k_shade", "k_nee_apply"):
                if f"rtg::{k}<" in n or f"rtg::{k}(" in n:
                    v[k] += float(r["Counter_Value"]); d[k].add(r["Dispatch_Id"])
    print(lib, c, {k: round(v[k] * 1024 / max(len(d[k]), 1) / 1e9, 3) for k in sorted(v)}, "GB per launch", flush=True)
PY
done
