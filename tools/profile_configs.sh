#!/bin/bash
# kernel traces of the C2 / C3 / C5 bench workloads on one stream
set -o pipefail
export TMPDIR=/tmp
for c in "c2:--scene random --width 1200 --spp 500" "c3:--scene cornell --width 600 --aspect 1 --spp 1000" "c5:--scene hdri-test --width 1920 --spp 2000"; do
  name=${c%%:*}; args=${c#*:}
  RTGPU_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_$name -o kt -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-configs --no-balance --no-pmc --no-three-pass $args > gpurun_out/kt_$name.json 2> gpurun_out/kt_$name.err || exit 1
  echo "$name done"
done
