#!/bin/bash
# One bench line per BASELINE.json GPU config at N=1 (gpurun_out/cfg_<scene>.json):
#   C2 RandomScene 1200x675 500 spp (depth 50), C3 CornellBoxScene 600x600
#   1000 spp, C4 CornellBoxLucy 1200x675 500 spp, C5 HDRITestScene 1920x1080
#   2000 spp.  CPU baseline only on the default (C4) bench run.
set -o pipefail
mkdir -p gpurun_out
run() {
  name=$1; shift
  timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/cfg_$name.json 2> gpurun_out/cfg_$name.err || { tail -20 gpurun_out/cfg_$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/cfg_$name.json'));print('$name',d['value'],d['unit'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['frac'])"
}
run random --scene random --width 1200 --spp 500
run cornell --scene cornell --width 600 --aspect 1 --spp 1000
run hdri --scene hdri-test --width 1920 --spp 2000
