#!/bin/bash
# One gpurun call as a sequence of steps (the parameterised form of the
# one-off round-5 recipes).  Each argument is one step, its first word the
# step's name:
#   tests [pytest args]        pytest -m gpu (plain test failures do not stop the call)
#   smoke                      __graft_entry__.smoke()
#   bench [bench args]         the default bench line -> gpurun_out/bench.json
#   bal <spec> ...             tools/bal_ab.sh (value + 2/4/8-way shard predictions)
#   ab <spec> ...              tools/ab.sh (value, per-kernel ms, work per sample; BENCH_ARGS from the env)
#   abc3 <spec> ...            tools/ab.sh on C3 (CornellBoxScene 600x600, 1000 spp)
#   abc2 / abc5 <spec> ...     the same on C2 (RandomScene) / C5 (HDRITestScene)
#   refresh                    tools/round_refresh.sh (tests, fp64 log, bench, profiles, configs)
# A spec is "label:ENV=v,ENV2=w:libdir" (tools/ab.sh).  Every GPU step runs
# under its own time limit; a timeout, crash or abort ends the call.
#   e.g. bash tools/gpu_steps.sh tests "bal r5::lib_r5 new::lib" "abc3 new::lib"
set -o pipefail
mkdir -p gpurun_out
fatal() {   # exit codes that mean a fault, a hang or a kill: start nothing more
  case $1 in 124|134|137|139|143) return 0 ;; *) return 1 ;; esac
}
C2="--scene random --width 1200 --spp 500"
C3="--scene cornell --width 600 --aspect 1 --spp 1000"
C5="--scene hdri-test --width 1920 --spp 2000"
QUICK="--no-pmc --no-count --no-three-pass"
for step in "$@"; do
  read -ra w <<< "$step"
  name=${w[0]}; args=("${w[@]:1}")
  echo "=== $step" >&2
  case $name in
    tests)
      timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "${args[@]}" \
        > gpurun_out/gpu_tests.log 2>&1; rc=$?
      tail -3 gpurun_out/gpu_tests.log
      if fatal $rc; then exit $rc; fi ;;
    smoke)
      timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
      tail -2 gpurun_out/smoke.log
      [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 400 python3 bench.py "${args[@]}" > gpurun_out/bench.json 2> gpurun_out/bench.err || { rc=$?; tail -20 gpurun_out/bench.err; exit $rc; }
      cat gpurun_out/bench.json ;;
    bal) bash tools/bal_ab.sh "${args[@]}" || exit $? ;;
    ab) bash tools/ab.sh "${args[@]}" || exit $? ;;
    abc2) BENCH_ARGS="$C2 $QUICK" bash tools/ab.sh "${args[@]}" || exit $? ;;
    abc3) BENCH_ARGS="$C3 $QUICK" bash tools/ab.sh "${args[@]}" || exit $? ;;
    abc5) BENCH_ARGS="$C5 $QUICK" bash tools/ab.sh "${args[@]}" || exit $? ;;
    refresh) bash tools/round_refresh.sh || exit $? ;;
    *) echo "unknown step $name" >&2; exit 2 ;;
  esac
done
echo steps-done
