#!/bin/bash
# Round-5 refresh, part 2: PMC counter passes and one bench line per config.
set -o pipefail
mkdir -p gpurun_out
bash tools/pmc_profile.sh || exit 1
bash tools/configs_round.sh || exit 1
echo refresh2-done
