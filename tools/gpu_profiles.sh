#!/bin/bash
# Round evidence (run on the GPU box from the repo root), everything under gpurun_out/:
#   rollout PMC summaries at the driver's launch size (20 moves) and at 100 moves,
#   the default bench line, the steady-state self-play kernel statistics (CSV) and PMC.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROUND=${1:-r02}
mkdir -p gpurun_out
bash tools/pmc_rollout.sh gpurun_out/pmc20 "$ROUND" 20 > gpurun_out/pmc20.log 2>&1
bash tools/pmc_rollout.sh gpurun_out/pmc100 "$ROUND" 100 > gpurun_out/pmc100.log 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sp -o sp -- \
    python3 bench.py --workload selfplay --steps 2000 --warmup 3000 --no-cpu-baseline > gpurun_out/prof_sp.log 2>&1
timeout -k 10 900 bash tools/pmc_selfplay.sh gpurun_out/pmc_sp "$ROUND" > gpurun_out/pmc_sp.log 2>&1
