#!/bin/bash
# Round evidence (run on the GPU box from the repo root): rollout PMC summary, default
# bench line, and the config-3 self-play kernel statistics (CSV) under gpurun_out/.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROUND=${1:-r01}
mkdir -p gpurun_out
bash tools/pmc_rollout.sh gpurun_out/pmc "$ROUND" > gpurun_out/pmc.log 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sp -o sp -- \
    python3 bench.py --workload selfplay --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/prof_sp.log 2>&1
