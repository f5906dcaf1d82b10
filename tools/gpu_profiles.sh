#!/bin/bash
# Round evidence (run on the GPU box from the repo root), everything under gpurun_out/:
#   the steady-state self-play kernel statistics (CSV) and PMC summary.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROUND=${1:-r03}
mkdir -p gpurun_out
# (k_rollout is unchanged since round 2: its PMC summaries in profiles/r02_rollout_pmc_c*.json stand;
#  tools/pmc_rollout.sh gpurun_out/pmc100 "$ROUND" 100 regenerates them)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sp -o sp -- \
    python3 bench.py --workload selfplay --steps 2000 --window 4000 --no-cpu-baseline > gpurun_out/prof_sp.log 2>&1
timeout -k 10 900 bash tools/pmc_selfplay.sh gpurun_out/pmc_sp "$ROUND" > gpurun_out/pmc_sp.log 2>&1
timeout -k 10 200 python3 -u bench.py --workload selfplay --no-cpu-baseline > gpurun_out/sp_bench.log 2> gpurun_out/sp_bench.err
