#!/bin/bash
# Round-4 evidence on the GPU box (repo root), outputs under gpurun_out/:
#   STEP=bench    the default bench line (config-3 headline + configs 2/5/4 objects)
#   STEP=profile  config-3 kernel trace + statistics and the PMC passes (tools/pmc_selfplay.sh)
#   STEP=nn       full-batch k_nn_forward trace + HBM counters (tools/nn_fullbatch.sh)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
ROUND=${ROUND:-r04}
case "${STEP:-bench}" in
bench)
    timeout -k 10 900 python3 -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err ;;
profile)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sp -o sp -- \
        python3 bench.py --workload selfplay --steps 2000 --window 4000 --no-cpu-baseline > gpurun_out/prof_sp.log 2>&1 &&
    timeout -k 10 900 bash tools/pmc_selfplay.sh gpurun_out/pmc_sp "$ROUND" > gpurun_out/pmc_sp.log 2>&1 ;;
nn)
    timeout -k 10 400 bash tools/nn_fullbatch.sh "$ROUND" > gpurun_out/nnfb.log 2>&1 ;;
esac
