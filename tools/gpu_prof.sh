#!/bin/bash
# Development profile: kernel trace of the config-3 bench (steady-state window).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/qprof -o sp -- python3 bench.py --workload selfplay --steps 2000 --window 0 --no-cpu-baseline > gpurun_out/qprof.log 2>&1
