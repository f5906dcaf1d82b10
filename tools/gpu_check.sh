#!/bin/bash
# GPU suite then the config-3 headline alone (GPU box, repo root)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 200 python3 -u bench.py --workload selfplay --no-cpu-baseline > gpurun_out/sp_bench.log 2> gpurun_out/sp_bench.err
