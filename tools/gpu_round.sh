#!/bin/bash
# GPU check used during development: full -m gpu suite, default bench, and a kernel-trace
# profile of the config-3 self-play workload (outputs under gpurun_out/).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sp -o sp -- \
    python bench.py --workload selfplay --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/prof_sp.log 2>&1
