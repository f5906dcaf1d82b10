#!/bin/bash
# Development check: search parity subset, then a kernel trace of a short config-3 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_mcts_gpu.py tests/test_selfplay_gpu.py tests/test_noise_gpu.py -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/quick_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload selfplay --steps 2000 --window 2000 --no-cpu-baseline > gpurun_out/quick_bench.log 2> gpurun_out/quick_bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/qprof -o sp -- python3 bench.py --workload selfplay --steps 2000 --window 0 --no-cpu-baseline > gpurun_out/qprof.log 2>&1
