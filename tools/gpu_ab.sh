#!/bin/bash
# Development check: search parity subset with the in-tree library, then an A/B script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_mcts_gpu.py tests/test_selfplay_gpu.py tests/test_noise_gpu.py tests/test_arena_gpu.py -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/quick_tests.log 2>&1 && \
bash ${AB:-tools/ab_overlap.sh}
