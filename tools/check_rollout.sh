#!/bin/bash
# Rollout change check on the GPU box (repo root): env + config parity tests, per-phase
# probes at 20 and 100 moves per launch, driver-style and default env bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py tests/test_configs_gpu.py -x -v -m gpu --timeout 300 \
    --timeout-method thread > gpurun_out/env_tests.log 2>&1 || exit 1
for k in 20 100; do timeout -k 10 60 ./tools/time_rollout $k > gpurun_out/tr$k.log 2>&1 || exit 1; done
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-selfplay --no-cpu-baseline > gpurun_out/b20.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --no-selfplay --no-cpu-baseline > gpurun_out/b1000.log 2>&1
