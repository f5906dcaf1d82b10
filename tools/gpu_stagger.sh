#!/bin/bash
# phase-stagger check (GPU box): restart test, then config 3 at two prefill lengths
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_selfplay_gpu.py tests/test_capi.py -x -v -k "restart or capi or export" --timeout 200 --timeout-method thread > gpurun_out/stagger_tests.log 2>&1 && \
timeout -k 10 200 python -u bench.py --workload selfplay --no-cpu-baseline > gpurun_out/stagger_a.log 2> gpurun_out/stagger_a.err && \
timeout -k 10 200 python -u bench.py --workload selfplay --no-cpu-baseline --prefill 15000 --stagger 4800 > gpurun_out/stagger_b.log 2> gpurun_out/stagger_b.err
