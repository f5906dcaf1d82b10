#!/bin/bash
# 24-byte edges: parity subset, config-3 A/B (ablib/libA = 16+16-byte halves, libB = 16+8), config 4 at steady state
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_mcts_gpu.py tests/test_selfplay_gpu.py tests/test_arena_gpu.py tests/test_noise_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_e24.log 2>&1 || { tail -30 gpurun_out/t_e24.log; exit 1; }
tail -2 gpurun_out/t_e24.log
VARIANTS="A B A B" bash tools/ab_libs.sh || exit 1
cat gpurun_out/ab.txt
timeout -k 10 400 python -u bench.py --workload config4 --no-cpu-baseline --prefill 45000 --stagger 40000 --window 4000 --steps 1000 > gpurun_out/c4.log 2> gpurun_out/c4.err
