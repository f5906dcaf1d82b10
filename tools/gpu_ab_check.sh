#!/bin/bash
# parity subset on the in-tree library, then a config-3 A/B of ablib/libA.so vs libB.so
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_mcts_gpu.py tests/test_selfplay_gpu.py tests/test_env_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_ab.log 2>&1 || { tail -30 gpurun_out/t_ab.log; exit 1; }
tail -2 gpurun_out/t_ab.log
VARIANTS="A B A B" bash tools/ab_libs.sh || exit 1
cat gpurun_out/ab.txt
