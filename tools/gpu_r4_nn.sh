#!/bin/bash
# Round-4 network experiment on the GPU box (repo root), outputs under gpurun_out/: accuracy
# against float64 (product build and the NN_SPLIT=1 build ablib/libsplit.so, 2 and 4
# players), the full-batch network timing of both, and the network parity tests on the split
# build.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
SPL=$PWD/ablib/libsplit.so
for n in 2 4; do
    timeout -k 10 120 python3 -u tools/nn_accuracy.py 4096 $n product >> gpurun_out/nn_accuracy.log 2>&1 || exit 1
    SPLENDOR_AMD_LIB=$SPL timeout -k 10 120 python3 -u tools/nn_accuracy.py 4096 $n split >> gpurun_out/nn_accuracy.log 2>&1 || exit 1
done
timeout -k 10 120 python3 -u tools/nn_fullbatch.py > gpurun_out/nnfb_product.log 2>&1 || exit 1
SPLENDOR_AMD_LIB=$SPL timeout -k 10 120 python3 -u tools/nn_fullbatch.py > gpurun_out/nnfb_split.log 2>&1 || exit 1
SPLENDOR_AMD_LIB=$SPL timeout -k 10 300 python3 -u -m pytest tests/test_nnet.py -m gpu -x -v \
    --timeout 120 --timeout-method thread > gpurun_out/nn_split_tests.log 2>&1
echo "split tests rc=$?"
