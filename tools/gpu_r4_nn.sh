#!/bin/bash
# Round-4 network evidence on the GPU box (repo root), outputs under gpurun_out/: accuracy
# against float64 and against the reference-recorded outputs, and the full-batch timing, for
# the product library (split-bf16 per-column layers) and the f32-MFMA build
# (ablib/libf32.so: hipcc ... -DNN_SPLIT=0, see alphazero-general-ori_amd/Makefile flags).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
F32=$PWD/ablib/libf32.so
for n in 2 4; do
    timeout -k 10 120 python3 -u tools/nn_accuracy.py 4096 $n split >> gpurun_out/nn_accuracy.log 2>&1 || exit 1
    SPLENDOR_AMD_LIB=$F32 timeout -k 10 120 python3 -u tools/nn_accuracy.py 4096 $n f32 >> gpurun_out/nn_accuracy.log 2>&1 || exit 1
done
timeout -k 10 120 python3 -u tools/nn_fixture_error.py split > gpurun_out/nnfix.log 2>&1 || exit 1
SPLENDOR_AMD_LIB=$F32 timeout -k 10 120 python3 -u tools/nn_fixture_error.py f32 >> gpurun_out/nnfix.log 2>&1 || exit 1
timeout -k 10 120 python3 -u tools/nn_fullbatch.py > gpurun_out/nnfb_split.log 2>&1 || exit 1
SPLENDOR_AMD_LIB=$F32 timeout -k 10 120 python3 -u tools/nn_fullbatch.py > gpurun_out/nnfb_f32.log 2>&1
echo "rc=$?"
