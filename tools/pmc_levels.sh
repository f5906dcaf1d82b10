#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/lv
for s in 10 25 50 100 200; do
  LD_LIBRARY_PATH=alphazero-general-ori_amd timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH --kernel-include-regex k_select --kernel-iteration-range "[1500-1600]" --output-format csv -d gpurun_out/lv/s$s -o run -- tools/time_select_w7 $s 1500 100 2048 > gpurun_out/lv/s$s.log 2>&1 || exit 1
  echo "sims $s done" >> gpurun_out/lv/progress.log
done
