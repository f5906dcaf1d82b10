#!/bin/bash
# A/B of rollout-kernel build variants (run on the GPU box from the repo root):
# tools/ab_rollout.sh ROUNDS base v1 v2 ... — "base" is the in-tree library, vN is
# exp/libvN.so (built with -D macros on the host); config-2 bench lines under gpurun_out/ab/.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$1; shift
mkdir -p gpurun_out/ab
for r in $(seq 1 "$R"); do
  for v in "$@"; do
    if [ "$v" = base ]; then unset SPLENDOR_AMD_LIB; else export SPLENDOR_AMD_LIB=$PWD/exp/lib$v.so; fi
    timeout -k 10 120 python3 bench.py --steps 1000 --warmup 100 --no-cpu-baseline --no-selfplay > "gpurun_out/ab/${v}_$r.log" 2>&1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']/1e9,4), round(d['roofline']['kernel_avg_us'],1))" "gpurun_out/ab/${v}_$r.log" "$v"
  done
done
