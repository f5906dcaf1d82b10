#!/bin/bash
# Full-batch k_nn_forward evidence for the headline roofline (GPU box, repo root): kernel trace
# + stats, then FETCH_SIZE and WRITE_SIZE in passes of their own, over tools/nn_fullbatch.py
# (60 launches at B = 32,768, 2 players); summary -> gpurun_out/nnfb/summary.json
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/nnfb
ROUND=${1:-r03}
mkdir -p "$OUT"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 tools/nn_fullbatch.py > "$OUT/trace.log" 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c --kernel-include-regex "k_nn_forward" --output-format csv -d "$OUT/$c" -o run -- python3 tools/nn_fullbatch.py > "$OUT/$c.log" 2>&1
done
python3 tools/nn_fullbatch_summary.py "$OUT" "$ROUND" > "$OUT/summary.json"
cat "$OUT/summary.json"
