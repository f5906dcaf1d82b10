#!/bin/bash
# Arena-size experiment (VERDICT r04 Next #2): config-3 steady state at several arena budgets
# (bench.py --mem-gib; 0 = the default 80 % of free HBM). Per budget: one bench line, then the
# PMC memory pass (UTCL1 translation hits / misses, L2 hits) and a kernel trace over the
# select / backup kernels (tools/pmc_selfplay.sh PASSES=mem). Outputs under gpurun_out/pool/.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/pool
mkdir -p "$OUT"
for MEM in ${MEMS:-0 80 40}; do
    echo "$(date +%T) mem $MEM bench" >> "$OUT/progress.log"
    timeout -k 10 240 python3 -u bench.py --workload selfplay --steps 1000 --window 2000 --no-cpu-baseline \
        --mem-gib "$MEM" > "$OUT/bench_$MEM.json" 2> "$OUT/bench_$MEM.err" || exit 1
    PASSES=mem BENCH_EXTRA="--mem-gib $MEM" timeout -k 10 600 bash tools/pmc_selfplay.sh "$OUT/pmc_$MEM" r05 6000 200 \
        > "$OUT/pmc_$MEM.log" 2>&1 || exit 1
done
echo "$(date +%T) done" >> "$OUT/progress.log"
