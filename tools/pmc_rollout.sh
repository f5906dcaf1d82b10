#!/bin/bash
# PMC passes for the fused rollout kernel (run on the GPU box from the repo root).
# Separate rocprofv3 runs per counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass;
# no --pmc run combines with any trace domain but the kernel trace), then a summary JSON.
# usage: tools/pmc_rollout.sh OUTDIR ROUND [MOVES_PER_LAUNCH]
set -euo pipefail
OUT=${1:-gpurun_out/pmc}
ROUND=${2:-r02}
CHUNK=${3:-100}
export TMPDIR=/tmp
mkdir -p "$OUT"
CMD=(python3 bench.py --workload env --steps $((2 * CHUNK)) --warmup "$CHUNK" --chunk "$CHUNK" --no-cpu-baseline)
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- "${CMD[@]}" > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- "${CMD[@]}" > "$OUT/write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
    --output-format csv -d "$OUT/sq" -o run -- "${CMD[@]}" > "$OUT/sq.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- "${CMD[@]}" > "$OUT/trace.log" 2>&1
python3 tools/pmc_summary.py "$OUT" "$ROUND" "$CHUNK" > "$OUT/summary.json"
cat "$OUT/summary.json"
