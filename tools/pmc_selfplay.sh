#!/bin/bash
# PMC passes for the config-3 self-play kernels (select / network / backup / commit), run on
# the GPU box from the repo root: one rocprofv3 --pmc run per counter group (FETCH_SIZE and
# WRITE_SIZE in passes of their own), then tools/pmc_selfplay_summary.py -> JSON.
# usage: tools/pmc_selfplay.sh OUTDIR ROUND
set -euo pipefail
OUT=${1:-gpurun_out/pmc_sp}
ROUND=${2:-r01}
export TMPDIR=/tmp
mkdir -p "$OUT"
CMD=(python3 bench.py --workload selfplay --steps 40 --warmup 10 --no-cpu-baseline)
pass() { local name=$1; shift; timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- "${CMD[@]}" > "$OUT/$name.log" 2>&1; }
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_MFMA
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- "${CMD[@]}" > "$OUT/trace.log" 2>&1
python3 tools/pmc_selfplay_summary.py "$OUT" "$ROUND" > "$OUT/summary.json"
cat "$OUT/summary.json"
