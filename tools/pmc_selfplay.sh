#!/bin/bash
# PMC passes for the self-play kernels (select / leaf mask / network / backup / commit) in a
# steady-state window (run on the GPU box from the repo root): one rocprofv3 --pmc run per
# counter group (FETCH_SIZE and WRITE_SIZE in passes of their own, <= 8 SQ / 4 TCP / 2 TCC
# counters per pass), then tools/pmc_selfplay_summary.py -> JSON over the last STEPS
# dispatches of each kernel.
# usage: tools/pmc_selfplay.sh OUTDIR ROUND [WARMUP] [STEPS]   (PASSES="sq sq2 ..." for a subset)
set -euo pipefail
OUT=${1:-gpurun_out/pmc_sp}
ROUND=${2:-r03}
WARM=${3:-6000}
STEPS=${4:-200}
export TMPDIR=/tmp
mkdir -p "$OUT"
CMD=(python3 bench.py --workload selfplay --prefill "$WARM" --warmup 20 --steps "$STEPS" --window 0 --no-cpu-baseline ${BENCH_EXTRA:-})
# counters only for the self-play kernels, dispatches WARM+40 .. WARM+40+STEPS of each (the
# timed steps; k_gc runs twice per iteration, so its range covers the second half of them)
FILT=(--kernel-include-regex "k_(select|leaf_mask|nn_forward|backup|commit|gc)" --kernel-iteration-range "[$((WARM + 40))-$((WARM + 40 + STEPS))]")
PASSES=${PASSES:-fetch write sq sq2 mem ea}
pass() {
    local name=$1; shift
    [[ " $PASSES " == *" $name "* ]] || return 0
    echo "$(date +%T) pass $name start" >> "$OUT/progress.log"
    timeout -k 10 170 rocprofv3 --pmc "$@" "${FILT[@]}" --output-format csv -d "$OUT/$name" -o run -- "${CMD[@]}" > "$OUT/$name.log" 2>&1
    echo "$(date +%T) pass $name done" >> "$OUT/progress.log"
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
pass sq2 SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM
pass mem TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCC_HIT_sum TCC_MISS_sum
pass ea TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_128B_sum
echo "$(date +%T) trace start" >> "$OUT/progress.log"
timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- "${CMD[@]}" > "$OUT/trace.log" 2>&1
python3 tools/pmc_selfplay_summary.py "$OUT" "$ROUND" "$STEPS" "$WARM" > "$OUT/summary.json"
cat "$OUT/summary.json"
