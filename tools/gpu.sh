#!/bin/bash
# The one runner for GPU-box evidence (run there from the repo root, e.g.
#   gpurun --timeout 900 -- 'bash tools/gpu.sh tests bench'
# ). Each step runs under its own time limit; the steps are chained and the script stops at
# the first failure (no GPU step runs after a fault, an abort or a time limit). Outputs go
# under gpurun_out/.
#
#   tests     pytest -m gpu (one process; per-test timeout)           -> gpurun_out/gpu_tests.log
#   smoke     __graft_entry__.smoke()                                  -> gpurun_out/smoke.log
#   bench     the default bench line (headline + secondary objects)    -> gpurun_out/bench.json
#   selfplay  the config-3 headline alone                              -> gpurun_out/selfplay.json
#   trace     config-3 kernel trace + stats (rocprofv3)                -> gpurun_out/prof_sp/ (or prof_<TREE>)
#   split     per-iteration kernel split from the trace (needs trace)  -> gpurun_out/split.txt
#   spikes    the slowest launches of each kernel and their iterations (needs trace) -> gpurun_out/spikes.json
#   pmc       PMC passes over the self-play kernels (pmc_selfplay.sh)  -> gpurun_out/pmc_sp/
#   nn        full-batch network trace + HBM counters (nn_fullbatch.sh) -> gpurun_out/nnfb/
#   trainprior  tools/train_prior.py: a few Coach.learn iterations -> gpurun_out/trained_2p.pt,
#             then the config-3 headline on those weights -> gpurun_out/selfplay_trained.json
#   accuracy  the fused network vs float64 on 4,096 positions at 2p and 4p (nn_accuracy.py)
#             -> gpurun_out/nn_accuracy.jsonl
#   ab        interleaved A/B of the product against each V in $AB: ablib/lib<V>.so, or a whole
#             older tree ablib/<V>/ (bench.py + package) (config-3 bench twice each) -> gpurun_out/ab.txt
#   probe     k_select_lanes phase probes (ablib/lib<V>.so for V in ${PROBES:-probe}, -DSELECT_PROBE=1) -> gpurun_out/<V>.json
#   gcprobe   compact_tree phase probes (ablib/libgcprobe.so, -DGC_PROBE=1)    -> gpurun_out/gcprobe.json
#   nnprobe   per-layer cycle probes of the network kernel (ablib/libnnprobe.so, -DNN_PROBE=1) -> gpurun_out/nnprobe.json
#   lmprobe   per-workgroup timeline of k_leaf_mask (ablib/liblmprobe.so, -DLM_PROBE=1) -> gpurun_out/lmprobe.json
#   nnidx     the network on the search's NN-leaf list alone (tools/nn_indexed_time.py)  -> gpurun_out/nnidx.jsonl
#   bounds    the bounds-checked build (ablib/libchk.so: tools/bounds_check.sh on
#             the host first) under capacity pressure                   -> gpurun_out/bounds_chk.json
# ROUND (default r05) names the summaries; EXTRA adds bench arguments to selfplay/trace; TREE=<V>
# makes trace / split / spikes run the older tree ablib/<V>/ (outputs *_<V>).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
ROUND=${ROUND:-r06}
TR=${TREE:-sp}                                             # trace / split / spikes: TREE=<V> traces
TB=bench.py; [ -n "${TREE:-}" ] && TB="ablib/$TREE/bench.py"  # the older tree ablib/<V>/ instead
step() {
    echo "$(date +%T) $1 start" >> gpurun_out/progress.log
    case "$1" in
    tests)
        timeout -k 10 1000 python3 -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread \
            > gpurun_out/gpu_tests.log 2>&1 ;;
    smoke)
        timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 ;;
    bench)
        timeout -k 10 900 python3 -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err ;;
    selfplay)
        timeout -k 10 300 python3 -u bench.py --workload selfplay --no-cpu-baseline ${EXTRA:-} \
            > gpurun_out/selfplay.json 2> gpurun_out/selfplay.err ;;
    trace)
        timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TR -o sp -- \
            python3 "$TB" --workload selfplay --steps 2000 --window 4000 --no-cpu-baseline ${EXTRA:-} \
            > gpurun_out/prof_$TR.log 2>&1 ;;
    split)
        python3 tools/trace_split.py "$(find gpurun_out/prof_$TR -name '*kernel_trace.csv' | head -n 1)" 6000 \
            > gpurun_out/split_$TR.txt ;;
    spikes)
        python3 tools/trace_spikes.py "$(find gpurun_out/prof_$TR -name '*kernel_trace.csv' | head -n 1)" 4000 8 \
            > gpurun_out/spikes_$TR.json ;;
    pmc)
        timeout -k 10 1000 bash tools/pmc_selfplay.sh gpurun_out/pmc_sp "$ROUND" > gpurun_out/pmc_sp.log 2>&1 ;;
    nn)
        timeout -k 10 400 bash tools/nn_fullbatch.sh "$ROUND" > gpurun_out/nnfb.log 2>&1 ;;
    trainprior)
        timeout -k 10 900 python3 -u tools/train_prior.py gpurun_out/trained_2p.pt "${ITERS:-4}" "${GAMES:-4096}" \
            > gpurun_out/train_prior.jsonl 2> gpurun_out/train_prior.err &&
        timeout -k 10 300 python3 -u bench.py --workload selfplay --no-cpu-baseline --net gpurun_out/trained_2p.pt \
            > gpurun_out/selfplay_trained.json 2> gpurun_out/selfplay_trained.err ;;
    accuracy)
        rm -f gpurun_out/nn_accuracy.jsonl
        for np_ in 2 4; do
            timeout -k 10 240 python3 -u tools/nn_accuracy.py 4096 $np_ >> gpurun_out/nn_accuracy.jsonl \
                2> gpurun_out/nn_accuracy.err || return 1
        done ;;
    ab)
        rm -f gpurun_out/ab.txt
        for rep in 1 2; do
            for v in product ${AB:-}; do
                # a variant is a library (ablib/lib<V>.so under this tree's Python) or a whole
                # tree (ablib/<V>/bench.py with its own package: builds whose ABI differs)
                b=bench.py; lib=""
                if [ -f "ablib/$v/bench.py" ]; then b="ablib/$v/bench.py"; elif [ "$v" != product ]; then lib="$PWD/ablib/lib$v.so"; fi
                SPLENDOR_AMD_LIB=$lib timeout -k 10 240 python3 -u "$b" --workload selfplay --steps 2000 \
                    --window 0 --no-cpu-baseline ${EXTRA:-} > gpurun_out/ab_$v.$rep.json 2> gpurun_out/ab_$v.$rep.err || return 1
                echo "$v $rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$v.$rep.json | head -1)" >> gpurun_out/ab.txt
            done
        done ;;
    probe)
        for v in ${PROBES:-probe}; do
            SPLENDOR_AMD_LIB=$PWD/ablib/lib$v.so timeout -k 10 200 python3 -u tools/select_probe.py \
                > gpurun_out/$v.json 2> gpurun_out/$v.err || { echo "$v rc=$?" >> gpurun_out/progress.log; return 1; }
        done ;;
    gcprobe)
        SPLENDOR_AMD_LIB=$PWD/ablib/libgcprobe.so timeout -k 10 200 python3 -u tools/gc_probe.py \
            > gpurun_out/gcprobe.json 2> gpurun_out/gcprobe.err ;;
    lmprobe)
        SPLENDOR_AMD_LIB=$PWD/ablib/liblmprobe.so timeout -k 10 300 python3 -u tools/lm_probe.py \
            > gpurun_out/lmprobe.json 2> gpurun_out/lmprobe.err ;;
    nnidx)
        timeout -k 10 120 python3 -u tools/nn_indexed_time.py >> gpurun_out/nnidx.jsonl 2>> gpurun_out/nnidx.err ;;
    nnprobe)
        SPLENDOR_AMD_LIB=$PWD/ablib/libnnprobe.so timeout -k 10 200 python3 -u tools/nn_probe.py \
            > gpurun_out/nnprobe.json 2> gpurun_out/nnprobe.err ;;
    bounds)
        SPLENDOR_AMD_LIB=$PWD/ablib/libchk.so timeout -k 10 300 python3 -u tools/bounds_check.py --tag chk \
            --iters "${ITERS:-6000}" > gpurun_out/bounds_chk.json 2> gpurun_out/bounds_chk.err ;;
    *)
        echo "unknown step $1" >&2; return 2 ;;
    esac
    local rc=$?
    echo "$(date +%T) $1 rc=$rc" >> gpurun_out/progress.log
    return $rc
}
for s in "$@"; do
    step "$s" || exit $?
done
