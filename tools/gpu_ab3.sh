#!/bin/bash
# A/B of library builds on the config-3 self-play step (GPU box, repo root): the product
# library and each ablib/lib<name>.so given, twice each, interleaved; bench value per run.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for v in product "$@"; do
    if [ "$v" = product ]; then lib=""; else lib="$PWD/ablib/lib$v.so"; fi
    SPLENDOR_AMD_LIB=$lib timeout -k 10 200 python3 -u bench.py --workload selfplay --steps 2000 --window 0 \
        --no-cpu-baseline > gpurun_out/ab_$v.$rep.json 2> gpurun_out/ab_$v.$rep.err || exit 1
    echo "$v $rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$v.$rep.json | head -1)"
  done
done
