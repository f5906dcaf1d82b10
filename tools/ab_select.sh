#!/bin/bash
# A/B of k_select variants (run on the GPU box from the repo root after building the
# libraries in ablib/ on the host, e.g.
#   hipcc ... -DSELECT_SPEC=0 -o ablib/libA.so; -DSELECT_SPEC=1 -DSELECT_WAVES=5 -o ablib/libB.so; ...):
# the config-3 bench with each library (SPLENDOR_AMD_LIB), twice, interleaved. The games are
# identical across variants (the search is exact), so only the time differs.
set -euo pipefail
for v in ${VARIANTS:-A B C A B C}; do
    SPLENDOR_AMD_LIB=$PWD/ablib/lib$v.so timeout -k 10 200 python -u bench.py --workload selfplay --steps 2000 \
        --prefill 3000 --window 4000 --no-cpu-baseline > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err
    python -c "import json;d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]);print('$v', round(d['value']/1e6,2), round(d['selfplay']['window']['rollouts_per_s']/1e6,2))" >> gpurun_out/ab.txt
done
