#!/bin/bash
# A/B on the GPU box (repo root): the config-3 bench with each of ablib/lib{A,B,C}.so
# (built on the host), interleaved twice; results in gpurun_out/ab.txt.
set -euo pipefail
rm -f gpurun_out/ab.txt
for v in ${VARIANTS:-A B C A B C}; do
    SPLENDOR_AMD_LIB=$PWD/ablib/lib$v.so timeout -k 10 200 python -u bench.py --workload selfplay \
        --steps 2000 --window 4000 --no-cpu-baseline > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err
    python -c "import json;d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]);print('$v', round(d['value']/1e6,2), round(d['ms_per_step'],4), round(d['selfplay']['window']['rollouts_per_s']/1e6,2))" >> gpurun_out/ab.txt
done
