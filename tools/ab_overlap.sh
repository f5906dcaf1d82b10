#!/bin/bash
# A/B on the GPU box (repo root): config-3 bench with ablib/libB.so (lane-serial backup scan,
# batches of 4) and ablib/libC.so (batches of 8), with and without the terminal-backup overlap
# (SPLENDOR_OVERLAP), interleaved twice. Results in gpurun_out/ab.txt.
set -euo pipefail
rm -f gpurun_out/ab.txt
for v in B1 C1 B0 B1 C1 B0; do
    lib=${v:0:1}; ov=${v:1:1}
    SPLENDOR_OVERLAP=$ov SPLENDOR_AMD_LIB=$PWD/ablib/lib$lib.so timeout -k 10 200 python -u bench.py --workload selfplay \
        --steps 2000 --prefill 3000 --window 4000 --no-cpu-baseline > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err
    python -c "import json;d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]);print('$v', round(d['value']/1e6,2), round(d['ms_per_step'],4), round(d['selfplay']['window']['rollouts_per_s']/1e6,2))" >> gpurun_out/ab.txt
done
