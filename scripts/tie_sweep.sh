#!/bin/bash
# WR_TIE_WAVE_MAX sweep: C2 at 1 / 20 / 256 iterations, C4 at 64 (bench lines to gpurun_out/tie_*.json)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="python -u bench.py --no-cpu --no-compare --no-count"
for tw in ${TIE_VALUES:-512 2048 8192}; do
  for cfg in "b1:--steps 1 --warmup 3" "b20:--steps 20 --warmup 3" "b256:--steps 256" "c4:--config c4 --steps 64"; do
    name=${cfg%%:*}; args=${cfg#*:}
    WR_TIE_WAVE_MAX=$tw timeout -k 10 200 $B $args > gpurun_out/tie_${name}_$tw.json 2> gpurun_out/tie_${name}_$tw.err
    rc=$?
    echo "$name tie_wave_max=$tw rc=$rc $(python3 -c "import json;print(json.loads(open('gpurun_out/tie_${name}_$tw.json').read().strip().splitlines()[-1])['value'])" 2>/dev/null)"
    if [[ $rc != 0 ]]; then exit $rc; fi
  done
done
