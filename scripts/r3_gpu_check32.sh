#!/bin/bash
# WR_RESOLVE_GRID (k_fast_resolve blocks per CU; unset = the search's grid,
# 21 per CU) at 1, 4, 20 and 256 iterations: the resolve's dispatch of
# thousands of mostly idle workgroups is ~36 us of each late step's chain.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=16
B="python -u bench.py --no-cpu --no-compare --no-count"
for rep in 1 2; do
for cs in "b1:--steps 1 --warmup 3" "b4:--steps 4 --warmup 3" "b20:--steps 20 --warmup 3" "b256:--steps 256"; do
  name=${cs%%:*}; args=${cs#*:}
  for g in def 2 4; do
    if [[ $g == def ]]; then unset WR_RESOLVE_GRID; else export WR_RESOLVE_GRID=$g; fi
    out=gpurun_out/rg2_${name}_${g}_r$rep.json
    timeout -k 10 240 $B $args > $out 2> ${out%.json}.err
    rc=$?
    echo "$name grid=$g rep$rep rc=$rc $(python3 -c "import json;print(json.loads(open('$out').read().strip().splitlines()[-1])['value'])" 2>/dev/null)"
    if [[ $rc != 0 ]]; then exit $rc; fi
  done
done
done
