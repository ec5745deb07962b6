#!/bin/bash
# GPU suite on the current build, then A/B of WR_RESOLVE_GRID (blocks per CU of
# k_fast_resolve; unset = the search's grid) on C2 20 / 256 iterations.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [[ $rc != 0 ]]; then exit $rc; fi
export GPU_MAX_HW_QUEUES=16
B="python -u bench.py --no-cpu --no-compare --no-count"
for rep in 1 2; do
for cs in "b20:--steps 20 --warmup 3" "b256:--steps 256"; do
  name=${cs%%:*}; args=${cs#*:}
  for g in def 1 2 4 8; do
    if [[ $g == def ]]; then unset WR_RESOLVE_GRID; else export WR_RESOLVE_GRID=$g; fi
    out=gpurun_out/rg_${name}_${g}_r$rep.json
    timeout -k 10 240 $B $args > $out 2> ${out%.json}.err
    rc=$?
    echo "$name grid=$g rep$rep rc=$rc $(python3 -c "import json;print(json.loads(open('$out').read().strip().splitlines()[-1])['value'])" 2>/dev/null)"
    if [[ $rc != 0 ]]; then exit $rc; fi
  done
done
done
