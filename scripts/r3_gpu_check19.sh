#!/bin/bash
# Round-3 GPU check 19: fused deferral (late work in the next step's launches):
# parity tests, then defer off / on A/B
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, timeout, command...: rc 0/1 go on, anything else stops
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep '^{' gpurun_out/$name.log 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["pipelines"])' 2>/dev/null)"
  if [[ $rc != 0 && $rc != 1 ]]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
step t19 600 env WR_DEFER=1 python -u -m pytest tests/test_gpu_bvh.py tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "bdpt or bvh or deferred or pieces or pipeline"
[[ $(grep -c failed gpurun_out/t19.log) == 0 ]] || { echo "tests failed"; tail -30 gpurun_out/t19.log; exit 1; }
B="python3 bench.py --no-cpu --no-compare --no-count"
for rep in 1 2; do
for st in 1 4 20 256; do
  step d0_s${st}_r$rep 300 env WR_DEFER=0 $B --steps $st --warmup 3
  step d1_s${st}_r$rep 300 env WR_DEFER=1 $B --steps $st --warmup 3
done
done
step d0_c4 300 env WR_DEFER=0 $B --config c4 --steps 64 --warmup 2
step d1_c4 300 env WR_DEFER=1 $B --config c4 --steps 64 --warmup 2
echo done
