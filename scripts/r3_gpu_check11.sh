#!/bin/bash
# Round-3 GPU check 11: deferred hard rays -- BDPT film parity with WR_DEFER=1,
# then A/B benches (defer off at 16 queues / on at 32 queues / off at 32 queues).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab11
export TMPDIR=/tmp
step() {  # name, timeout, command...: rc 0/1 go on, anything else stops
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [[ $rc != 0 && $rc != 1 ]]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
step defer_tests 600 env WR_DEFER=1 python -u -m pytest tests/test_gpu.py tests/test_gpu_bvh.py -m gpu -x -v --timeout 300 --timeout-method thread -k "bdpt or bvh or pieces or pipeline or cli"
B="python3 bench.py --no-cpu --no-compare"
for st in 20 1; do
  step ab_off16_s$st 300 env WR_ISSUE_LOG=1 $B --steps $st --warmup 3
  step ab_on32_s$st 300 env WR_ISSUE_LOG=1 GPU_MAX_HW_QUEUES=32 $B --steps $st --warmup 3
  step ab_off32_s$st 300 env WR_ISSUE_LOG=1 GPU_MAX_HW_QUEUES=32 WR_DEFER=0 $B --steps $st --warmup 3
done
step ab_off16_c4 400 $B --config c4 --steps 64 --warmup 2 --no-count
step ab_on32_c4 400 env GPU_MAX_HW_QUEUES=32 $B --config c4 --steps 64 --warmup 2 --no-count
step ab_on32_s256 400 env GPU_MAX_HW_QUEUES=32 $B --steps 256 --warmup 3 --no-count
echo done
