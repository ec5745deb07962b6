#!/bin/bash
# Round-3 GPU check 12: deferral test with the counter, and a queue / pipeline matrix
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, timeout, command...: rc 0/1 go on, anything else stops
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [[ $rc != 0 && $rc != 1 ]]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
step defer_test 400 python -u -m pytest tests/test_gpu_bvh.py -m gpu -x -v --timeout 300 --timeout-method thread -k "deferred"
B="python3 bench.py --no-cpu --no-compare --no-count"
for st in 20 1; do
  step m_q16_p8_d0_s$st 300 env WR_PIPES=8 WR_DEFER=0 $B --steps $st --warmup 3
  step m_q16_p8_d1_s$st 300 env WR_PIPES=8 WR_DEFER=1 $B --steps $st --warmup 3
  step m_q16_p16_d1_s$st 300 env WR_DEFER=1 $B --steps $st --warmup 3
  step m_q32_p16_d1_s$st 300 env GPU_MAX_HW_QUEUES=32 WR_DEFER=1 $B --steps $st --warmup 3
  step m_q24_p12_d1_s$st 300 env GPU_MAX_HW_QUEUES=24 WR_PIPES=12 WR_DEFER=1 $B --steps $st --warmup 3
done
echo done
