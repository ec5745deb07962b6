#!/bin/bash
# Round-3 GPU check 13: events without the system-scope fence (default now) vs
# with it (WR_EVENT_SYSTEM_FENCE=1), deferral on / off; BVH + BDPT film tests.
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
step tests13 600 python -u -m pytest tests/test_gpu_bvh.py tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "bdpt or bvh or deferred or film or device"
B="python3 bench.py --no-cpu --no-compare --no-count"
for st in 20 1; do
  step f_sys_d0_s$st 300 env WR_EVENT_SYSTEM_FENCE=1 $B --steps $st --warmup 3
  step f_dev_d0_s$st 300 $B --steps $st --warmup 3
  step f_dev_d1q32_s$st 300 env GPU_MAX_HW_QUEUES=32 WR_DEFER=1 $B --steps $st --warmup 3
  step f_dev_d1p8_s$st 300 env WR_PIPES=8 WR_DEFER=1 $B --steps $st --warmup 3
  step f_dev_d0p8_s$st 300 env WR_PIPES=8 WR_DEFER=0 $B --steps $st --warmup 3
done
step f_dev_d0_c4 400 $B --config c4 --steps 64 --warmup 2
step f_dev_d1q32_c4 400 env GPU_MAX_HW_QUEUES=32 WR_DEFER=1 $B --config c4 --steps 64 --warmup 2
echo done
