#!/bin/bash
# Round-3 GPU check 26: knob re-sweep on the records build (C2, 20 and 256 iterations)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, timeout, command...: rc 0/1 go on, anything else stops
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep '^{' gpurun_out/$name.log 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])' 2>/dev/null)"
  if [[ $rc != 0 && $rc != 1 ]]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
B="python3 bench.py --no-cpu --no-compare --no-count"
for st in 20 256; do
  step k_def_s$st 300 $B --steps $st --warmup 3
  step k_grid1_s$st 300 env WR_SHADE_GRID=1 $B --steps $st --warmup 3
  step k_grid4_s$st 300 env WR_SHADE_GRID=4 $B --steps $st --warmup 3
  step k_tie256_s$st 300 env WR_TIE_WAVE_MAX=256 $B --steps $st --warmup 3
  step k_tie1024_s$st 300 env WR_TIE_WAVE_MAX=1024 $B --steps $st --warmup 3
  step k_pipes12_s$st 300 env WR_PIPES=12 $B --steps $st --warmup 3
  step k_def2_s$st 300 $B --steps $st --warmup 3
done
echo done
