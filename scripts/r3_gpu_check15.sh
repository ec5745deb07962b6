#!/bin/bash
# Round-3 GPU check 15: piece_min sweep, finer (BDPT C2, 1 .. 256 iterations)
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
B="python3 bench.py --no-cpu --no-compare --no-count"
for pm in 393216 524288 655360 786432; do
  for st in 1 2 4 20 256; do
    step pmb${pm}_s$st 300 env WR_PIECE_MIN=$pm $B --steps $st --warmup 3
  done
done
step pmb524288_c4 300 env WR_PIECE_MIN=524288 $B --config c4 --steps 64 --warmup 2
step pmb16384_c4 300 env WR_PIECE_MIN=16384 $B --config c4 --steps 64 --warmup 2
echo done
