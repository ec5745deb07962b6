#!/bin/bash
# Round-3 GPU check 14: reserve test, wr_tot with wr_reserve, piece_min sweep
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
step api14 400 python -u -m pytest tests/test_gpu_api.py -m gpu -x -q --timeout 300 --timeout-method thread
step wrtot14 400 python3 scripts/wr_tot_profile.py 20 256
B="python3 bench.py --no-cpu --no-compare --no-count"
for pm in 16384 262144 524288 1048576; do
  for st in 1 4 20; do
    step pm${pm}_s$st 300 env WR_PIECE_MIN=$pm $B --steps $st --warmup 3
  done
done
echo done
