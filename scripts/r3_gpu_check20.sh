#!/bin/bash
# Round-3 GPU check 20: C5 rank-shard line (C4 scene, 512 iterations at
# iter_begin 512), 1-iteration issue timing with 1-3 issue threads
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, timeout, command...: rc 0/1 go on, anything else stops
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep '^{' gpurun_out/$name.log 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["pipelines"])' 2>/dev/null) $(grep 'wr issue\] [0-9]* pipe' gpurun_out/$name.log | tail -1)"
  if [[ $rc != 0 && $rc != 1 ]]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
step c5shard 600 python3 bench.py --config c4 --steps 512 --iter-begin 512 --warmup 3 --no-cpu --no-compare
B="python3 bench.py --no-cpu --no-compare --no-count"
for th in 1 3; do
  step it1_th$th 300 env WR_ISSUE_LOG=1 WR_ISSUE_THREADS=$th $B --steps 1 --warmup 3
  step it2_th$th 300 env WR_ISSUE_LOG=1 WR_ISSUE_THREADS=$th $B --steps 2 --warmup 3
done
step it20_th4 300 env WR_ISSUE_LOG=1 WR_ISSUE_THREADS=4 $B --steps 20 --warmup 3
step it20_th1 300 env WR_ISSUE_LOG=1 WR_ISSUE_THREADS=1 $B --steps 20 --warmup 3
echo done
