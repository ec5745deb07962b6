#!/bin/bash
# Round-3 GPU check 17: group size 1 vs 2 (library variants), piece_cap sweep
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="product= g1=winmad-s-raytracer-v1.0_amd/variants/g1.so" \
CASES="b1:--steps 1 --warmup 3|b4:--steps 4 --warmup 3|b20:--steps 20 --warmup 3|b256:--steps 256 --warmup 3|c4:--config c4 --steps 64 --warmup 2" \
  timeout -k 10 900 bash scripts/ab_libs.sh || exit $?
step() {  # name, timeout, command...: rc 0/1 go on, anything else stops
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep '^{' gpurun_out/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["pipelines"])' 2>/dev/null)"
  if [[ $rc != 0 && $rc != 1 ]]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
B="python3 bench.py --no-cpu --no-compare --no-count"
for pc in 524288 1048576; do
  for st in 1 4 20 256; do
    step pc${pc}_s$st 300 env WR_PIECE_CAP=$pc $B --steps $st --warmup 3
  done
done
echo done
