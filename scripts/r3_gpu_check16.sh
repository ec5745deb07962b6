#!/bin/bash
# Round-3 GPU check 16: grazing winners to the KD walk + piece_min default:
# full -m gpu suite, default bench, C4 bench, BVH verification runs
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
step gputest16 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread
step bench16 300 python3 bench.py --steps 20 --warmup 5
step bench16_c4 400 python3 bench.py --config c4 --steps 64 --warmup 2 --no-cpu --no-compare
step verify16 600 python3 scripts/verify_bvh.py --configs c2,vcm,c3,c4 --iters 64,16,16,8 --out gpurun_out/verify16.json
echo done
