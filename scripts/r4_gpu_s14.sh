#!/bin/bash
# Round-4 session: the -m gpu suite and BVH verification on the build with the
# per-scene tree width (C4 searches the 4-wide tree) and the hash-table wave
# walk; then the C4 and C2 lines with their work counts.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r4_$n.out 2> gpurun_out/r4_$n.err
  local rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r4_$n.out | head -1) $(tail -c 160 gpurun_out/r4_$n.out | tr '\n' ' ')"
  [ $rc -eq 0 ] || exit $rc
}
step suite 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step verify 400 python3 scripts/verify_bvh.py --out gpurun_out/bvh_verify_r4b.json
step c4_line 400 python3 bench.py --config c4 --no-cpu --no-compare
step c2_line 300 python3 bench.py --no-cpu --no-compare
