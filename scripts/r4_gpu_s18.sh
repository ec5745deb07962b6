#!/bin/bash
# Round-4 closing lines on the final build: the driver's default C2 run, C2 at
# 1 and 20 iterations, C3, C4, VCM (with their work counts), the smoke test.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r4_$n.out 2> gpurun_out/r4_$n.err
  local rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r4_$n.out | head -1)"
  [ $rc -eq 0 ] || exit $rc
}
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step fin_c2_default 400 python3 bench.py
B="python3 bench.py --no-cpu --no-compare"
step fin_c2_s1 200 $B --steps 1
step fin_c2_s20 300 $B --steps 20
step fin_c4 400 $B --config c4
step fin_vcm 400 $B --config vcm
step fin_c3 300 $B --config c3
