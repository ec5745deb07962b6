#!/bin/bash
# Round-4 session: C2 at 1 iteration with the binary / 4-wide search tree and
# with three issue threads; then C4's kernel trace with stats.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r4_$n.out 2> gpurun_out/r4_$n.err
  local rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r4_$n.out | head -1)"
  [ $rc -eq 0 ] || exit $rc
}
B="python3 bench.py --warmup 3 --no-cpu --no-compare --no-count"
for r in 1 2; do
  WR_BVH_WIDE=2 step s1_w2_r$r 120 $B --steps 1
  WR_BVH_WIDE=4 step s1_w4_r$r 120 $B --steps 1
  WR_ISSUE_THREADS=3 step s1_it3_r$r 120 $B --steps 1
done
WR_BVH_WIDE=4 step s20_w4 200 $B --steps 20
step s20_w2 200 $B --steps 20
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4b -o run -- \
  python3 bench.py --config c4 --warmup 2 --no-cpu --no-compare --no-count > gpurun_out/r4_c4_prof.out 2>&1
echo "c4 prof rc=$?"
