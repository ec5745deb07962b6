#!/bin/bash
# Round-4 session: the scan list with the cell filter and four leaves per lane
# per round -- BVH parity tests, C2 at 1 / 20 iterations, C4, the per-step log
# at 1 iteration; INTEGRATION.md section 1's program (example_main) against
# bench.py at 1920x1080 / 256 iterations, each in a fresh process.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r4_$n.out 2> gpurun_out/r4_$n.err
  local rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r4_$n.out | head -1) $(tail -c 120 gpurun_out/r4_$n.out | tr '\n' ' ')"
  [ $rc -eq 0 ] || exit $rc
}
step btests 500 python -u -m pytest tests/test_gpu_bvh.py -x -q --timeout 300 --timeout-method thread
B="python3 bench.py --warmup 3 --no-cpu --no-compare --no-count"
step s10_b1_r1 120 $B --steps 1
step s10_b1_r2 120 $B --steps 1
step s10_b20 200 $B --steps 20
step s10_c4 300 $B --config c4
WR_TRACE_LOG=1 step s10_log_b1 200 python3 bench.py --warmup 1 --steps 1 --no-cpu --no-compare
EX=$(mktemp -d)
mkdir -p $EX/src && printf '7\n1\n8\n4\n1920\n1080\n5\n400\n' > $EX/src/parameters.para
SCENE=$(python3 -c "import os, sys; sys.path[:0] = ['tests', 'winmad-s-raytracer-v1.0_amd']; import _scenes; print(os.path.abspath(_scenes.torus(1920, 1080)))")
( cd $EX && timeout -k 10 300 "$GRAFT_REPO_ROOT/winmad-s-raytracer-v1.0_amd/example_main" "$SCENE" o.ppm -bpt 256 ) \
  > gpurun_out/r4_example_main.out 2>&1
rc=$?
echo "example_main rc=$rc $(tail -1 gpurun_out/r4_example_main.out)"
[ $rc -eq 0 ] || exit $rc
step s10_b256 300 $B --steps 256
