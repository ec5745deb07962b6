#!/bin/bash
# Round-4 session: the C2 bench lines of this build (the driver's default
# command, 1 / 20 / 256 iterations), INTEGRATION.md section 1's program
# (example_main) against bench.py at the headline configuration, each in a
# fresh process, and a 1-iteration kernel timeline.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r4_$n.out 2> gpurun_out/r4_$n.err
  local rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r4_$n.out | head -1) $(grep -o 'render: .*' gpurun_out/r4_$n.out | head -1)"
  [ $rc -eq 0 ] || exit $rc
}
step c2_default 300 python3 bench.py
B="python3 bench.py --warmup 3 --no-cpu --no-compare"
step c2_s1 120 $B --steps 1
step c2_s1b 120 $B --steps 1 --no-count
step c2_s20 200 $B --steps 20
step c2_s256 300 $B --steps 256
# example_main: the reference's main() over the mirror, 1920x1080, 256 iterations
EX=$(mktemp -d)
mkdir -p $EX/src && printf '7\n1\n8\n4\n1920\n1080\n5\n400\n' > $EX/src/parameters.para
SCENE=$(python3 -c "import sys; sys.path.insert(0, 'tests'); import _scenes; print(_scenes.torus(1920, 1080))")
( cd $EX && timeout -k 10 300 "$GRAFT_REPO_ROOT/winmad-s-raytracer-v1.0_amd/example_main" "$SCENE" o.ppm -bpt 256 ) \
  > gpurun_out/r4_example_main.out 2>&1
echo "example_main rc=$? $(tail -1 gpurun_out/r4_example_main.out)"
step c2_s256_after_main 300 $B --steps 256 --no-count
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_s9 -o run -- \
  python3 bench.py --steps 1 --warmup 3 --no-cpu --no-count --no-compare > gpurun_out/r4_tl_s9.out 2>&1
echo "tl_s9 rc=$?"
