#!/bin/bash
# Round-3 GPU check 6: one path's splat printed by the debug build; benches
# with the early-exit persistent waves (1 / 20 / 256 iterations, C4), and a
# 256-index ray grab (A/B).
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
step debug_path 200 env WR_LIB=winmad-s-raytracer-v1.0_amd/variants/debugpath.so python -u scripts/debug_path.py 0 69 88
B="python -u bench.py --no-cpu --no-compare --no-count"
step e_b1 200 $B --steps 1 --warmup 2
step e_b20 200 $B --steps 20 --warmup 5
step e_b256 300 $B --steps 256
step e_c4 300 $B --config c4 --steps 64
step g_b20 200 env WR_LIB=winmad-s-raytracer-v1.0_amd/variants/grab256.so $B --steps 20 --warmup 5
step g_b256 300 env WR_LIB=winmad-s-raytracer-v1.0_amd/variants/grab256.so $B --steps 256
step g_c4 300 env WR_LIB=winmad-s-raytracer-v1.0_amd/variants/grab256.so $B --config c4 --steps 64
echo done
