#!/bin/bash
# Round-4 diagnostics: grazing-probe mismatches, and 1-iteration kernel
# timelines of the sequential and overlapped schedules (and a variant library).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/graze_mismatch.py torus 99 7 > gpurun_out/r4_graze.out 2>&1; rc=$?
echo "graze rc=$rc $(tail -2 gpurun_out/r4_graze.out | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
tl() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_$n -o run -- \
    python3 bench.py --steps ${TLSTEPS:-1} --warmup 3 --no-cpu --no-count --no-compare > gpurun_out/r4_tl_$n.out 2>&1
  local rc=$?; echo "tl_$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r4_tl_$n.out)"; [ $rc -eq 0 ] || exit $rc
}
tl seq WR_BDPT_OVERLAP=0
tl ov WR_BDPT_OVERLAP=1
tl ov6 WR_LIB=winmad-s-raytracer-v1.0_amd/variants/ov6.so
