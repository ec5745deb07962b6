#!/bin/bash
# Round-3 GPU check 18: stability of the default bench after allocating the
# BVH scratch on every pipeline that fits (3 repeats per case)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
REPS=3 LIBS="product=" CASES="b1:--steps 1 --warmup 3|b20:--steps 20 --warmup 3|b256:--steps 256 --warmup 3" \
  timeout -k 10 900 bash scripts/ab_libs.sh || exit $?
echo done
