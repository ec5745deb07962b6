#!/bin/bash
# k_fast_resolve loads the ray and the winner records for hits only: GPU suite, BVH verification
# on C2, then A/B against the previous build (variants/base.so).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [[ $rc != 0 ]]; then exit $rc; fi
LIBS="new= base=winmad-s-raytracer-v1.0_amd/variants/base.so" REPS=2 \
CASES="b20:--steps 20 --warmup 3|b256:--steps 256|c4:--config c4 --steps 64|vcm:--config vcm --steps 64" \
  bash scripts/ab_libs.sh
