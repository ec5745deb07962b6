#!/bin/bash
# Round-3 GPU check 24: per-primitive records for the hit rebuild -- full -m gpu
# suite, then A/B against the build without them (variants/rec.so)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 400 --timeout-method thread > gpurun_out/gputest24.log 2>&1
rc=$?; echo "gputest24 rc=$rc"; tail -2 gpurun_out/gputest24.log
[[ $rc == 0 ]] || exit $rc
REPS=2 LIBS="rec=winmad-s-raytracer-v1.0_amd/variants/rec.so prim=" \
CASES="b20:--steps 20 --warmup 3|b256:--steps 256 --warmup 3|c4:--config c4 --steps 64 --warmup 2|vcm:--config vcm --steps 64 --warmup 3|c3:--config c3 --steps 64 --warmup 3" \
  timeout -k 10 1000 bash scripts/ab_libs.sh
echo done
