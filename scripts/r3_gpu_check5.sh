#!/bin/bash
# Round-3 GPU check 5: bad-pixel probe, the round's profile of the headline
# bench command (trace + PMC passes), and a kernel trace of a 1-iteration render.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/vcm_census.py > gpurun_out/vcm_census.log 2>&1
rc=$?; echo "census rc=$rc"; [[ $rc == 0 || $rc == 1 ]] || exit $rc
timeout -k 10 500 python -u scripts/bad_pixels.py > gpurun_out/bad_pixels.log 2>&1
rc=$?; echo "bad_pixels rc=$rc"; [[ $rc == 0 || $rc == 1 ]] || exit $rc
bash scripts/profile_round.sh r3 --steps 20 --warmup 5
rc=$?; echo "profile rc=$rc"; [[ $rc == 0 ]] || exit $rc
mkdir -p gpurun_out/prof_r3_1it
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r3_1it -o run -- \
  python3 bench.py --steps 1 --warmup 2 --no-cpu --no-compare --no-count > gpurun_out/prof_r3_1it/bench.log 2>&1
echo "1it rc=$?"
echo done
