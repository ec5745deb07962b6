#!/bin/bash
# Closing-build profiles of the driver's command (20 steps, 5 warm-up) for the
# given configs: kernel trace + PMC passes (scripts/profile_round.sh), then the
# roofline reproduced from the trace (scripts/trace_union.py).
# Usage (on the GPU box, repo root): scripts/closing_profile.sh <tag> c2 [c4 ...]
set -o pipefail
TAG=$1; shift
for cfg in "$@"; do
  bash scripts/profile_round.sh ${TAG}_$cfg --config $cfg --steps 20 --warmup 5 --no-cpu --no-compare || exit 1
  python3 scripts/summarize_profile.py gpurun_out/prof_${TAG}_$cfg gpurun_out/prof_${TAG}_$cfg/sum $cfg > /dev/null || exit 1
  python3 scripts/trace_union.py gpurun_out/prof_${TAG}_$cfg/trace gpurun_out/prof_${TAG}_$cfg/trace.log \
    --out gpurun_out/prof_${TAG}_$cfg/sum/trace_union_$cfg.json > /dev/null || exit 1
  echo "$cfg done"
done
