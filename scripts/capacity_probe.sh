#!/bin/bash
# Where the BVH mode's capacity goes: bench with k_fast_hard skipped
# (WR_BVH_DIAG=32) and with k_fast_resolve too (48) -- wrong answers,
# measurement only -- beside the real run.  Usage: scripts/capacity_probe.sh [cfg] [steps]
set -o pipefail
cfg=${1:-c2}; K=${2:-64}
for dg in ${DIAGS:-0 32 48}; do
  WR_BVH_DIAG=$dg timeout -k 10 300 python3 bench.py --config $cfg --trace bvh --steps $K --no-cpu --no-compare --no-count \
    > gpurun_out/cap_${cfg}_$dg.json 2>/dev/null || exit 1
  echo "$cfg diag $dg: $(python3 -c "import json; print(json.load(open('gpurun_out/cap_${cfg}_$dg.json'))['value'])")"
done
