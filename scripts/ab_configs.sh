#!/bin/bash
# BVH-mode bench of every config for each library variant (VARIANTS, "default" =
# libwinmad_rt.so), then the C2 capacity probes: WR_BVH_DIAG=32 (k_fast_hard
# skipped) and 48 (k_fast_resolve too) -- wrong answers, measurement only.
set -o pipefail
for cfg in c2 vcm c4 c3; do
  STEPS=$([ $cfg = c4 ] && echo 32 || echo 64) BENCH_ARGS="--no-compare --no-count --trace bvh" \
    bash scripts/variant_bench.sh $cfg ${VARIANTS:-default} || exit 1
done
for dg in 32 48; do
  WR_BVH_DIAG=$dg timeout -k 10 200 python3 bench.py --steps 64 --no-cpu --no-compare --no-count > gpurun_out/diag$dg.json 2>/dev/null || exit 1
  echo "c2 diag $dg: $(python3 -c "import json; print(json.load(open('gpurun_out/diag$dg.json'))['value'])")"
done
