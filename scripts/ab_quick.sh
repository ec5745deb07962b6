#!/bin/bash
# Quick A/B: BVH verify (c2 8 it., c3 4 spp, c4 2 it.) of the default build, then
# bench of each variant (VARIANTS, "default" = libwinmad_rt.so) on CONFIGS.
set -o pipefail
timeout -k 10 300 python3 scripts/verify_bvh.py --configs ${VCONFIGS:-c2,c3,c4} --iters ${VITERS:-8,4,2} > gpurun_out/ver_default.log 2>&1 || { echo "verify failed"; tail -3 gpurun_out/ver_default.log; exit 1; }
echo "verify: $(grep -o '"mismatches": [0-9]*' gpurun_out/ver_default.log | tr '\n' ' ')"
for cfg in ${CONFIGS:-c2 vcm c4}; do
  STEPS=$([ $cfg = c4 ] && echo 32 || echo 64) BENCH_ARGS="--no-compare --no-count --trace bvh" \
    bash scripts/variant_bench.sh $cfg ${VARIANTS:-default} || exit 1
done
