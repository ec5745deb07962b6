#!/bin/bash
# GPU suite, BVH verification and the WR_PAIR_RECORD A/B (1 = pair record in the
# tie list only, 2 = + the pair list outside latency-bound renders) on one box.
mkdir -p gpurun_out/plist
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/plist/gpu_suite.txt 2>&1 || exit 1
timeout -k 10 240 python scripts/verify_bvh.py --configs c2,c2,vcm,c3,c4 --iters 1,32,16,16,4 > gpurun_out/plist/verify.log 2>&1 || exit 1
for rep in 1 2; do
  STEPS=20 BENCH_ARGS="--no-compare --no-count" bash scripts/env_bench.sh c2 WR_PAIR_RECORD 1 2 || exit 1
  STEPS=1 BENCH_ARGS="--no-compare --no-count" bash scripts/env_bench.sh c2 WR_PAIR_RECORD 1 2 || exit 1
  STEPS=64 BENCH_ARGS="--no-compare --no-count" bash scripts/env_bench.sh c4 WR_PAIR_RECORD 1 2 || exit 1
  STEPS=16 BENCH_ARGS="--no-compare --no-count" bash scripts/env_bench.sh vcm WR_PAIR_RECORD 1 2 || exit 1
done > gpurun_out/plist/ab.txt 2>&1
