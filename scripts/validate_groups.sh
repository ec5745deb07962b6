#!/bin/bash
# GPU suite, BVH verification, and the one-iteration A/B of WR_PAIR_GROUPS --
# the four-near-ties-per-wave experiment (not kept: its change is
# profiles/r6/pair_groups/pair_groups.diff; the knob exists only with it applied).
mkdir -p gpurun_out/grp
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/grp/gpu_suite.txt 2>&1 || exit 1
timeout -k 10 240 python scripts/verify_bvh.py --configs c2,c2,vcm,c3,c4 --iters 1,32,16,16,4 > gpurun_out/grp/verify.log 2>&1 || exit 1
for rep in 1 2 3; do
  STEPS=1 BENCH_ARGS="--no-compare --no-count" bash scripts/env_bench.sh c2 WR_PAIR_GROUPS 0 1 || exit 1
done > gpurun_out/grp/ab.txt 2>&1
WR_TRACE_LOG=1 timeout -k 10 100 python scripts/hard_probe.py 1 0 > gpurun_out/grp/probe_1it.log 2>&1
