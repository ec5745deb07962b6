#!/bin/bash
# GPU suite + BVH verification of the in-tree library, then an A/B against a
# variant build: scripts/validate_variant.sh <tag> <variant .so>
TAG=$1; VAR=$2
mkdir -p gpurun_out/$TAG
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/gpu_suite.txt 2>&1 || exit 1
timeout -k 10 240 python scripts/verify_bvh.py --configs c2,c2,vcm,c3,c4 --iters 1,32,16,16,4 > gpurun_out/$TAG/verify.log 2>&1 || exit 1
LIBS="old=$VAR new=" CASES="b1:--steps 1 --warmup 3|b20:--steps 20 --warmup 3|c4:--config c4 --steps 64" REPS=2 bash scripts/ab_libs.sh > gpurun_out/$TAG/ab.txt 2>&1
