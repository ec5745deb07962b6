#!/bin/bash
# Round-3 BVH verification on the full bench workloads (WR_BVH_VERIFY: every
# ray's answer compared with the KD walk's, bit for bit)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python3 scripts/verify_bvh.py --configs c2,vcm,c3,c4 --iters 256,64,64,16 --out gpurun_out/verify_full.json > gpurun_out/verify_full.log 2>&1
echo "verify rc=$?"
