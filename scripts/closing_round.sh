#!/bin/bash
# Closing evidence of the final build on one box: the GPU suite, smoke(), BVH
# verification, closing profiles of C2 and C4 (scripts/closing_profile.sh) and
# the bench lines (the driver's default command -- after the profiles' traffic
# files are in place, so that its line prices the PMC passes of this very
# library -- one iteration, C4 at 64).  Usage: scripts/closing_round.sh <tag>
set -o pipefail
TAG=${1:-r6h}
mkdir -p gpurun_out/$TAG
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/gpu_suite.txt 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || exit 1
timeout -k 10 240 python scripts/verify_bvh.py --configs c2,c2,vcm,c3,c4 --iters 1,32,16,16,4 > gpurun_out/$TAG/verify.log 2>&1 || exit 1
bash scripts/closing_profile.sh $TAG c2 c4 || exit 1
cp gpurun_out/prof_${TAG}_c2/sum/traffic_c2.json gpurun_out/prof_${TAG}_c4/sum/traffic_c4.json profiles/r6/
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/$TAG/bench_default.json 2> gpurun_out/$TAG/bench_default.err || exit 1
timeout -k 10 200 python bench.py --steps 1 --warmup 3 --no-cpu --no-compare > gpurun_out/$TAG/bench_1it.json 2> gpurun_out/$TAG/bench_1it.err || exit 1
timeout -k 10 200 python bench.py --config c4 --steps 64 --no-cpu --no-compare > gpurun_out/$TAG/bench_c4_64.json 2> gpurun_out/$TAG/bench_c4_64.err || exit 1
echo closing done
