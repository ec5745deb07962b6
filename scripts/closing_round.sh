#!/bin/bash
# Closing evidence of the final build on one box: closing profiles of C2 and C4
# (scripts/closing_profile.sh) and the driver's default bench command.
set -o pipefail
bash scripts/closing_profile.sh r6f c2 c4 || exit 1
mkdir -p gpurun_out/r6f
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r6f/bench_default.json 2> gpurun_out/r6f/bench_default.err || exit 1
timeout -k 10 200 python bench.py --steps 1 --warmup 3 --no-cpu --no-compare > gpurun_out/r6f/bench_1it.json 2> gpurun_out/r6f/bench_1it.err || exit 1
timeout -k 10 200 python bench.py --config c4 --steps 64 --no-cpu --no-compare > gpurun_out/r6f/bench_c4_64.json 2> gpurun_out/r6f/bench_c4_64.err || exit 1
echo closing done
