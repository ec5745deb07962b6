#!/bin/bash
# One-iteration render: rocprofv3 kernel trace -> per-queue timeline (kernel
# durations vs idle gaps on the critical chain).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tl1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl1/trace -o run -- python3 bench.py --steps 1 --warmup 3 --no-cpu --no-compare --no-count > gpurun_out/tl1/bench.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -c 400 gpurun_out/tl1/bench.log; if [[ $rc != 0 ]]; then exit $rc; fi
f=$(find gpurun_out/tl1/trace -name '*kernel_trace.csv' | head -1)
python3 scripts/timeline.py "$f" > gpurun_out/tl1/timeline.txt 2>&1; echo "timeline rc=$?"
head -80 gpurun_out/tl1/timeline.txt
