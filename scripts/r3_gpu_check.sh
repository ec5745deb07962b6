#!/bin/bash
# Round-3 GPU check: -m gpu suite, parity statistics, 20- and 256-step C2 bench.
# Every GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
what="${1:-all}"
if [[ "$what" == all || "$what" == tests ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/gputest.log 2>&1
fi
if [[ "$what" == all || "$what" == parity ]]; then
  timeout -k 10 600 python -u scripts/parity_stats.py --out gpurun_out/parity_stats.jsonl > gpurun_out/parity.log 2>&1
fi
if [[ "$what" == all || "$what" == bench ]]; then
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-compare > gpurun_out/bench20.json 2> gpurun_out/bench20.err
  timeout -k 10 300 python -u bench.py --steps 1 --warmup 2 --no-cpu --no-compare > gpurun_out/bench1.json 2> gpurun_out/bench1.err
  timeout -k 10 300 python -u bench.py --steps 256 --no-cpu --no-compare > gpurun_out/bench256.json 2> gpurun_out/bench256.err
fi
echo done
