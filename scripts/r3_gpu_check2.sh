#!/bin/bash
# Round-3 GPU check 2: full -m gpu suite (new gates, two-rank test), parity
# statistics with the gates' verdicts, the perturbation check, a C5 rank shard.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread \
  > gpurun_out/gputest.log 2>&1 || echo "gpu tests failed: rc=$?"
timeout -k 10 600 python -u scripts/parity_stats.py --out gpurun_out/parity_stats2.jsonl > gpurun_out/parity2.log 2>&1
bash scripts/perturbation_check.sh || echo "perturbation check rc=$?"
timeout -k 10 400 python -u bench.py --config c4 --steps 512 --iter-begin 512 --no-compare --no-cpu \
  > gpurun_out/bench_c5_shard.json 2> gpurun_out/bench_c5_shard.err
echo done
