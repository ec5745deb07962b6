#!/bin/bash
# Round-3 GPU check 8: kernel trace of a 1-iteration render, perturbation check, full -m gpu suite.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof_1it_b
export TMPDIR=/tmp
step() {  # name, timeout, command...: rc 0/1 go on, anything else stops
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [[ $rc != 0 && $rc != 1 ]]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
step prof1 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_1it_b -o run -- python3 bench.py --steps 1 --warmup 2 --no-cpu --no-compare --no-count
step perturb 1200 bash scripts/perturbation_check.sh
step gputest 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread
echo done
