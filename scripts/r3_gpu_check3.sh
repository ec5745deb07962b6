#!/bin/bash
# Round-3 GPU check 3: the new API tests, the whole -m gpu suite, VCM and
# perturbation probes, the perturbation check.  Stops at the first GPU step
# that crashes or times out.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, timeout, command...: test failures (rc 1) go on, anything else stops
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [[ $rc != 0 && $rc != 1 ]]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
step api 400 python -u -m pytest tests/test_gpu_api.py -m gpu -v --timeout 300 --timeout-method thread
step gputest 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread
step vcm_probe 300 python -u scripts/vcm_probe.py
step pert_probe 300 python -u scripts/perturbation_probe.py
step pert_check 600 bash scripts/perturbation_check.sh
echo done
