#!/bin/bash
# Round-3 GPU check 21: the full -m gpu suite on the current tree, smoke, the driver's bench command
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, timeout, command...: rc 0/1 go on, anything else stops
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [[ $rc != 0 && $rc != 1 ]]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
step gputest21 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread
step smoke21 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench21 300 python3 bench.py --steps 20 --warmup 5
echo done
