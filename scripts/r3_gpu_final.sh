#!/bin/bash
# Round-3 final measurements: smoke, the default bench command under rocprofv3
# (kernel trace + stats) and its PMC passes, the other configurations' lines.
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
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step prof 900 bash scripts/profile_round.sh r3 --steps 20 --warmup 5
step vcm 400 python3 bench.py --config vcm --steps 64 --warmup 3 --no-cpu
step c3 400 python3 bench.py --config c3 --steps 64 --warmup 3 --no-cpu
echo done
