#!/bin/bash
# Round-3 GPU check 25: the records build -- full -m gpu suite, smoke, the
# driver's bench command, then the profile passes (kernel trace + PMC) of it
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
step gputest25 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread
step smoke25 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench25 300 python3 bench.py --steps 20 --warmup 5
step prof25 900 bash scripts/profile_round.sh r3 --steps 20 --warmup 5
step c4_25 400 python3 bench.py --config c4 --steps 64 --warmup 2 --no-cpu
step vcm25 400 python3 bench.py --config vcm --steps 64 --warmup 3 --no-cpu
step c3_25 400 python3 bench.py --config c3 --steps 64 --warmup 3 --no-cpu
step b256_25 400 python3 bench.py --steps 256 --warmup 5 --no-cpu
echo done
