#!/bin/bash
# Round-3 GPU check 7: step-interleaved issue -- timelines, benches, full -m gpu suite.
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
rm -f gpurun_out/tl1.csv gpurun_out/tl20.csv
step tl1 150 python -u scripts/timeline_events.py 1 gpurun_out/tl1.csv
step tl20 150 python -u scripts/timeline_events.py 20 gpurun_out/tl20.csv
B="python -u bench.py --no-cpu --no-compare --no-count"
step i_b1 200 $B --steps 1 --warmup 2
step i_b20 200 $B --steps 20 --warmup 5
step i_b256 300 $B --steps 256
step i_c4 300 $B --config c4 --steps 64
step gputest 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread
echo done
