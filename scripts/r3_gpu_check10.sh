#!/bin/bash
# Round-3 GPU check 10: per-queue kernel chain of 1- and 20-iteration renders
# (rocprofv3 kernel trace), wr_tot throughput at 1080p, a 4K BDPT bench line.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/p1 gpurun_out/p20
export TMPDIR=/tmp
step() {  # name, timeout, command...: rc 0/1 go on, anything else stops
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [[ $rc != 0 && $rc != 1 ]]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
step prof1 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/p1 -o run -- python3 bench.py --steps 1 --warmup 2 --no-cpu --no-compare --no-count
step prof20 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/p20 -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-compare --no-count
step wrtot 400 python3 scripts/wr_tot_profile.py 20 256
step bench4k 400 python3 bench.py --width 3840 --height 2160 --steps 16 --warmup 2 --no-cpu --no-compare
echo done
