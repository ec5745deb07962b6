#!/bin/bash
# Round-3 closing measurements on the final build: smoke, the default bench
# command under rocprofv3 (kernel trace + stats) and its PMC passes, the other
# configurations' lines, the drop-in CLI, and the full-workload BVH verification.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final
export TMPDIR=/tmp
step() {  # name, timeout, command...: rc 0 goes on, anything else stops
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/final/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(tail -c 300 gpurun_out/final/$name.log | tail -1 | cut -c1-160)"
  if [[ $rc != 0 ]]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step prof 900 bash scripts/profile_round.sh r3 --steps 20 --warmup 5
export GPU_MAX_HW_QUEUES=16
step c2_s256 300 python3 bench.py --steps 256 --warmup 5 --no-cpu
step c4_s64 300 python3 bench.py --config c4 --steps 64 --warmup 2 --no-cpu
step vcm_s64 300 python3 bench.py --config vcm --steps 64 --warmup 3 --no-cpu
step c3_s64 300 python3 bench.py --config c3 --steps 64 --warmup 3 --no-cpu
step c2_4k_s16 300 python3 bench.py --width 3840 --height 2160 --steps 16 --warmup 2 --no-cpu --no-compare
step c5_shard 400 python3 bench.py --config c4 --steps 512 --warmup 3 --iter-begin 512 --no-cpu --no-compare
step c2_s1 200 python3 bench.py --steps 1 --warmup 3 --no-cpu --no-compare
unset GPU_MAX_HW_QUEUES
step wr_tot 400 python3 scripts/wr_tot_profile.py 20 256
step verify 600 python3 scripts/verify_bvh.py --out gpurun_out/final/bvh_verify.json
echo done
