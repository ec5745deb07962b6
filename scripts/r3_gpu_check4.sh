#!/bin/bash
# Round-3 GPU check 4: VCM bisect, perturbation check, C2 bench at 20 / 1 / 256
# steps with the stagger + adaptive tie mode and without (A/B), C4 at 64.
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
B="python -u bench.py --no-cpu --no-compare --no-count"
step vcm_bisect 300 python -u scripts/vcm_bisect.py
step pert_check 900 bash scripts/perturbation_check.sh
step b20 200 $B --steps 20 --warmup 5
step b1 200 $B --steps 1 --warmup 2
step b20_nostag 200 env WR_STAGGER=0 $B --steps 20 --warmup 5
step b20_notie 200 env WR_TIE_WAVE_MAX=0 $B --steps 20 --warmup 5
step b1_notie 200 env WR_TIE_WAVE_MAX=0 $B --steps 1 --warmup 2
step b256 300 $B --steps 256
step b256_notie 300 env WR_TIE_WAVE_MAX=0 $B --steps 256
step c4_64 300 $B --config c4 --steps 64
step c4_64_notie 300 env WR_TIE_WAVE_MAX=0 $B --config c4 --steps 64
echo done
