#!/bin/bash
# Round-3 GPU check 27: VCM per-path state in the records (A/B vs variants/novcm.so),
# vertex-kernel grid 1 vs 2 blocks per CU (WR_SHADE_GRID) on every config; VCM tests
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_vcm.py tests/test_gpu_bvh.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/vcmtest27.log 2>&1
rc=$?; echo "vcmtest27 rc=$rc"; tail -1 gpurun_out/vcmtest27.log
[[ $rc == 0 ]] || exit $rc
REPS=2 LIBS="novcm=winmad-s-raytracer-v1.0_amd/variants/novcm.so vcmrec=" CASES="vcm:--config vcm --steps 64 --warmup 3" \
  timeout -k 10 600 bash scripts/ab_libs.sh || exit $?
step() {  # name, timeout, command...: rc 0/1 go on, anything else stops
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep '^{' gpurun_out/$name.log 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])' 2>/dev/null)"
  if [[ $rc != 0 && $rc != 1 ]]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
B="python3 bench.py --no-cpu --no-compare --no-count"
for rep in 1 2; do
for cfg in "s20:--steps 20 --warmup 3" "s256:--steps 256 --warmup 3" "c4:--config c4 --steps 64 --warmup 2" "vcm:--config vcm --steps 64 --warmup 3" "c3:--config c3 --steps 64 --warmup 3"; do
  n=${cfg%%:*}; a=${cfg#*:}
  step g2_${n}_r$rep 300 env WR_SHADE_GRID=2 $B $a
  step g1_${n}_r$rep 300 env WR_SHADE_GRID=1 $B $a
done
done
echo done
