#!/bin/bash
# Round-4 session 3: the grazing probe after the search-side guard, the BVH
# test file, and the overlapped / sequential / separate-queue A/B.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r4_$n.out 2> gpurun_out/r4_$n.err
  local rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r4_$n.out | head -1) $(tail -c 200 gpurun_out/r4_$n.out | tr '\n' ' ' | cut -c1-160)"
  [ $rc -eq 0 ] || exit $rc
}
for s in torus cbox torus1m; do run graze_$s 300 python3 scripts/graze_mismatch.py $s 99 7; done
run bvh 600 python -u -m pytest tests/test_gpu_bvh.py -x -q --timeout 300 --timeout-method thread
B="python3 bench.py --warmup 3 --no-cpu --no-count --no-compare"
for st in 20 1; do
  run ov_$st 150 $B --steps $st
  WR_BDPT_OVERLAP=0 run seq_$st 150 $B --steps $st
  WR_LIB=winmad-s-raytracer-v1.0_amd/variants/ov6.so run ov6_$st 150 $B --steps $st
done
