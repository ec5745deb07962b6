#!/bin/bash
# Round-4 session: the one-ray-per-wave KD walk (kd_walk_wave) -- its parity
# tests, A/B against the serial walk at 1 and 20 iterations, and a 1-iteration
# kernel timeline with the latency tails (WR_TRACE_LOG).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r4_$n.out 2> gpurun_out/r4_$n.err
  local rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r4_$n.out | head -1) $(tail -c 200 gpurun_out/r4_$n.out | tr '\n' ' ')"
  [ $rc -eq 0 ] || exit $rc
}
step wtests 400 python -u -m pytest tests/test_gpu_bvh.py -x -q --timeout 300 --timeout-method thread -k "wave or grazing or corpus"
B="python3 bench.py --warmup 3 --no-cpu --no-compare --no-count"
for r in 1 2; do
  for w in 1 0; do
    WR_WALK_WAVE=$w step ww${w}_b1_r$r 120 $B --steps 1
  done
done
for w in 1 0; do
  WR_WALK_WAVE=$w step ww${w}_b20 200 $B --steps 20
done
WR_TRACE_LOG=1 step log_b1 200 python3 bench.py --warmup 1 --steps 1 --no-cpu --no-compare
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_ww -o run -- \
  python3 bench.py --steps 1 --warmup 3 --no-cpu --no-count --no-compare > gpurun_out/r4_tl_ww.out 2>&1
echo "tl_ww rc=$?"
