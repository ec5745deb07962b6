#!/bin/bash
# Interleaved A/B (REPS rounds of every library / mode) at 20 and 1 iterations,
# plus 1-iteration kernel timelines of the current overlapped schedule and of
# the separate-queue variant.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --warmup 3 --no-cpu --no-count --no-compare"
V=winmad-s-raytracer-v1.0_amd/variants
for rep in $(seq 1 ${REPS:-3}); do
  for st in ${STEPS:-20 1}; do
    for cfg in ${CFGS:-ov seq ov6}; do
      case $cfg in
        ov) e="WR_BDPT_OVERLAP=1" ;;
        seq) e="WR_BDPT_OVERLAP=0" ;;
        *) e="WR_LIB=$V/$cfg.so" ;;
      esac
      o=gpurun_out/r4_ab_${cfg}_${st}_r$rep.out
      env $e timeout -k 10 150 $B --steps $st > $o 2> ${o%.out}.err; rc=$?
      echo "$cfg st=$st rep=$rep rc=$rc $(grep -o '"value": [0-9.]*' $o | head -1)"
      [ $rc -eq 0 ] || exit $rc
    done
  done
done
if [ "${TL:-1}" = 1 ]; then
  for cfg in ov ov6; do
    case $cfg in ov) e="WR_BDPT_OVERLAP=1" ;; *) e="WR_LIB=$V/$cfg.so" ;; esac
    env $e timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl2_$cfg -o run -- \
      python3 bench.py --steps 1 --warmup 3 --no-cpu --no-count --no-compare > gpurun_out/r4_tl2_$cfg.out 2>&1
    rc=$?; echo "tl2_$cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
fi
