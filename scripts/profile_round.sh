#!/bin/bash
# Profiling passes on the GPU box (run from the repo root via gpurun).
# 1) kernel trace + stats for the bench command, 2) PMC passes (one counter
# group per run, --kernel-trace only: no sys/runtime trace with --pmc).
# Usage: scripts/profile_round.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r1}; shift
# trace pass: the default bench command itself (so that rocprof's average
# k_trace duration is comparable with the line's roofline.avg_launch_ms: with
# 16 overlapping pipelines a launch's duration depends on the run's length)
ARGS=${@:-}
# the PMC passes take the config / trace / steps arguments of the trace pass, so
# that their per-dispatch means describe the same launch mix
PMC_ARGS=$(echo " $ARGS " | grep -oE -- "--(config|trace|steps) [a-z0-9]+" | tr "\n" " ")
[[ "$PMC_ARGS" == *--steps* ]] || PMC_ARGS="$PMC_ARGS --steps 2"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
# the library these counters describe (bench.py compares it with the one it loads)
sha256sum winmad-s-raytracer-v1.0_amd/libwinmad_rt.so | cut -c1-16 > $OUT/lib.sha
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || { echo "trace pass failed rc=$?"; tail -5 $OUT/trace.log; exit 1; }
echo "trace pass ok"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS TCC_HIT_sum TCC_MISS_sum" \
           "FETCH_SIZE" "WRITE_SIZE" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_BUSY_avr"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- python3 bench.py $PMC_ARGS --warmup 0 --no-cpu --no-count --no-compare > $OUT/pmc$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc pass $i failed rc=$rc"; tail -5 $OUT/pmc$i.log; fi
  if [ $rc -ge 124 ]; then exit 1; fi  # timeout / abort / segfault: stop using the GPU
done
echo done
