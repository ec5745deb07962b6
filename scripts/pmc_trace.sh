#!/bin/bash
# Focused PMC passes on one kernel family (one counter group per run,
# --kernel-trace only).  Usage: scripts/pmc_trace.sh <tag> [kernel regex] [bench config]
# (defaults: k_trace, c2; run with WR_PIPES=1 for a serial profile; extra bench
# arguments in $BENCH_ARGS, e.g. "--trace bvh")
set -o pipefail
TAG=${1:-x}
KRE=${2:-k_trace}
CFG=${3:-c2}
export TMPDIR=/tmp
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_MISC TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
           "TA_BUSY_avr TD_BUSY_avr TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "$KRE" --output-format csv -d $OUT/p$i -o run -- python3 bench.py --config $CFG --steps 2 --warmup 0 --no-cpu --no-count $BENCH_ARGS > $OUT/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc pass $i failed rc=$rc"; tail -5 $OUT/p$i.log; fi
  if [ $rc -ge 124 ]; then exit 1; fi
done
echo done
