#!/bin/bash
# Pipeline count in BVH mode (16 default / 20 / 24 with matching hardware queues).
# Usage: scripts/pipes_bvh.sh "c4 c2"
set -o pipefail
mkdir -p gpurun_out
for cfg in ${1:-c4 c2}; do
  st=$([ $cfg = c4 ] && echo 32 || echo 64)
  for v in 16 20 24; do
    lib=""; [ $v != 16 ] && lib=winmad-s-raytracer-v1.0_amd/variants/p$v.so
    GPU_MAX_HW_QUEUES=$v WR_LIB=$lib timeout -k 10 300 python3 bench.py --config $cfg --steps $st --warmup 2 --no-cpu \
      --no-count --no-compare --trace bvh > gpurun_out/pb_${cfg}_$v.log 2>&1 || { echo "$cfg $v failed"; tail -3 gpurun_out/pb_${cfg}_$v.log; exit 1; }
    echo "$cfg pipes=$v $(tail -1 gpurun_out/pb_${cfg}_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["hw_queues"])')"
  done
done
