#!/bin/bash
# C2 (20 iterations) under BVH build knobs (env, read by wr_create's build).
set -o pipefail
mkdir -p gpurun_out/r6
export GPU_MAX_HW_QUEUES=16
for rep in 1 2 3; do
for kv in ${KNOBS:-"default=" "sweep64=WR_BVH_SWEEP=64" "sweep256=WR_BVH_SWEEP=256" "bins64=WR_BVH_BINS=64" "ct03=WR_BVH_CT=0.3" "ct1=WR_BVH_CT=1.0"}; do
  n=${kv%%=*}; e=${kv#*=}
  out=gpurun_out/r6/knob_${n}_r$rep.json
  env ${e//,/ } timeout -k 10 120 python3 -u bench.py --steps 20 --warmup 5 --no-cpu --no-compare > $out 2>/dev/null || exit 1
  echo "$n rep$rep $(python3 -c "import json;d=json.loads(open('$out').read().strip().splitlines()[-1]);r=d['roofline']['bvh'];print(d['value'], r['nodes_per_ray'], r['tests_per_ray'])")"
done
done
