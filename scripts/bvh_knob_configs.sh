#!/bin/bash
# Other configurations under the old (16 bins, ct 0.5) and new (64, 1.0) BVH build defaults.
set -o pipefail
mkdir -p gpurun_out/r6
export GPU_MAX_HW_QUEUES=16
for rep in 1 2; do
for cfg in "c4:--config c4 --steps 16 --warmup 2" "c3:--config c3 --steps 16 --warmup 2" "vcm:--config vcm --steps 20 --warmup 3" "b1:--steps 1 --warmup 3"; do
  cn=${cfg%%:*}; args=${cfg#*:}
  for kv in "old=WR_BVH_BINS=16,WR_BVH_CT=0.5" "new=WR_BVH_BINS=64,WR_BVH_CT=1.0"; do
    n=${kv%%=*}; e=${kv#*=}
    out=gpurun_out/r6/kc_${cn}_${n}_r$rep.json
    env ${e//,/ } timeout -k 10 200 python3 -u bench.py $args --no-cpu --no-compare --no-count > $out 2>/dev/null || exit 1
    echo "$cn $n rep$rep $(python3 -c "import json;d=json.loads(open('$out').read().strip().splitlines()[-1]);print(d['value'])")"
  done
done
done
