#!/bin/bash
# Every bench configuration in both traversal modes (reference KD walk, verified
# BVH): one JSON line each under gpurun_out/modes_<cfg>_<mode>.json.
set -o pipefail
for cfg in ${CFGS:-c2 vcm c3 c4}; do
  for mode in reference bvh; do
    timeout -k 10 400 python3 -u bench.py --config $cfg --trace $mode --no-cpu ${STEPS:+--steps $STEPS} \
      > gpurun_out/modes_${cfg}_$mode.log 2>&1 || { echo "$cfg $mode failed rc=$?"; tail -5 gpurun_out/modes_${cfg}_$mode.log; exit 1; }
    tail -1 gpurun_out/modes_${cfg}_$mode.log > gpurun_out/modes_${cfg}_$mode.json
    echo "$cfg $mode: $(python3 -c "import json; d=json.load(open('gpurun_out/modes_${cfg}_$mode.json')); r=d['roofline']; print(d['value'], 'Mrays/s', round(r['frac'], 4), r.get('bvh'))")"
  done
done
