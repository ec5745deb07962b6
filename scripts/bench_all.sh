#!/bin/bash
# All bench configurations (one JSON line each) + the kernel-trace summary of
# the VCM bench; outputs under gpurun_out/ (copied into profiles/<round>/).
set -o pipefail
for cfg in ${@:-c2 vcm c3 c4}; do
  timeout -k 10 400 python3 -u bench.py --config $cfg > gpurun_out/bench_$cfg.log 2>&1 \
    || { echo "bench $cfg failed rc=$?"; tail -5 gpurun_out/bench_$cfg.log; exit 1; }
  tail -1 gpurun_out/bench_$cfg.log > gpurun_out/bench_$cfg.json
  echo "$cfg: $(python3 -c "import json; d=json.load(open('gpurun_out/bench_$cfg.json')); print(d['value'], d['unit'], 'cpu', d['cpu_baseline']['value'], d['cpu_baseline']['kind'], d['cpu_baseline'].get('film_bit_exact'))")"
done
