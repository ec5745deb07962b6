#!/bin/bash
# Serial per-kernel breakdown (one pipeline: launches do not overlap) of the
# VCM and BDPT torus 1080p benches: rocprofv3 kernel stats per run.
set -o pipefail
export TMPDIR=/tmp
for cfg in ${@:-vcm c2}; do
  WR_PIPES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/brk_$cfg -o run -- \
    python3 bench.py --config $cfg --steps 4 --warmup 1 --no-cpu --no-count > gpurun_out/brk_$cfg.log 2>&1 \
    || { echo "$cfg failed"; tail -3 gpurun_out/brk_$cfg.log; exit 1; }
  python3 - "$cfg" <<'PY'
import csv, sys
cfg = sys.argv[1]
rows = list(csv.DictReader(open(f"gpurun_out/brk_{cfg}/run_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"== {cfg}: {tot / 1e6:.2f} ms total kernel time (5 iterations)")
for r in rows[:10]:
    print(f"  {r['Name'].split('(')[0][-40:]:40s} calls {r['Calls']:>4s}  {float(r['TotalDurationNs']) / 1e6:8.2f} ms  {float(r['Percentage']):5.1f}%")
PY
done
