#!/bin/bash
# Serial (one pipeline) kernel-trace A/B of the two traversal modes on one
# config: rocprofv3 --stats per mode under gpurun_out/ab_<mode>/.
# Usage: scripts/ab_trace.sh [config] [steps]
set -o pipefail
CFG=${1:-c2}; K=${2:-4}
export TMPDIR=/tmp
for mode in reference bvh; do
  OUT=gpurun_out/ab_$mode
  mkdir -p $OUT
  WR_PIPES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
    python3 bench.py --config $CFG --trace $mode --steps $K --warmup 1 --no-cpu --no-count > $OUT/bench.log 2>&1 \
    || { echo "$mode failed rc=$?"; tail -5 $OUT/bench.log; exit 1; }
  echo "== $mode: $(tail -1 $OUT/bench.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["unit"])')"
  python3 - $OUT <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print(f'{r["Name"][:60]:60s} calls={r["Calls"]:>6s} avg_us={float(r["AverageNs"])/1e3:9.1f} tot_ms={float(r["TotalDurationNs"])/1e6:9.2f}')
PY
done
