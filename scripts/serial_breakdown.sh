#!/bin/bash
# One-pipeline kernel-time breakdown (no overlap between streams) of one bench
# configuration: rocprofv3 --kernel-trace --stats, summed per kernel.
# Usage: scripts/serial_breakdown.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/serial_$TAG
mkdir -p $OUT
WR_PIPES=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 bench.py --no-cpu --no-count --no-compare --warmup 1 "$@" > $OUT/bench.log 2>&1 || { echo "failed rc=$?"; tail -5 $OUT/bench.log; exit 1; }
python3 - $OUT <<'PY'
import csv, glob, json, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "<true" not in r["Name"]]
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:10]:
    n = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:40]
    print(f'{n:40s} calls={r["Calls"]:>6s} avg_us={float(r["AverageNs"])/1e3:8.1f} tot_ms={float(r["TotalDurationNs"])/1e6:8.1f} {100*float(r["TotalDurationNs"])/tot:5.1f}%')
line = [l for l in open(sys.argv[1] + "/bench.log") if l.startswith('{"metric"')][-1]
print("bench (1 pipeline):", json.loads(line)["value"], "Mrays/s")
PY
