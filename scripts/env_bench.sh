#!/bin/bash
# bench.py --config CFG under each VAR=value setting (A/B of run-time knobs).
# Usage: scripts/env_bench.sh CFG VAR v1 v2 ...   ("-" = unset); extra bench.py arguments in $BENCH_ARGS
set -o pipefail
cfg=$1; var=$2; shift 2
for v in "$@"; do
  if [ "$v" = "-" ]; then envset=""; else envset="$var=$v"; fi
  env $envset timeout -k 10 300 python3 bench.py --config $cfg --steps ${STEPS:-48} --warmup 2 --no-cpu $BENCH_ARGS > gpurun_out/env_${cfg}_$v.log 2>&1 \
    || { echo "$v failed"; tail -3 gpurun_out/env_${cfg}_$v.log; exit 1; }
  echo "$cfg $var=$v: $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/env_${cfg}_$v.log') if l.startswith('{')][-1]); print(d['value'], 'Mrays/s')")"
done
