#!/bin/bash
# C2 (or $CONFIG) at the driver's 20 iterations ($STEPS) under library knobs, one bench run each
# (usage: bash scripts/knob_sweep_c2.sh "name:ENV=V ..." ...; no args: the default set)
set -o pipefail
B="timeout -k 10 150 python -u bench.py --config ${CONFIG:-c2} --steps ${STEPS:-20} --no-cpu --no-compare --no-count"
cfgs=("$@")
[ ${#cfgs[@]} -eq 0 ] && cfgs=("base:" "notime:WR_TIME_KERNELS=0" "cap1M:WR_PIECE_CAP=1048576" "cap1.4M:WR_PIECE_CAP=1400000" "pipes12:WR_PIPES=12" "base2:" "notime2:WR_TIME_KERNELS=0")
mkdir -p gpurun_out/r5
for cfg in "${cfgs[@]}"; do
  name=${cfg%%:*}; kv=${cfg#*:}
  env $kv $B > gpurun_out/r5/knob_$name.log 2>&1 || exit $?
  echo "$name $(tail -1 gpurun_out/r5/knob_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["pipelines"])')"
done
