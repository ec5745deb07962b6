#!/bin/bash
# A/B of library builds on one box: LIBS="name=path ..." (path empty = the product),
# CASES="name:bench args|..." ; each case runs every library before the next case.
# Lines to gpurun_out/ab_<case>_<lib>.json; prints a table.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=16
B="python -u bench.py --no-cpu --no-compare --no-count"
IFS='|' read -ra CS <<< "${CASES:-b1:--steps 1 --warmup 3|b20:--steps 20 --warmup 3|b256:--steps 256|c4:--config c4 --steps 64}"
for rep in $(seq 1 ${REPS:-1}); do
for cs in "${CS[@]}"; do
  name=${cs%%:*}; args=${cs#*:}
  for lb in ${LIBS:-product=}; do
    ln=${lb%%=*}; lp=${lb#*=}
    if [[ -n "$lp" ]]; then export WR_LIB=$lp; else unset WR_LIB; fi
    out=gpurun_out/ab_${name}_${ln}_r$rep.json
    timeout -k 10 240 $B $args > $out 2> ${out%.json}.err
    rc=$?
    echo "$name $ln rep$rep rc=$rc $(python3 -c "import json;print(json.loads(open('$out').read().strip().splitlines()[-1])['value'])" 2>/dev/null)"
    if [[ $rc != 0 ]]; then exit $rc; fi
  done
done
done
