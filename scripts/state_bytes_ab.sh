#!/bin/bash
# HBM bytes of the path-state kernels per traversal step for library builds
# side by side: FETCH_SIZE and WRITE_SIZE passes of the same bench command
# (C2, 20 iterations) per library.  Usage: LIBS="name=path ..." scripts/state_bytes_ab.sh
set -o pipefail
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16
for lb in ${LIBS:-product=}; do
  ln=${lb%%=*}; lp=${lb#*=}
  if [[ -n "$lp" ]]; then export WR_LIB=$lp; else unset WR_LIB; fi
  OUT=gpurun_out/sb_$ln
  mkdir -p $OUT
  i=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- python3 bench.py --steps 20 --warmup 0 --no-cpu --no-count --no-compare > $OUT/pmc$i.log 2>&1 || { echo "pmc pass failed ($ln $grp)"; exit 1; }
  done
  python3 scripts/summarize_profile.py $OUT $OUT/sum c2 > /dev/null && python3 -c "
import json; t=json.load(open('$OUT/sum/traffic_c2.json'))
print('$ln', 'trace', round(t['hbm_bytes_per_launch']/1e6,1), 'state', round(t['state_bytes_per_launch']/1e6,1), {k:round(v['bytes_per_step']/1e6,1) for k,v in t['state_kernels'].items() if k.startswith('k_')})"
done
