#!/bin/bash
# VCM merge-grid cell size sweep (WR_VCM_CELL = cell edge / query half-width)
# on the torus 1080p VCM bench; one bench line per setting.
set -o pipefail
for k in ${@:-2 1 0.75 0.5}; do
  WR_VCM_CELL=$k timeout -k 10 200 python3 bench.py --config vcm --steps 16 --warmup 2 --no-cpu --no-count \
    > gpurun_out/vcm_cell_$k.log 2>&1 || { echo "cell $k failed"; tail -3 gpurun_out/vcm_cell_$k.log; exit 1; }
  echo "cell $k: $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/vcm_cell_$k.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
