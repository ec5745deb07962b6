#!/bin/bash
# bench.py --config CFG with each library variant (WR_LIB) and the default build.
# Usage: scripts/variant_bench.sh CFG name1 name2 ...   ("default" = libwinmad_rt.so)
# Extra bench.py arguments in $BENCH_ARGS (e.g. "--trace bvh").
set -o pipefail
cfg=$1; shift
for v in "$@"; do
  lib=""; [ "$v" != default ] && lib=winmad-s-raytracer-v1.0_amd/variants/$v.so
  WR_LIB=$lib timeout -k 10 300 python3 bench.py --config $cfg --steps ${STEPS:-32} --warmup 2 --no-cpu $BENCH_ARGS \
    > gpurun_out/var_${cfg}_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/var_${cfg}_$v.log; exit 1; }
  echo "$cfg $v: $(python3 -c "import json; d=json.loads(open('gpurun_out/var_${cfg}_$v.log').read().strip().splitlines()[-1]); r=d['roofline'] or {}; print(d['value'], 'Mrays/s', r.get('tests_per_ray'), 'tests/ray', r.get('bvh'))")"
done
