#!/bin/bash
# Grazing-guard threshold: probe mismatches (4 seeds x 3 scenes), the share of
# rays sent to the KD walk (bench count pass) and the rates, per library.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=winmad-s-raytracer-v1.0_amd/variants
for lib in ${LIBS:-product g6 g7}; do
  if [ $lib = product ]; then unset WR_LIB; else export WR_LIB=$V/$lib.so; fi
  for s in torus cbox torus1m; do
    timeout -k 10 300 python3 scripts/graze_mismatch.py $s 99 7 3 11 > gpurun_out/r4_g_${lib}_$s.out 2>&1; rc=$?
    echo "$lib $s rc=$rc $(grep -o '[0-9]* mismatches' gpurun_out/r4_g_${lib}_$s.out | tr '\n' ' ')"
    cp gpurun_out/graze_mm_$s.json gpurun_out/graze_mm_${lib}_$s.json 2>/dev/null
    [ $rc -eq 0 ] || exit $rc
  done
  for st in 20 1; do
    o=gpurun_out/r4_g_${lib}_b$st.out
    timeout -k 10 200 python3 bench.py --steps $st --warmup 3 --no-cpu --no-compare > $o 2>&1; rc=$?
    echo "$lib st=$st rc=$rc $(grep -o '"value": [0-9.]*' $o | head -1) $(grep -o '"fallback_frac": [0-9.e-]*' $o)"
    [ $rc -eq 0 ] || exit $rc
  done
done
