#!/bin/bash
# Round-4 GPU session: focused parity tests, the overlapped-schedule A/B, BVH
# width / speculation variants, then the whole -m gpu suite.  Every GPU step
# has its own time limit; the script stops at the first failure.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r4_$n.out 2> gpurun_out/r4_$n.err
  local rc=$?
  echo "$n rc=$rc $(tail -c 300 gpurun_out/r4_$n.out | tr '\n' ' ' | cut -c1-200)"
  [ $rc -eq 0 ] || exit $rc
}
B="python3 bench.py --warmup 3 --no-cpu --no-count"
if [ "${FOCUS:-1}" = 1 ]; then
  run focus 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread \
      -k "overlapped or never_exceed or pieces_render"
fi
for st in ${STEPS:-20 1 256}; do
  run ov_$st 150 $B --steps $st
  WR_BDPT_OVERLAP=0 run seq_$st 150 $B --steps $st
done
for v in ${VARIANTS:-}; do
  WR_LIB=winmad-s-raytracer-v1.0_amd/variants/$v.so run var_${v}_20 150 $B --steps 20
done
if [ "${EM:-0}" = 1 ]; then  # INTEGRATION.md 1's main() (example_main) alone at the headline config
  mkdir -p gpurun_out/em/src
  python3 -c "import sys; sys.path.insert(0, 'winmad-s-raytracer-v1.0_amd'); from winmad_rt import scenes; scenes.write('gpurun_out/em/torus.scene', scenes.torus_scene(1920, 1080)); open('gpurun_out/em/src/parameters.para', 'w').write('7\n1\n8\n4\n1920\n1080\n5\n400\n')"
  for it in 256 20 1; do
    (cd gpurun_out/em && timeout -k 10 120 ../../winmad-s-raytracer-v1.0_amd/example_main torus.scene o.ppm -bpt $it \
      > ../r4_em_$it.out 2> ../r4_em_$it.err); rc=$?
    echo "em_$it rc=$rc $(tail -1 gpurun_out/r4_em_$it.out)"; [ $rc -eq 0 ] || exit $rc
  done
fi
if [ "${TL:-0}" = 1 ]; then  # kernel timeline of one overlapped iteration
  export TMPDIR=/tmp
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl1 -o run -- \
    python3 bench.py --steps 1 --warmup 3 --no-cpu --no-count --no-compare > gpurun_out/r4_tl1.out 2>&1
  rc=$?; echo "tl1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if [ "${SUITE:-1}" = 1 ]; then
  run suite 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
fi
