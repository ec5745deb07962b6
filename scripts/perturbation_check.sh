#!/bin/bash
# Shows that the film parity gates (tests/_parity.py) catch a 1e-3 error in an
# MIS weight.  Three libraries, built beforehand on the CPU side by
#   scripts/build_variant.sh perturb_conn  -DWR_TEST_CONN_W=1.001f   # connectVertices (:658-664)
#   scripts/build_variant.sh perturb_di    -DWR_TEST_DI_W=1.001f     # getDirectIllumination (:529)
#   scripts/build_variant.sh perturb_splat -DWR_TEST_SPLAT_W=1.001f  # connectToCamera (:360)
# each run the BDPT film tests; every one must FAIL somewhere while the
# product library passes them.  (On torus.scene connectVertices adds exactly
# nothing -- its unweighted f*f*G is below the EPS of Color3::isBlack at that
# scene's scale, DESIGN.md section 8 -- so its variant is caught by the
# Cornell-box and spheres BDPT films.)  Writes gpurun_out/perturbation.log.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
sel="test_bdpt_matches_oracle_counter_rng or test_bdpt_all_lengths or test_bdpt_1080p_matches_oracle or test_bdpt_1m_scene_film_matches_oracle or test_bdpt_pieces or test_bdpt_tiny or test_spheres_bdpt or test_cbox_bdpt"
run() {  # name lib
  if [[ -n "$2" ]]; then export WR_LIB=$2; else unset WR_LIB; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -v --timeout 200 --timeout-method thread -k "$sel" \
    > "gpurun_out/perturbation_$1.log" 2>&1
  local rc=$?
  echo "$1 rc=$rc: $(grep -c PASSED gpurun_out/perturbation_$1.log) passed, $(grep -c FAILED gpurun_out/perturbation_$1.log) failed" \
    | tee -a gpurun_out/perturbation.log
  grep FAILED "gpurun_out/perturbation_$1.log" | grep "::" >> gpurun_out/perturbation.log
  if [[ $rc != 0 && $rc != 1 ]]; then exit $rc; fi
  return $rc
}
: > gpurun_out/perturbation.log
run product "" ; p=$?
ok=1
[[ $p == 0 ]] || ok=0
for v in conn di splat; do
  run "$v" "winmad-s-raytracer-v1.0_amd/variants/perturb_$v.so"; [[ $? == 1 ]] || ok=0
done
echo "verdict: $([[ $ok == 1 ]] && echo 'gates catch every perturbation' || echo 'NOT as expected')" | tee -a gpurun_out/perturbation.log
[[ $ok == 1 ]]
