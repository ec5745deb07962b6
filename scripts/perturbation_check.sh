#!/bin/bash
# Shows that the film parity gates (tests/_parity.py) catch a 1e-3 error in an
# MIS weight: runs the BDPT-vs-oracle parity tests against a library whose
# connectVertices weight (bidirPathTracing.cpp:658-664) is scaled by 1.001
# (variant built beforehand on the CPU side: scripts/build_variant.sh
# perturb_conn -DWR_TEST_CONN_W=1.001f).  Those tests must FAIL; the same
# tests pass on the product library.  Writes gpurun_out/perturbation.log.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
sel="test_bdpt_matches_oracle_counter_rng or test_bdpt_all_lengths or test_bdpt_1080p_matches_oracle or test_bdpt_1m_scene_film_matches_oracle or test_bdpt_pieces or test_bdpt_tiny"
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -v --timeout 200 --timeout-method thread -k "$sel" \
  > gpurun_out/perturbation_product.log 2>&1
prod=$?
WR_LIB=winmad-s-raytracer-v1.0_amd/variants/perturb_conn.so timeout -k 10 300 python -u -m pytest tests/test_gpu.py \
  -m gpu -v --timeout 200 --timeout-method thread -k "$sel" > gpurun_out/perturbation_variant.log 2>&1
var=$?
echo "product rc=$prod (expect 0); perturbed rc=$var (expect 1: failures)" | tee gpurun_out/perturbation.log
grep -E "PASSED|FAILED" gpurun_out/perturbation_variant.log >> gpurun_out/perturbation.log
[[ $prod == 0 && $var == 1 ]]
