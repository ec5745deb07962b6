#!/bin/bash
# Round-4 session: the BVH parity tests on the scan list's four-leaves-per-lane
# form (cell filter off), then the s10 measurements.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 500 python -u -m pytest tests/test_gpu_bvh.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r4_btests.out 2>&1 || { echo "btests rc=$?"; tail -5 gpurun_out/r4_btests.out; exit 1; }
echo "btests ok: $(tail -1 gpurun_out/r4_btests.out)"
exec_s10() { bash scripts/r4_gpu_s10.sh; }
sed -e '/^step btests/d' scripts/r4_gpu_s10.sh > /tmp/s10_rest.sh && bash /tmp/s10_rest.sh
