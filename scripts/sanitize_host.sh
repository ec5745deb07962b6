#!/bin/bash
# ASan+UBSan and TSan runs of the host translation units (tests/test_sanitize.py),
# CPU only; logs to profiles/r4/sanitize_{asan,tsan}.log.
set -euo pipefail
cd "$(dirname "$0")/.."
rm -f profiles/r4/sanitize_asan.log profiles/r4/sanitize_tsan.log
WR_SANITIZE_LOG=1 python -m pytest tests/test_sanitize.py -q
