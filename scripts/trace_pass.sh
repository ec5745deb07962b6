#!/bin/bash
# rocprofv3 kernel-trace pass of a bench command and the roofline recomputed
# from its trace (scripts/trace_union.py).  Usage (GPU box, repo root):
#   scripts/trace_pass.sh <tag> [bench args...]   -> gpurun_out/trace_<tag>/{line.json,union.json,trace/}
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/trace_$TAG
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --no-compare --no-cpu "$@" > $OUT/line.json 2> $OUT/trace.err || { echo "trace pass failed"; tail -5 $OUT/trace.err; exit 1; }
python3 scripts/trace_union.py $OUT/trace $OUT/line.json --out $OUT/union.json
