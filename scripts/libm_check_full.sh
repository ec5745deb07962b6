#!/bin/bash
# Every-input run of tests/native/libm_check.c (the device's glibc-exact
# cosf / sinf / powf vs this machine's libm) -> profiles/r6/libm_check.json.
# About 5 minutes on one core.
set -e
cd "$(dirname "$0")/.."
exe=$(mktemp -d)/libm_check
gcc -O2 -std=c99 -ffp-contract=off -Wall -o "$exe" tests/native/libm_check.c -lm
{
  "$exe" sampler
  "$exe" range 0 256
  "$exe" range 256 3.4e38 7
  for e in 0 1 20 90 400; do "$exe" powexp $e; done
  "$exe" powrand 100000000 1
} | python3 -c '
import json, sys, platform, subprocess
rows = [json.loads(l) for l in sys.stdin if l.strip()]
glibc = subprocess.run(["ldd", "--version"], capture_output=True, text=True).stdout.splitlines()[0]
fma = "fma" in open("/proc/cpuinfo").read().split()
out = {"glibc": glibc, "cpu_has_fma": fma, "machine": platform.machine(),
       "comparisons": sum(r["n"] for r in rows), "differences": sum(r["diff"] for r in rows), "checks": rows}
json.dump(out, open("profiles/r6/libm_check.json", "w"), indent=1)
print(out["comparisons"], "comparisons,", out["differences"], "differences")
'
