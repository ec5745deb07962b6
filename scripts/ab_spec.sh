set -o pipefail
export TMPDIR=/tmp
for v in ${VARIANTS:-head spec1l2}; do
  WR_LIB=winmad-s-raytracer-v1.0_amd/variants/$v.so timeout -k 10 120 python3 scripts/verify_bvh.py --configs c2,c3 --iters 8,4 > gpurun_out/ver_$v.log 2>&1 || { echo "verify $v failed"; tail -3 gpurun_out/ver_$v.log; exit 1; }
  echo "$v verify: $(grep -o '"mismatches": [0-9]*' gpurun_out/ver_$v.log | tr '\n' ' ')"
  WR_LIB=winmad-s-raytracer-v1.0_amd/variants/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/coh_$v -o run -- python3 scripts/coherence_probe.py gpurun_out/coh_$v > gpurun_out/coh_$v.log 2>&1 || { echo "probe $v failed"; exit 1; }
  python3 scripts/coherence_probe.py --parse gpurun_out/coh_$v | sed "s/^/$v /" | grep -E "primary raster|secondary raster|secondary shuffled"
done
STEPS=64 BENCH_ARGS="--no-compare --no-count" bash scripts/variant_bench.sh c2 ${VARIANTS:-head spec1l2}
