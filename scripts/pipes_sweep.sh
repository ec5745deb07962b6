set -o pipefail
mkdir -p gpurun_out
for cfg in c2 vcm; do
  timeout -k 10 200 python3 bench.py --config $cfg --no-cpu --no-count > gpurun_out/pp_${cfg}_16.log 2>&1 || exit 1
  WR_PIPES=12 timeout -k 10 200 python3 bench.py --config $cfg --no-cpu --no-count > gpurun_out/pp_${cfg}_12.log 2>&1 || exit 1
  GPU_MAX_HW_QUEUES=20 WR_LIB=winmad-s-raytracer-v1.0_amd/variants/p20.so timeout -k 10 200 python3 bench.py --config $cfg --no-cpu --no-count > gpurun_out/pp_${cfg}_20.log 2>&1 || exit 1
  for v in 16 12 20; do echo "$cfg pipes=$v $(tail -1 gpurun_out/pp_${cfg}_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["hw_queues"])')"; done
done
