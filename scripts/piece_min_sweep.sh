mkdir -p gpurun_out/r6
export GPU_MAX_HW_QUEUES=16
for rep in 1 2; do
for pm in 655360 393216 262144 131072; do
  WR_PIECE_MIN=$pm timeout -k 10 120 python -u bench.py --steps 1 --warmup 3 --no-cpu --no-compare --no-count > gpurun_out/r6/pm_$pm.json 2>/dev/null || exit 1
  echo "pm $pm $(python3 -c "import json;d=json.loads(open('gpurun_out/r6/pm_$pm.json').read().strip().splitlines()[-1]);print(d['value'], d['config']['pipelines'])")"
done
done
