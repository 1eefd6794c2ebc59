# A/B of pinned line-search variants (bench.py --ro-variant) at $BATCHES, interleaved.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for b in ${BATCHES:-2048 4096}; do
  for v in ${ROS:-auto pair pipe_staged fused_staged}; do
    timeout -k 10 200 python bench.py --steps ${STEPS:-6} --warmup 2 --batch-per-gpu $b --no-cpu-baseline --ro-variant $v --profile-steps 2 > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('ro=$v', $b, round(d['value']), round(d['ms_per_step'],3), {k: round(v, 2) for k, v in d['kernel_ms_per_step'].items()})"
  done
done
done
