# line-search launch variants pinned at the given batches (bench --ro-variant)
set -o pipefail
mkdir -p gpurun_out
for b in ${BATCHES:-2048 4096}; do
  for v in ${VARS:-auto pair pipe_staged fused_staged}; do
    timeout -k 10 200 python bench.py --steps ${STEPS:-4} --warmup 2 --batch-per-gpu $b --no-cpu-baseline --ro-variant $v > gpurun_out/rov.json 2>gpurun_out/rov.err || { tail gpurun_out/rov.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/rov.json')); print('$v', $b, round(d['value']), {k: round(x, 2) for k, x in d['kernel_ms_per_step'].items()})"
  done
done
