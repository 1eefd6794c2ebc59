# A/B of one environment switch ($ENVV, e.g. MHPC_SPLIT_SERIAL=1) against the plain run:
# bench at $BATCHES, $STEPS steps, alternating.   usage: ENVV=NAME=1 BATCHES="1024" bash tools/gpu_ab_env.sh
set -o pipefail
mkdir -p gpurun_out
for b in ${BATCHES:-1024 4096}; do
  for v in plain "$ENVV"; do
    if [ "$v" = plain ]; then e=""; else e="$v"; fi
    env $e timeout -k 10 200 python bench.py --steps ${STEPS:-8} --warmup 2 --batch-per-gpu $b --no-cpu-baseline > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$v', $b, round(d['value']), {k: round(v, 3) for k, v in d['kernel_ms_per_step'].items()})"
  done
done
