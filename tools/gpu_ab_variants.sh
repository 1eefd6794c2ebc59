# A/B of pinned launch variants (bench.py --bws-variant / --ro-variant), interleaved, plus
# the variant parity tests.  usage: BWS="1wave pairwave" BATCHES="1024 4096" bash tools/gpu_ab_variants.sh
set -o pipefail
mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_variants.py -x -v --timeout 300 --timeout-method thread > gpurun_out/ab_variants_tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/ab_variants_tests.log | head -20; tail -5 gpurun_out/ab_variants_tests.log; exit 1; }
tail -1 gpurun_out/ab_variants_tests.log
fi
for rep in 1 2; do
for b in ${BATCHES:-1024 4096}; do
  for v in ${BWS:-1wave pairwave}; do
    timeout -k 10 200 python bench.py --steps ${STEPS:-6} --warmup 2 --batch-per-gpu $b --no-cpu-baseline --bws-variant $v --ro-variant ${RO:-auto} ${EXTRA:-} > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$v', $b, round(d['value']), {k: round(v, 2) for k, v in d['kernel_ms_per_step'].items()})"
  done
done
done
