# Sub-batch scheduling A/B (bench.py --sub-batches, MHPC_SUB_LAG), interleaved, after the
# sub-batch parity test.  usage: CONFIGS="1:1 2:0 2:1" (sub-batches:lag) BATCHES="1024 4096" bash tools/gpu_subbatch_ab.sh
set -o pipefail
mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
timeout -k 10 300 python -u -m pytest tests/test_gpu_variants.py -x -v -k "sub_batches" --timeout 200 --timeout-method thread > gpurun_out/ab_sub_tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/ab_sub_tests.log | head -20; tail -5 gpurun_out/ab_sub_tests.log; exit 1; }
tail -1 gpurun_out/ab_sub_tests.log
fi
for rep in 1 2; do
for b in ${BATCHES:-1024 4096}; do
  for c in ${CONFIGS:-1:1 2:1}; do
    v=${c%%:*}; lag=${c##*:}
    MHPC_SUB_LAG=$lag timeout -k 10 200 python bench.py --steps ${STEPS:-6} --warmup 2 --batch-per-gpu $b --no-cpu-baseline --sub-batches $v ${EXTRA:-} > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('sub=$v lag=$lag', $b, round(d['value']), round(d['ms_per_step'],3), {k: round(v, 2) for k, v in d['kernel_ms_per_step'].items()})"
  done
done
done
