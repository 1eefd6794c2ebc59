# Quick check of a kernel change: pair/variant parity tests, then C3 bench at 1024 and 4096.
# usage: bash tools/gpu_quick_ab.sh [tag]
set -o pipefail
TAG=${1:-q}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_kernels.py tests/test_gpu_variants.py tests/test_gpu_solve.py} -x -q --timeout 200 --timeout-method thread > gpurun_out/quick_${TAG}.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/quick_${TAG}.log | head -20; tail -5 gpurun_out/quick_${TAG}.log; exit 1; }
tail -1 gpurun_out/quick_${TAG}.log
for b in ${BATCHES:-1024 4096}; do
  timeout -k 10 200 python bench.py --steps 6 --warmup 2 --batch-per-gpu $b --no-cpu-baseline > gpurun_out/q.json 2>gpurun_out/q.err || { tail gpurun_out/q.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/q.json')); print($b, round(d['value']), round(d['ms_per_step'],3), {k: round(v, 2) for k, v in d['kernel_ms_per_step'].items()})"
done
