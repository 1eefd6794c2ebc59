# GPU suite + smoke + C3 bench at batch 1024 / 4096 (quick check of a change).
# usage: bash tools/gpu_check.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-chk}
mkdir -p gpurun_out
K=${2:+-k "$2"}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread $K > gpurun_out/tests_${TAG}.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/tests_${TAG}.log | head -30; tail -30 gpurun_out/tests_${TAG}.log; exit 1; }
tail -1 gpurun_out/tests_${TAG}.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/smoke_${TAG}.log; exit 1; }
for B in 1024 4096; do
  timeout -k 10 300 python bench.py --batch-per-gpu $B --no-cpu-baseline > gpurun_out/bench_${TAG}_b$B.json 2> gpurun_out/bench_${TAG}_b$B.err || { echo "bench $B failed"; tail gpurun_out/bench_${TAG}_b$B.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_b$B.json'));print($B, round(d['value']), round(d['ms_per_step'],3), {k: round(v, 3) for k, v in d['kernel_ms_per_step'].items()})"
done
