# HIP-graph replay of the solve schedule vs host-issued launches (bench.py --graph), after the
# GPU test suite.  usage: bash tools/gpu_graph_ab.sh
set -o pipefail
mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/graph_tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/graph_tests.log | head -20; tail -5 gpurun_out/graph_tests.log; exit 1; }
tail -1 gpurun_out/graph_tests.log
fi
for rep in 1 2; do
for b in ${BATCHES:-1 1024 4096}; do
  for g in on off; do
    timeout -k 10 200 python bench.py --steps ${STEPS:-8} --warmup 2 --batch-per-gpu $b --no-cpu-baseline --graph $g --profile-steps 1 > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('graph=$g', $b, round(d['value']), round(d['ms_per_step'],3))"
  done
done
done
