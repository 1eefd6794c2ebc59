# GPU parity tests, then bench at batch 1024 / 4096 and (if built) the rollout cycle breakdown
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/tests.log; exit 1; }
tail -1 gpurun_out/tests.log
for b in ${BATCHES:-1024 4096}; do
  timeout -k 10 300 python bench.py --steps ${STEPS:-6} --warmup 2 --batch-per-gpu $b --no-cpu-baseline > gpurun_out/bench_b$b.json 2> gpurun_out/bench.err || { echo "BENCH FAILED"; tail gpurun_out/bench.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_b$b.json')); print($b, round(d['value']), {k: round(v, 2) for k, v in d['kernel_ms_per_step'].items()})"
done
V=mhpc_minimal_env_amd/csrc/_build/var
if [ -f $V/tr/libmhpc_amd.so ]; then
  timeout -k 10 200 python tools/ro_timing.py $V/tr/libmhpc_amd.so 1024 > gpurun_out/ro_timing.log 2>&1 && cat gpurun_out/ro_timing.log
fi
if [ -f $V/tb/libmhpc_amd.so ]; then
  timeout -k 10 200 python tools/bws_timing.py $V/tb/libmhpc_amd.so 1024 > gpurun_out/bws_timing.log 2>&1 && cat gpurun_out/bws_timing.log
fi
exit 0
