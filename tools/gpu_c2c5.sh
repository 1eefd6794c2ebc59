# C2 rollout and C5 solve workloads: parity tests + bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
grep -E "^(c2|c3) " gpurun_out/tests.log || true
timeout -k 10 300 python bench.py --workload c2 > gpurun_out/bench_c2_b1.json 2> gpurun_out/bench_c2.err || { echo "c2 failed"; tail gpurun_out/bench_c2.err; exit 1; }
timeout -k 10 300 python bench.py --workload c2 --batch-per-gpu 1024 --no-cpu-baseline > gpurun_out/bench_c2_b1024.json 2>> gpurun_out/bench_c2.err || { echo "c2 b1024 failed"; exit 1; }
timeout -k 10 300 python bench.py --workload c5 --cpu-sample 2048 > gpurun_out/bench_c5_b4096.json 2> gpurun_out/bench_c5.err || { echo "c5 failed"; tail gpurun_out/bench_c5.err; exit 1; }
for f in bench_c2_b1 bench_c2_b1024 bench_c5_b4096; do python -c "import json;d=json.load(open('gpurun_out/$f.json'));print('$f', round(d['value']), d['unit'], round(d['ms_per_step'],3), 'cpu', d['cpu_baseline'].get('value'))"; done
