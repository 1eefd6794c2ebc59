# correctness (GPU parity tests) then the 1-GPU bench at two batch sizes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/tests.log; exit 1; }
tail -3 gpurun_out/tests.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_b1024.json 2> gpurun_out/bench.err || { echo "BENCH FAILED"; tail gpurun_out/bench.err; exit 1; }
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --batch-per-gpu 4096 --no-cpu-baseline > gpurun_out/bench_b4096.json 2>> gpurun_out/bench.err || { echo "BENCH FAILED"; tail gpurun_out/bench.err; exit 1; }
python - <<'PY'
import json
for b in (1024, 4096):
    d = json.load(open(f"gpurun_out/bench_b{b}.json"))
    print(b, f"{d['value']:.0f} solves/s", {k: round(v, 2) for k, v in d["kernel_ms_per_step"].items()}, "roofline", d["roofline"]["kernel"], round(d["roofline"]["achieved"], 1))
PY
