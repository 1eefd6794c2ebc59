# One GPU call: full GPU test suite (no -x: every failure listed), smoke, bench at batch
# 1024 (with CPU baseline) and 4096, rocprofv3 kernel stats + HBM counters at 1024.
# usage: bash tools/gpu_round.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-r02}
K=${2:-}
mkdir -p gpurun_out
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread "${KARG[@]}" > gpurun_out/tests_${TAG}.log 2>&1
trc=$?
grep -E "FAILED|ERROR" gpurun_out/tests_${TAG}.log | head -20
tail -1 gpurun_out/tests_${TAG}.log
# a timeout / crash ends the call here (nothing more on the GPU)
if [ $trc -ne 0 ] && [ $trc -ne 1 ]; then echo "pytest rc=$trc: stopping"; exit $trc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/smoke_${TAG}.log; exit 1; }
tail -1 gpurun_out/smoke_${TAG}.log
timeout -k 10 400 python bench.py > gpurun_out/bench_${TAG}_b1024.json 2> gpurun_out/bench_${TAG}_b1024.err || { echo "bench failed"; tail gpurun_out/bench_${TAG}_b1024.err; exit 1; }
timeout -k 10 400 python bench.py --batch-per-gpu 4096 --no-cpu-baseline > gpurun_out/bench_${TAG}_b4096.json 2> gpurun_out/bench_${TAG}_b4096.err || { echo "bench 4096 failed"; exit 1; }
python - <<PY
import json
for b in (1024, 4096):
    d = json.load(open(f"gpurun_out/bench_${TAG}_b{b}.json"))
    print(b, round(d["value"]), "solves/s", round(d["ms_per_step"], 3), "ms", {k: round(v, 3) for k, v in d["kernel_ms_per_step"].items()}, "cpu", (d.get("cpu_baseline") or {}).get("value"))
PY
bash tools/gpu_profile.sh ${TAG}_b1024 1024 && exit $trc
