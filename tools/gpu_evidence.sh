# Round evidence, in two GPU calls (each well inside gpurun's 20-minute limit):
#   bash tools/gpu_evidence.sh <tag> run    parity tests + smoke, bench lines (C3 at 1024 with the
#                                           CPU baseline, 4096; C2; C5 / C5-fp32 / mixed at 4096),
#                                           batch sweep, knot cycle breakdowns
#   bash tools/gpu_evidence.sh <tag> prof   rocprofv3 kernel stats + PMC HBM traffic (C3 1024 /
#                                           4096, C5, C5-fp32, mixed at 4096) and SQ counters
set -o pipefail
TAG=${1:-r01}
WHAT=${2:-run}
mkdir -p gpurun_out
if [ "$WHAT" = run ]; then
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests_${TAG}.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/tests_${TAG}.log; exit 1; }
tail -1 gpurun_out/tests_${TAG}.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/smoke_${TAG}.log; exit 1; }
tail -1 gpurun_out/smoke_${TAG}.log
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/bench_${TAG}_$n.json 2> gpurun_out/bench_${TAG}_$n.err || { echo "bench $n failed"; tail gpurun_out/bench_${TAG}_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_$n.json'));print('$n', round(d['value']), d['unit'], round(d['ms_per_step'],3), 'cpu', (d.get('cpu_baseline') or {}).get('value'))"
}
run b1024
run b4096 --batch-per-gpu 4096 --no-cpu-baseline --no-north-star
run c2_b1 --workload c2 --no-north-star
run c2_b1024 --workload c2 --batch-per-gpu 1024 --no-cpu-baseline --no-north-star
run c5_b4096 --workload c5 --cpu-sample 2048 --no-north-star
run c5f32_b4096 --workload c5f32 --no-cpu-baseline --no-north-star
run mixed_b4096 --workload mixed --no-north-star
timeout -k 10 400 python bench.py --batch-sweep 1,16,64,256,512,1024,2048,4096,8192 --steps 5 --warmup 2 > gpurun_out/sweep_${TAG}.jsonl 2> gpurun_out/sweep_${TAG}.err || { echo "sweep failed"; tail gpurun_out/sweep_${TAG}.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/sweep_${TAG}.jsonl'):
    d = json.loads(l); print('sweep', d['batch'], round(d['value']), 'solves/s', round(d['ms_per_step'], 3), 'ms')
"
V=mhpc_minimal_env_amd/csrc/_build/var
{ timeout -k 10 120 python tools/ro_timing.py $V/rotime/libmhpc_amd.so 1024 && timeout -k 10 120 python tools/ro_timing.py $V/rotime/libmhpc_amd.so 1 \
  && timeout -k 10 120 python tools/bws_timing.py $V/bwstime/libmhpc_amd.so 1024 && timeout -k 10 120 python tools/bws_timing.py $V/bwstime/libmhpc_amd.so 1; } > gpurun_out/cycles_${TAG}.txt 2>&1 || { echo "cycle timing failed"; tail gpurun_out/cycles_${TAG}.txt; exit 1; }
echo cycles done
else
bash tools/gpu_profile.sh ${TAG}_b1024 1024 && bash tools/gpu_profile.sh ${TAG}_b4096 4096 && WL=c5 bash tools/gpu_profile.sh ${TAG}_c5_b4096 4096 && WL=c5f32 bash tools/gpu_profile.sh ${TAG}_c5f32_b4096 4096 && WL=mixed bash tools/gpu_profile.sh ${TAG}_mixed_b4096 4096 && B=1024 bash tools/gpu_pmc_stalls.sh ${TAG}_sq > gpurun_out/sq_${TAG}.txt 2>&1
fi
