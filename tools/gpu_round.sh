# One GPU call: parity tests (-m gpu), smoke, then the round evidence (bench lines + rocprof
# passes).  usage: bash tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests_${TAG}.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/tests_${TAG}.log; exit 1; }
tail -1 gpurun_out/tests_${TAG}.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/smoke_${TAG}.log; exit 1; }
tail -1 gpurun_out/smoke_${TAG}.log
bash tools/gpu_round_profile.sh ${TAG}
