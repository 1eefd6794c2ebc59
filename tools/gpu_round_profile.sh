# Round-end evidence: full bench lines (with CPU baseline at the default batch) and the
# rocprofv3 kernel-trace + PMC passes at batch 1024 and 4096.  usage: bash tools/gpu_round_profile.sh <tag>
set -o pipefail
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_${TAG}_b1024.json 2> gpurun_out/bench_${TAG}.err || { echo "bench failed"; tail gpurun_out/bench_${TAG}.err; exit 1; }
timeout -k 10 300 python bench.py --batch-per-gpu 4096 --no-cpu-baseline > gpurun_out/bench_${TAG}_b4096.json 2>> gpurun_out/bench_${TAG}.err || { echo "bench 4096 failed"; exit 1; }
bash tools/gpu_profile.sh ${TAG}_b1024 1024 && bash tools/gpu_profile.sh ${TAG}_b4096 4096
