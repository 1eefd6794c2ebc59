set -o pipefail
ROUNDS=2 BATCHES="4096 1024" EXTRA="--no-north-star" bash tools/gpu_ab.sh base8 pu2 pu5 || exit 1
ROUNDS=1 BATCHES="4096" EXTRA="--workload c5 --no-north-star" bash tools/gpu_ab.sh base8 pu2 pu5 || exit 1
