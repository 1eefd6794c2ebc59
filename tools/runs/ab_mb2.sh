set -o pipefail
ROUNDS=2 BATCHES="1024 4096" EXTRA="--no-north-star" bash tools/gpu_ab.sh base8 mb2 || exit 1
