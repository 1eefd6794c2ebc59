set -o pipefail
ROUNDS=2 BATCHES="1024" EXTRA="--no-north-star" bash tools/gpu_ab.sh base6 pg1a pg1b64 || exit 1
ROUNDS=1 BATCHES="4096" EXTRA="--workload c5" bash tools/gpu_ab.sh base6 pg1a pg1b64 || exit 1
ROUNDS=1 BATCHES="4096" EXTRA="--workload c5f32" bash tools/gpu_ab.sh base6 pg1a pg1b64 || exit 1
ROUNDS=1 BATCHES="4096" EXTRA="--workload mixed" bash tools/gpu_ab.sh base6 pg1a pg1b64 || exit 1
ROUNDS=1 BATCHES="4096" EXTRA="--no-north-star" bash tools/gpu_ab.sh base6 pg1a pg1b64 || exit 1
