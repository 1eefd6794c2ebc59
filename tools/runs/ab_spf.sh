set -o pipefail
REFLIB=ab/base8.so NEWLIB=ab/spf2.so BWDIR=/tmp/bw1 timeout -k 10 300 bash tools/gpu_bitwise.sh > gpurun_out/bw_spf2.txt 2>&1 || { tail -5 gpurun_out/bw_spf2.txt; exit 1; }
ROUNDS=2 BATCHES="1024 4096" EXTRA="--no-north-star" bash tools/gpu_ab.sh base8 spf2 spfw1 || exit 1
ROUNDS=1 BATCHES="4096" EXTRA="--workload c5 --no-north-star" bash tools/gpu_ab.sh base8 spf2 || exit 1
