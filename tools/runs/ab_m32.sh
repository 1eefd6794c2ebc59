set -o pipefail
REFLIB=ab/base7.so NEWLIB=ab/m32.so BWDIR=/tmp/bw1 timeout -k 10 300 bash tools/gpu_bitwise.sh > gpurun_out/bw_m32.txt 2>&1 || { tail -5 gpurun_out/bw_m32.txt; exit 1; }
ROUNDS=2 BATCHES="4096" EXTRA="--workload c5f32" bash tools/gpu_ab.sh base7 m32 || exit 1
