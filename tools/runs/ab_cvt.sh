set -o pipefail
REFLIB=ab/base9.so NEWLIB=ab/cvt.so BWDIR=/tmp/bw1 timeout -k 10 300 bash tools/gpu_bitwise.sh > gpurun_out/bw_cvt.txt 2>&1 || { tail -5 gpurun_out/bw_cvt.txt; exit 1; }
ROUNDS=2 BATCHES="4096" EXTRA="--workload c5f32 --no-north-star" bash tools/gpu_ab.sh base9 cvt || exit 1
ROUNDS=1 BATCHES="1024" EXTRA="--no-north-star" bash tools/gpu_ab.sh base9 cvt || exit 1
