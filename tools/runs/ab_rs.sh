set -o pipefail
REFLIB=ab/base10.so NEWLIB=ab/rs1.so BWDIR=/tmp/bw1 timeout -k 10 300 bash tools/gpu_bitwise.sh > gpurun_out/bw_rs1.txt 2>&1 || { tail -5 gpurun_out/bw_rs1.txt; exit 1; }
ROUNDS=3 BATCHES="1024" EXTRA="--no-north-star" bash tools/gpu_ab.sh base10 rs0 rs1 || exit 1
ROUNDS=1 BATCHES="1 256" EXTRA="--no-north-star" bash tools/gpu_ab.sh base10 rs1 || exit 1
