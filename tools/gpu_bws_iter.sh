# parity tests + bench (default build) + backward-sweep round timing (tb variant)
set -o pipefail
mkdir -p gpurun_out
BATCHES=${BATCHES:-1024 4096} bash tools/gpu_quick2.sh > gpurun_out/quick.log 2>&1; rc=$?; grep -v "^WB\|^SRB\|^chunk\|^  of\|knots timed" gpurun_out/quick.log; [ $rc -eq 0 ] || exit 1
VARS=tb bash tools/gpu_bws_timing.sh
