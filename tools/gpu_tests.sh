# GPU test suite (+ optional extra pytest args), log under gpurun_out/.  usage:
#   bash tools/gpu_tests.sh <tag> [pytest args...]
set -o pipefail
TAG=${1:-t}; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread "$@" \
  > gpurun_out/tests_${TAG}.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|SKIPPED" gpurun_out/tests_${TAG}.log | tail -60
tail -30 gpurun_out/tests_${TAG}.log | grep -v PASSED
exit $rc
