# experiment driver: GPU suite of a variant build, A/B bench, rollout timing, fp32 per-phase diag
set -o pipefail
V=mhpc_minimal_env_amd/csrc/_build/var
mkdir -p gpurun_out
for v in ${TESTVARS:-}; do
  MHPC_AMD_LIB=$V/$v/libmhpc_amd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_variants.py tests/test_gpu_solve.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/tests_$v.log 2>&1 || { echo "TESTS $v FAILED"; grep -E "FAILED|Error|assert" gpurun_out/tests_$v.log | head; tail -5 gpurun_out/tests_$v.log; exit 1; }
  echo "tests $v: $(tail -1 gpurun_out/tests_$v.log)"
done
[ -n "${VARS:-}" ] && { bash tools/gpu_ab.sh || exit 1; }
[ -n "${TVARS:-}" ] && { VARS="$TVARS" bash tools/gpu_ro_timing.sh || exit 1; }
[ -n "${FP32DIAG:-}" ] && { MHPC_AMD_LIB=${FP32LIB:-} timeout -k 10 300 python tools/diag_fp32_stages.py 64 || exit 1; }
exit 0
