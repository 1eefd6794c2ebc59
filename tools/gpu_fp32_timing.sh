# fp64 regression + fp32 C5 diagnostic + per-round cycle breakdowns (bws / rollout)
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_check_bench.sh || exit 1
timeout -k 10 300 python tools/diag_fp32.py 64 > gpurun_out/diag32.log 2>&1 || { echo "DIAG32 FAILED"; tail -20 gpurun_out/diag32.log; exit 1; }
cat gpurun_out/diag32.log
V=mhpc_minimal_env_amd/csrc/_build/var
timeout -k 10 200 python tools/bws_timing.py $V/tb/libmhpc_amd.so 1024 > gpurun_out/bws_timing.log 2>&1 || { echo "BWS TIMING FAILED"; tail gpurun_out/bws_timing.log; exit 1; }
cat gpurun_out/bws_timing.log
timeout -k 10 200 python tools/ro_timing.py $V/tr/libmhpc_amd.so 1024 > gpurun_out/ro_timing.log 2>&1 || { echo "RO TIMING FAILED"; tail gpurun_out/ro_timing.log; exit 1; }
cat gpurun_out/ro_timing.log
