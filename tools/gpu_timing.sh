# Per-part cycle breakdowns of the rollout (tr variant) and the backward sweep (tb variant).
set -o pipefail
mkdir -p gpurun_out
V=mhpc_minimal_env_amd/csrc/_build/var
for b in ${BATCHES:-1024 4096}; do
  timeout -k 10 200 python tools/ro_timing.py $V/tr/libmhpc_amd.so $b > gpurun_out/ro_timing_$b.log 2>&1 && cat gpurun_out/ro_timing_$b.log || exit 1
  timeout -k 10 200 python tools/bws_timing.py $V/tb/libmhpc_amd.so $b > gpurun_out/bws_timing_$b.log 2>&1 && cat gpurun_out/bws_timing_$b.log || exit 1
done
