# parity tests + bench of the default build, then the rollout cycle breakdown of the timing variants
set -o pipefail
mkdir -p gpurun_out
BATCHES=${BATCHES:-1024 4096} bash tools/gpu_quick2.sh || exit 1
V=mhpc_minimal_env_amd/csrc/_build/var
for v in tr trnp; do
timeout -k 10 200 python tools/ro_timing.py $V/$v/libmhpc_amd.so 1024 > gpurun_out/ro_$v.log 2>&1 && echo $v && cat gpurun_out/ro_$v.log || exit 1
done
