# rollout cycle breakdown of the timing variants (tools/build_variants.sh tr / trnp)
set -o pipefail
mkdir -p gpurun_out
V=mhpc_minimal_env_amd/csrc/_build/var
for v in ${VARS:-tr trnp}; do
timeout -k 10 200 python tools/ro_timing.py $V/$v/libmhpc_amd.so ${B:-1024} > gpurun_out/ro_$v.log 2>&1 && echo $v && cat gpurun_out/ro_$v.log || exit 1
done
