# backward-sweep round breakdown of the timing variants (tools/build_variants.sh)
set -o pipefail
mkdir -p gpurun_out
V=mhpc_minimal_env_amd/csrc/_build/var
for v in ${VARS:-tb}; do
timeout -k 10 200 python tools/bws_timing.py $V/$v/libmhpc_amd.so ${B:-1024} > gpurun_out/bws_$v.log 2>&1 && echo $v && cat gpurun_out/bws_$v.log | tail -12 || exit 1
done
