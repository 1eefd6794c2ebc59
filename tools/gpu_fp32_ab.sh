# fp32 C5 variants: staged divergence diagnostic and bench line per variant build
# usage: VARS="default v1 v2" bash tools/gpu_fp32_ab.sh
set -o pipefail
mkdir -p gpurun_out
V=mhpc_minimal_env_amd/csrc/_build/var
for v in ${VARS:-default}; do
  lib=""; [ $v != default ] && lib=$V/$v/libmhpc_amd.so
  echo "#### $v"
  [ -n "${DIAG:-1}" ] && { MHPC_AMD_LIB=$lib timeout -k 10 300 python tools/diag_fp32_stages.py 64 > gpurun_out/fp32diag_$v.log 2>&1 || { tail gpurun_out/fp32diag_$v.log; exit 1; }; grep -E "^==" gpurun_out/fp32diag_$v.log; }
  MHPC_AMD_LIB=$lib timeout -k 10 300 python bench.py --workload c5f32 --no-cpu-baseline > gpurun_out/c5f32_$v.json 2>gpurun_out/c5f32_$v.err || { tail gpurun_out/c5f32_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/c5f32_$v.json'));print('$v', round(d['value']), {k: round(x,2) for k,x in d['kernel_ms_per_step'].items()})"
done
