# Bench A/B of saved builds at small batches (latency end): usage VARS="old" bash tools/gpu_ab_small.sh
set -o pipefail
V=mhpc_minimal_env_amd/csrc/_build/var
for v in default ${VARS:-}; do lib=""; [ $v != default ] && lib=$V/$v/libmhpc_amd.so
  for b in ${BATCHES:-1 256}; do MHPC_AMD_LIB=$lib timeout -k 10 200 python bench.py --steps 5 --warmup 2 --batch-per-gpu $b --no-cpu-baseline > gpurun_out/ab1.json 2>gpurun_out/ab1.err || { tail gpurun_out/ab1.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab1.json')); print('$v', $b, round(d['value']), round(d['ms_per_step'],3), {k: round(v, 3) for k, v in d['kernel_ms_per_step'].items()})"; done; done
