# A/B of variant builds against the default build: bench at $BATCHES, $STEPS steps, alternating
set -o pipefail
mkdir -p gpurun_out
V=mhpc_minimal_env_amd/csrc/_build/var
for b in ${BATCHES:-1024 2048}; do
  for v in default ${VARS:-np}; do
    lib=""; [ $v != default ] && lib=$V/$v/libmhpc_amd.so
    MHPC_AMD_LIB=$lib timeout -k 10 200 python bench.py --steps ${STEPS:-6} --warmup 2 --batch-per-gpu $b --no-cpu-baseline > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$v', $b, round(d['value']), {k: round(v, 2) for k, v in d['kernel_ms_per_step'].items()})"
  done
done
