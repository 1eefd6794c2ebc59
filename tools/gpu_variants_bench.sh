# bench every variant library under _build/var (or the names given) at BATCHES
set -o pipefail
mkdir -p gpurun_out/var
V=mhpc_minimal_env_amd/csrc/_build/var
names=${@:-$(ls $V)}
for n in $names; do
  for b in ${BATCHES:-1024 4096}; do
    MHPC_AMD_LIB=$V/$n/libmhpc_amd.so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --batch-per-gpu $b --no-cpu-baseline > gpurun_out/var/$n.$b.json 2> gpurun_out/var/$n.$b.err || { echo "$n $b FAILED"; tail -3 gpurun_out/var/$n.$b.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/var/$n.$b.json')); print('$n', $b, round(d['value']), {k.split('(')[0]: round(v, 2) for k, v in d['kernel_ms_per_step'].items()})"
  done
done
