# bench every variant built by tools/build_variants.sh at the batch sizes in $BATCHES
set -o pipefail
mkdir -p gpurun_out/var
for d in mhpc_minimal_env_amd/csrc/_build/var/*/; do
  n=$(basename $d)
  for b in ${BATCHES:-1024 4096}; do
    MHPC_AMD_LIB=$d/libmhpc_amd.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --batch-per-gpu $b --no-cpu-baseline > gpurun_out/var/$n.$b.json 2>gpurun_out/var/$n.$b.err || { echo "FAILED $n $b"; tail -5 gpurun_out/var/$n.$b.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/var/$n.$b.json'));print('$n',$b,round(d['value']),{k:round(v,2) for k,v in d['kernel_ms_per_step'].items()})"
  done
done
