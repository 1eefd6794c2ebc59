set -o pipefail
mkdir -p gpurun_out/v2
V=mhpc_minimal_env_amd/csrc/_build/var
for t in tb tbp1 tbp2 tbns; do
  timeout -k 10 200 python tools/bws_timing.py $V/$t/libmhpc_amd.so 1024 > gpurun_out/v2/$t.log 2>&1 || { echo "$t FAILED"; tail gpurun_out/v2/$t.log; exit 1; }
  echo "== $t"; tail -8 gpurun_out/v2/$t.log
done
MHPC_AMD_LIB=$V/p1/libmhpc_amd.so timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/v2/p1_tests.log 2>&1; tail -3 gpurun_out/v2/p1_tests.log
for b in 1024 4096; do
MHPC_AMD_LIB=$V/p1/libmhpc_amd.so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --batch-per-gpu $b --no-cpu-baseline > gpurun_out/v2/p1_$b.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/v2/p1_$b.json')); print('p1', $b, round(d['value']), {k: round(v, 2) for k, v in d['kernel_ms_per_step'].items()})"
done
