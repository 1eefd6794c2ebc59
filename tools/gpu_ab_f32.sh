set -o pipefail
mkdir -p gpurun_out/ab
for r in 1 2; do
 for n in cur f32noslp; do
  MHPC_AMD_LIB=ab/$n.so timeout -k 10 200 python bench.py --workload c5f32 --steps 5 --no-cpu-baseline > gpurun_out/ab/$n.$r.json 2> gpurun_out/ab/$n.$r.err || { echo "$n FAILED"; tail -3 gpurun_out/ab/$n.$r.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab/$n.$r.json')); print('$n', $r, round(d['value']), round(d['ms_per_step'],3), {k.split('(')[0]: round(v, 3) for k, v in d['kernel_ms_per_step'].items()})"
 done
done
MHPC_AMD_LIB=ab/f32noslp.so timeout -k 10 300 python -m pytest tests/test_gpu_fp32.py -x -q -s --timeout 200 2>&1 | grep -E "fp32 C5|passed|failed" 
