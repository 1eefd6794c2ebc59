set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_variants.py -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/tests_r02b.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/tests_r02b.log | tail -15
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_r02b.json 2>gpurun_out/bench_r02b.err && python -c "
import json; d=json.load(open('gpurun_out/bench_r02b.json')); print(round(d['value']), {k: round(v,3) for k,v in d['kernel_ms_per_step'].items()})"
