set -o pipefail
for r in 1 2; do for n in 0 2 3 6; do
  timeout -k 10 200 python bench.py --steps 10 --workload mixed --no-cpu-baseline --no-north-star --sub-batches $n > gpurun_out/ms_$n.$r.json 2> gpurun_out/ms.err || { tail -3 gpurun_out/ms.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ms_$n.$r.json')); print('sub', $n, $r, round(d['value']), round(d['ms_per_step'],2), 'serial', round(d['serial_homogeneous']['value']))"
done; done
