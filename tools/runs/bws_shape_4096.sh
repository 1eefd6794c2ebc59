set -o pipefail
for r in 1 2; do for v in auto pairs2 rows2; do
  timeout -k 10 200 python bench.py --steps 10 --batch-per-gpu 4096 --no-cpu-baseline --no-north-star --bws-variant $v > gpurun_out/bws_$v.$r.json 2> gpurun_out/bws_$v.$r.err || { tail -3 gpurun_out/bws_$v.$r.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bws_$v.$r.json')); print('$v', $r, round(d['value']), round(d['ms_per_step'],3), {k: round(v['avg_launch_ms'],4) for k, v in d['roofline']['per_kernel'].items()})"
done; done
