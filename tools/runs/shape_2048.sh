set -o pipefail
for r in 1 2; do for B in 2048 3072; do for cfg in "auto auto" "pair auto" "auto rows4" "pair rows4"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --steps 10 --batch-per-gpu $B --no-cpu-baseline --no-north-star --ro-variant $1 --bws-variant $2 > gpurun_out/sh_$B_$1_$2.$r.json 2> gpurun_out/sh.err || { tail -3 gpurun_out/sh.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sh_$B_$1_$2.$r.json')); print('$B', '$1', '$2', $r, round(d['value']), round(d['ms_per_step'],3), {k: round(v['avg_launch_ms'],4) for k, v in d['roofline']['per_kernel'].items()})"
done; done; done
