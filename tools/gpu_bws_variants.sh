# A/B of the backward-sweep launch variants around the automatic thresholds (bench.py --bws-variant)
set -o pipefail
for cfg in "1024 auto" "1024 pairwave" "1024 2wave" "2048 auto" "2048 pairwave" "512 auto" "512 1wave"; do set -- $cfg
  timeout -k 10 200 python bench.py --steps 6 --warmup 2 --batch-per-gpu $1 --bws-variant $2 --no-cpu-baseline > gpurun_out/v.json 2>gpurun_out/v.err || { tail gpurun_out/v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/v.json')); print('$1 $2', round(d['value']), {k: round(v, 2) for k, v in d['kernel_ms_per_step'].items() if 'bws' in k})"
done
