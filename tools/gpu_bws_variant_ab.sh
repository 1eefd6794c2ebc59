# C3 bench with a launch variant pinned (the backward sweep's, or VFLAG=--ro-variant the line
# search's): usage  BATCHES="1 256 1024" bash tools/gpu_bws_variant_ab.sh rows4 pairs2
set -o pipefail
mkdir -p gpurun_out/bwsab
for r in $(seq ${ROUNDS:-1}); do
  for v in "$@"; do
    for b in ${BATCHES:-1 256 1024 2048}; do
      o=gpurun_out/bwsab/$v.$b.$r
      timeout -k 10 200 python bench.py --steps ${STEPS:-10} --batch-per-gpu $b --no-cpu-baseline ${VFLAG:---bws-variant} $v ${EXTRA:-} > $o.json 2> $o.err || { echo "$v $b FAILED"; tail -3 $o.err; exit 1; }
      python -c "import json; d=json.load(open('$o.json')); print('$v', $b, $r, round(d['value']), round(d['ms_per_step'], 3), {k.split('(')[0]: round(v, 3) for k, v in d['kernel_ms_per_step'].items()})"
    done
  done
done
