# A/B of library builds copied to ab/<name>.so (tools/build_variants.sh, then cp): C3 bench at
# $BATCHES, $ROUNDS interleaved rounds.  usage: BATCHES="1024 4096" bash tools/gpu_ab.sh a b ...
set -o pipefail
mkdir -p gpurun_out/ab
for r in $(seq ${ROUNDS:-2}); do
  for n in "$@"; do
    for b in ${BATCHES:-1024 4096}; do
      MHPC_AMD_LIB=ab/$n.so timeout -k 10 200 python bench.py --steps ${STEPS:-10} --batch-per-gpu $b --no-cpu-baseline ${EXTRA:-} > gpurun_out/ab/$n.$b.$r.json 2> gpurun_out/ab/$n.$b.$r.err || { echo "$n $b FAILED"; tail -3 gpurun_out/ab/$n.$b.$r.err; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/ab/$n.$b.$r.json')); print('$n', $b, $r, round(d['value']), round(d['ms_per_step'], 3), {k.split('(')[0]: round(v, 3) for k, v in d['kernel_ms_per_step'].items()}, 'per launch', {k: round(v['avg_launch_ms'], 4) for k, v in d['roofline']['per_kernel'].items()})"
    done
  done
done
