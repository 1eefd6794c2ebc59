# One GPU call: bench.py's process-group path over RCCL (backend nccl) at world size 1 --
# init_process_group("nccl", device_id), the device-tensor MAX / SUM all-reduces of the timing,
# the all-gather of per-problem summaries and rank 0's bitwise shard check -- the code the
# 8-GPU C4 run executes, on the one GPU this pool gives us.
# usage: bash tools/gpu_rccl1.sh <tag>
set -o pipefail
TAG=${1:-rccl1}
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --dist --no-cpu-baseline \
  > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo "rccl bench failed"; tail -30 gpurun_out/bench_${TAG}.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}.json'));print(round(d['value']), d.get('sharding') or d.get('shard') or {k: v for k, v in d.items() if 'shard' in k})"
