set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_b1024.json 2> gpurun_out/bench_b1024.err && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --batch-per-gpu 4096 --no-cpu-baseline > gpurun_out/bench_b4096.json 2> gpurun_out/bench_b4096.err && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1 -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1
echo rc=$?
