# rocprofv3 passes for the committed profiles: kernel-trace stats, then HBM counters
# (FETCH_SIZE and WRITE_SIZE in separate passes, MI355X_MICROARCH.md §HBM / PMC slots).
# usage: [WL=c5] bash tools/gpu_profile.sh <tag> [batch]
set -o pipefail
TAG=${1:-r01}
B=${2:-1024}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python bench.py --steps 2 --warmup 1 --batch-per-gpu $B --no-cpu-baseline --no-north-star --workload ${WL:-c3}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $CMD > $OUT/trace.log 2>&1 || { echo "trace pass failed"; tail -20 $OUT/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $CMD > $OUT/fetch.log 2>&1 || { echo "fetch pass failed"; tail -20 $OUT/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $CMD > $OUT/write.log 2>&1 || { echo "write pass failed"; tail -20 $OUT/write.log; exit 1; }
find $OUT -name "*.csv" | head -20
echo done
