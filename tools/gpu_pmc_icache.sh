# instruction-cache and issue counters per kernel at batch $B
set -o pipefail
OUT=gpurun_out/pmc_icache_${B:-4096}${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python bench.py --steps 1 --warmup 1 --batch-per-gpu ${B:-4096} --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAVES --output-format csv -d $OUT/p1 -o run -- $CMD > $OUT/p1.log 2>&1 || { echo "pass failed"; tail -5 $OUT/p1.log; exit 1; }
python tools/pmc_table.py $OUT
