# LDS / issue counters of one bench step for the in-tree build and the saved builds $VARS,
# at batch $B (default 4096).  usage: B=4096 VARS="old" bash tools/gpu_pmc_lds.sh <tag>
set -o pipefail
TAG=${1:-lds}
export TMPDIR=/tmp
V=mhpc_minimal_env_amd/csrc/_build/var
for v in default ${VARS:-}; do
  lib=""; [ $v != default ] && lib=$V/$v/libmhpc_amd.so
  OUT=gpurun_out/pmc_${TAG}_$v
  mkdir -p $OUT
  CMD="python bench.py --steps 1 --warmup 1 --batch-per-gpu ${B:-4096} --no-cpu-baseline"
  i=0
  for set in "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU" \
             "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"; do
    i=$((i+1))
    MHPC_AMD_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  done
  echo "== $v"
  python tools/pmc_table.py $OUT | grep -A16 "^k_bws\|_bws" | head -60
done
