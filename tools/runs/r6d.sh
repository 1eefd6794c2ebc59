# Round 6, call d: padded partials columns (pcol) bitwise + A/B + partials counters; fp32
# worst-problem diagnosis (double vs float sweep); variant suite on the in-tree build.
source tools/gpu_step.sh
O=gpurun_out/r6d; mkdir -p $O
export TMPDIR=/tmp
REFLIB=ab/base.so NEWLIB=ab/pcol.so BWDIR=/tmp/bw step timeout -k 10 900 bash tools/gpu_bitwise.sh > $O/bitwise.txt 2>&1
step timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_gpu_variants.py tests/test_gpu_layouts.py > $O/tests.txt 2>&1
ROUNDS=2 BATCHES="1024 4096" step timeout -k 10 900 bash tools/gpu_ab.sh base lds18 pcol > $O/ab.txt 2>&1
for n in base pcol; do
  MHPC_AMD_LIB=ab/$n.so step timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU --output-format csv -d $O/pmc_$n -o run -- python3 bench.py --steps 1 --warmup 1 --batch-per-gpu 1024 --no-cpu-baseline --no-north-star > $O/pmc_$n.log 2>&1
  python tools/pmc_table.py $O/pmc_$n > $O/pmc_$n.txt
done
for n in pcol f32flt; do
  MHPC_AMD_LIB=ab/$n.so step timeout -k 10 300 python -u tools/diag_fp32_stages.py 64 50 > $O/diag_$n.txt 2>&1
  MHPC_AMD_LIB=ab/$n.so step timeout -k 10 300 python bench.py --workload c5f32 --steps 5 --no-cpu-baseline > $O/c5f32_$n.json 2> $O/c5f32_$n.err
done
echo done
