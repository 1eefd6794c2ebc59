# Round 6, call b: LDS layout (pitch 18 single reads / pitch 17 read2) bitwise + A/B + LDS
# counters, SRB knot segments, impact-first partials (C5 fp32), mixed vs serial homogeneous.
source tools/gpu_step.sh
O=gpurun_out/r6b; mkdir -p $O
export TMPDIR=/tmp
V=mhpc_minimal_env_amd/csrc/_build/var
MHPC_AMD_LIB=ab/lds18.so step timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_layouts.py -k "shrinking or validation" > $O/layouts.txt 2>&1
REFLIB=ab/base.so NEWLIB=ab/lds18.so BWDIR=/tmp/bw step timeout -k 10 900 bash tools/gpu_bitwise.sh > $O/bitwise18.txt 2>&1
REFLIB=ab/base.so NEWLIB=$V/lds17/libmhpc_amd.so BWDIR=/tmp/bw17 step timeout -k 10 900 bash tools/gpu_bitwise.sh > $O/bitwise17.txt 2>&1
cp $V/lds17/libmhpc_amd.so ab/lds17.so
ROUNDS=2 BATCHES="1024 4096" step timeout -k 10 900 bash tools/gpu_ab.sh base lds18 lds17 > $O/ab.txt 2>&1
for n in base lds18 lds17; do
  MHPC_AMD_LIB=ab/$n.so step timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY --output-format csv -d $O/pmc_$n -o run -- python3 bench.py --steps 1 --warmup 1 --batch-per-gpu 1024 --no-cpu-baseline --no-north-star > $O/pmc_$n.log 2>&1
  python tools/pmc_table.py $O/pmc_$n > $O/pmc_$n.txt
done
for b in 1024 1; do step timeout -k 10 200 python tools/bws_timing.py $V/bwst/libmhpc_amd.so $b > $O/bws_timing_b$b.txt 2>&1; done
cp $V/impf/libmhpc_amd.so ab/impf.so
for n in base impf; do
  MHPC_AMD_LIB=ab/$n.so step timeout -k 10 300 python bench.py --workload c5f32 --steps 5 --no-cpu-baseline > $O/c5f32_$n.json 2> $O/c5f32_$n.err
  MHPC_AMD_LIB=ab/$n.so step timeout -k 10 300 python bench.py --workload c5 --steps 5 --no-cpu-baseline > $O/c5_$n.json 2> $O/c5_$n.err
done
MHPC_AMD_LIB=ab/impf.so step timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_impf -o run -- python3 bench.py --workload c5f32 --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_impf.log 2>&1
MHPC_AMD_LIB=ab/lds18.so step timeout -k 10 400 python bench.py --workload mixed --steps 5 --no-cpu-baseline > $O/mixed.json 2> $O/mixed.err
echo done
