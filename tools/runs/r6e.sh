# Round 6, call e: full GPU suite at the candidate head; A/B base / head / float-sweep fp32;
# fp32 accuracy of the three.
source tools/gpu_step.sh
O=gpurun_out/r6e; mkdir -p $O
export TMPDIR=/tmp
step timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/gpu_tests.txt 2>&1
step timeout -k 10 600 python -u tools/fp32_bisect.py $O/fp32.json ab/trees/base ab/trees/f32flt2 . > $O/fp32.txt 2>&1
ROUNDS=2 BATCHES="1024 4096" step timeout -k 10 900 bash tools/gpu_ab.sh base head > $O/ab.txt 2>&1
for n in base head f32flt2; do
  MHPC_AMD_LIB=ab/$n.so step timeout -k 10 300 python bench.py --workload c5f32 --steps 5 --no-cpu-baseline > $O/c5f32_$n.json 2> $O/c5f32_$n.err
done
for n in base head; do
  MHPC_AMD_LIB=ab/$n.so step timeout -k 10 300 python bench.py --workload c5 --steps 5 --no-cpu-baseline > $O/c5_$n.json 2> $O/c5_$n.err
done
echo done
