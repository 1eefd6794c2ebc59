# Round 6, call c: fp64-bitwise check of the folded PSD test + double sweep (fp32 build), fp32
# accuracy, variant suites (fp32 variants stay bitwise among themselves), A/B, SRB segments.
source tools/gpu_step.sh
O=gpurun_out/r6c; mkdir -p $O
export TMPDIR=/tmp
V=mhpc_minimal_env_amd/csrc/_build/var
REFLIB=ab/base.so BWDIR=/tmp/bw step timeout -k 10 900 bash tools/gpu_bitwise.sh > $O/bitwise.txt 2>&1
step timeout -k 10 600 python -u tools/fp32_bisect.py $O/fp32.json ab/bisect/ae6b1e0 . > $O/fp32.txt 2>&1
step timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_gpu_fp32.py tests/test_gpu_variants.py > $O/tests.txt 2>&1
ROUNDS=2 BATCHES="1024 4096" step timeout -k 10 900 bash tools/gpu_ab.sh base psd > $O/ab.txt 2>&1
for n in base psd; do
  MHPC_AMD_LIB=ab/$n.so step timeout -k 10 300 python bench.py --workload c5f32 --steps 5 --no-cpu-baseline > $O/c5f32_$n.json 2> $O/c5f32_$n.err
done
for b in 1024 1; do step timeout -k 10 200 python tools/bws_timing.py $V/bwst/libmhpc_amd.so $b > $O/bws_timing_b$b.txt 2>&1; done
echo done
