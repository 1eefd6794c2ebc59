# Round 6, call f: row-major LDS default restored (fp64 must equal base bitwise), fp32 double
# sweep default + float sweep variant (must equal base fp32 bitwise); fp32 tests; A/B.
source tools/gpu_step.sh
O=gpurun_out/r6f; mkdir -p $O
export TMPDIR=/tmp
REFLIB=ab/base.so BWDIR=/tmp/bw step timeout -k 10 900 bash tools/gpu_bitwise.sh > $O/bitwise.txt 2>&1
MHPC_AMD_LIB=ab/base.so step timeout -k 10 200 python tools/lib_bitwise.py dump /tmp/bw/b32.npz c5 64 auto 32
step timeout -k 10 200 python tools/lib_bitwise.py dump /tmp/bw/h32f.npz c5 64 auto 32 32
step timeout -k 10 100 python tools/lib_bitwise.py cmp /tmp/bw/b32.npz /tmp/bw/h32f.npz > $O/bitwise_f32float.txt 2>&1
ROUNDS=2 BATCHES="1024 4096" step timeout -k 10 900 bash tools/gpu_ab.sh base head2 > $O/ab.txt 2>&1
echo done
