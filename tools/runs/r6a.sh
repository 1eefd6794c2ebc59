# Round 6, first GPU call: LDS-layout bitwise check + A/B, the stride-shrink test, fp32 bisect.
source tools/gpu_step.sh
O=gpurun_out/r6a; mkdir -p $O
step timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_layouts.py -k "shrinking or validation" > $O/layouts.txt 2>&1
REFLIB=ab/base.so BWDIR=/tmp/bw step timeout -k 10 900 bash tools/gpu_bitwise.sh > $O/bitwise.txt 2>&1
step timeout -k 10 1200 python -u tools/fp32_bisect.py $O/bisect.json ab/bisect/2fbff71 ab/bisect/fd2fea1 ab/bisect/273896b ab/bisect/615cdd5 ab/bisect/05165da ab/bisect/3292873 ab/bisect/3bb1db8 ab/bisect/fae04b8 ab/bisect/29213e5 ab/bisect/9fa8102 ab/bisect/9351e9f ab/bisect/403a5a1 ab/bisect/4f60f2a ab/bisect/ae6b1e0 . > $O/bisect.txt 2>&1
ROUNDS=2 BATCHES="1024 4096" step timeout -k 10 900 bash tools/gpu_ab.sh base lds > $O/ab.txt 2>&1
echo done
