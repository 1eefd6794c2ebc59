# GPU: the host-writable-table reproduction builds vs the shipping build (C5 fp64, 64 problems)
set -o pipefail
mkdir -p gpurun_out/repro_cw
for v in base cw cw_pat "$@"; do
  echo "== $v: $(cat tools/repro_cw/_build/$v/FLAGS)"
  MHPC_AMD_LIB=tools/repro_cw/_build/$v/libmhpc_amd.so timeout -k 10 120 python tools/repro_cw/diag_cw.py gpurun_out/repro_cw/$v.npz > gpurun_out/repro_cw/$v.log 2>&1
  rc=$?; cat gpurun_out/repro_cw/$v.log | grep -v "^  warn"
  [ $rc -ne 0 ] && { echo "rc=$rc: stop"; exit $rc; }
done
exit 0
