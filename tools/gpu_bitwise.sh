# Bitwise comparison of the in-tree build against a saved build (tools/lib_bitwise.py) on
# C3 (automatic variant at 1024; every k_bws variant at 256) and C5 (fp64 / fp32, 64).
# usage: REF=old bash tools/gpu_bitwise.sh
set -o pipefail
BW=${BWDIR:-/tmp/bw}; mkdir -p $BW
V=mhpc_minimal_env_amd/csrc/_build/var
rc=0
for cfg in "c3 1024 auto 64" "c3 256 rows2 64" "c3 256 rows1 64" "c3 256 rows4 64" "c5 64 auto 64" "c5 64 auto 32"; do
  set -- $cfg; tag=$1_$2_$3_$4
  MHPC_AMD_LIB=${REFLIB:-$V/${REF:-old}/libmhpc_amd.so} timeout -k 10 200 python tools/lib_bitwise.py dump $BW/ref_$tag.npz $1 $2 $3 $4 || exit 1
  MHPC_AMD_LIB=${NEWLIB:-} timeout -k 10 200 python tools/lib_bitwise.py dump $BW/new_$tag.npz $1 $2 $3 $4 || exit 1
  python tools/lib_bitwise.py cmp $BW/ref_$tag.npz $BW/new_$tag.npz || rc=1
done
exit $rc
