# Reproduction of the round-2 "host-writable cost tables" discrepancy:
# the fp64 kernels TU with the constant weight tables referenced from host code, built
# into tools/repro_cw/_build/<name>/libmhpc_amd.so with optional extra flags.
# usage: bash tools/repro_cw/build.sh name "flags" [src]   (src default k_cw.hip)
set -e
R=/root/repo; C=$R/mhpc_minimal_env_amd/csrc; H=$R/tools/repro_cw
name=$1; flags=$2; src=${3:-$H/k_cw.hip}
d=$H/_build/$name; mkdir -p $d
make -s -C $C all >/dev/null
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function $flags -c -o $d/kern.o $src
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $d/libmhpc_amd.so $d/kern.o $C/_build/mhpc_bws.o $C/_build/mhpc_runtime.o \
    $C/_build/mhpc_kernels32.o $C/_build/mhpc_bws32.o $C/_build/mhpc_runtime32.o $C/_build/mhpc_capi.o
echo "$name: $src $flags" > $d/FLAGS
