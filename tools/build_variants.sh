# Build alternate copies of libmhpc_amd.so with different compile-time tuning flags into
# mhpc_minimal_env_amd/csrc/_build/var/<name>/ (travels with the gpurun snapshot).
# (flags apply to the fp64 kernels; the fp32 objects and the dispatcher are the default build)
# usage: bash tools/build_variants.sh name1 "-DFLAG=.." name2 "-DFLAG=.." ...
set -e
C=/root/repo/mhpc_minimal_env_amd/csrc
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  d=$C/_build/var/$name; mkdir -p $d
  make -s -C $C all >/dev/null
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $flags -c -o $d/bws.o $C/mhpc_bws.hip &
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $flags -c -o $d/kern.o $C/mhpc_kernels.hip &
  k32=$C/_build/mhpc_kernels32.o; b32=$C/_build/mhpc_bws32.o
  if [ -n "${ALL32:-}" ]; then  # the fp32 kernels with the same flags
    k32=$d/kern32.o; b32=$d/bws32.o
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DMHPC_FP32 $flags -c -o $k32 $C/mhpc_kernels.hip &
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DMHPC_FP32 -fno-slp-vectorize $flags -c -o $b32 $C/mhpc_bws.hip &
  fi
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $d/libmhpc_amd.so $d/bws.o $d/kern.o $C/_build/mhpc_runtime.o \
      $k32 $b32 $C/_build/mhpc_bws32f.o $C/_build/mhpc_runtime32.o $C/_build/mhpc_capi.o
  echo "$name: $flags" > $d/FLAGS
done
