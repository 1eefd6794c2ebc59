# Alternate copies of libmhpc_amd.so whose fp32 kernels are built with extra flags (the fp64
# objects and the dispatcher are the default build), into
# mhpc_minimal_env_amd/csrc/_build/var/<name>/.  usage: bash tools/build_variants32.sh name "-DFLAG" ...
set -e
C=/root/repo/mhpc_minimal_env_amd/csrc
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  d=$C/_build/var/$name; mkdir -p $d
  make -s -C $C all >/dev/null
  F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -DMHPC_FP32"
  /opt/rocm/bin/hipcc $F -fno-slp-vectorize $flags -c -o $d/bws32.o $C/mhpc_bws.hip &
  /opt/rocm/bin/hipcc $F $flags -c -o $d/kern32.o $C/mhpc_kernels.hip &
  /opt/rocm/bin/hipcc $F $flags -x hip -c -o $d/rt32.o $C/mhpc_runtime.cpp &
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $d/libmhpc_amd.so $C/_build/mhpc_bws.o $C/_build/mhpc_kernels.o $C/_build/mhpc_runtime.o \
      $d/kern32.o $d/bws32.o $d/rt32.o $C/_build/mhpc_capi.o
  echo "$name (fp32): $flags" > $d/FLAGS
done
