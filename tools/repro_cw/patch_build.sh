# Proof of the diagnosis: rebuild the repro library from its own device
# assembly with ONE instruction moved -- the live-range copy `v_mov_b64 v[168:169],
# v[124:125]` placed ahead of the exec restore of join block .LBB18_220 in
# k_rollout<false,false,false> goes after `s_or_b64 exec, exec, s[6:7]` -- and nothing else.
# usage: bash tools/repro_cw/patch_build.sh   (run after build.sh cw; writes _build/cw_fixed)
set -e
R=/root/repo; C=$R/mhpc_minimal_env_amd/csrc; H=$R/tools/repro_cw; L=/opt/rocm/lib/llvm/bin
T=$(mktemp -d); cd $T
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -save-temps -c -o kern.o $H/k_cw.hip 2>/dev/null
S=k_cw-hip-amdgcn-amd-amdhsa-gfx950.s
relink() {  # device asm $1 -> fat binary $2
  $L/clang -cc1as -triple amdgcn-amd-amdhsa -filetype obj -target-cpu gfx950 -mrelocation-model pic -o dev.o $1
  $L/lld -flavor gnu -m elf64_amdgpu --no-undefined -shared -o dev.out dev.o
  $L/clang-offload-bundler -type=o -bundle-align=4096 -targets=host-x86_64-unknown-linux-gnu,hipv4-amdgcn-amd-amdhsa--gfx950 -input=/dev/null -input=dev.out -output=$2
}
relink $S same.hipfb   # the pipeline reproduces the compiler's own fat binary bit for bit
cmp same.hipfb k_cw.hip-hip-amdgcn-amd-amdhsa.hipfb
python3 - $S <<'PY'
import sys
p = sys.argv[1]
L = open(p).read().split("\n")
i = [k for k, l in enumerate(L) if l.startswith(".LBB18_220:")][0]
a, b = [k for k in range(i + 1, i + 20) if L[k].split(";")[0].strip()][:2]
assert L[a].strip() == "v_mov_b64_e32 v[168:169], v[124:125]", L[a]
assert L[b].strip() == "s_or_b64 exec, exec, s[6:7]", L[b]
L[a], L[b] = L[b], L[a]
open("patched.s", "w").write("\n".join(L))
PY
relink patched.s fixed.hipfb
objcopy --update-section .hip_fatbin=fixed.hipfb kern.o kern_fixed.o
d=$H/_build/cw_fixed; mkdir -p $d
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $d/libmhpc_amd.so kern_fixed.o $C/_build/mhpc_bws.o $C/_build/mhpc_runtime.o \
    $C/_build/mhpc_kernels32.o $C/_build/mhpc_bws32.o $C/_build/mhpc_runtime32.o $C/_build/mhpc_capi.o
echo "cw_fixed: k_cw.hip with the .LBB18_220 copy moved after the exec restore" > $d/FLAGS
python3 $R/tools/check_exec_prologue.py patched.s
rm -rf $T
