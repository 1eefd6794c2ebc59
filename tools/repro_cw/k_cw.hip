#include "../../mhpc_minimal_env_amd/csrc/mhpc_kernels.hip"
// reproduction: the constant weight tables referenced from host code (host-writable)
extern "C" int mhpc_dbg_touch_tables(const void* src) {
  using namespace MHPC_NS;
  int e = 0;
  e |= hipMemcpyToSymbol(HIP_SYMBOL(cQwb), src, sizeof(cQwb));
  e |= hipMemcpyToSymbol(HIP_SYMBOL(cQfwb), src, sizeof(cQfwb));
  e |= hipMemcpyToSymbol(HIP_SYMBOL(cRwb), src, sizeof(cRwb));
  e |= hipMemcpyToSymbol(HIP_SYMBOL(cSwb), src, sizeof(cSwb));
  e |= hipMemcpyToSymbol(HIP_SYMBOL(cQfb), src, sizeof(cQfb));
  e |= hipMemcpyToSymbol(HIP_SYMBOL(cQffb), src, sizeof(cQffb));
  e |= hipMemcpyToSymbol(HIP_SYMBOL(cRfb), src, sizeof(cRfb));
  return e;
}
