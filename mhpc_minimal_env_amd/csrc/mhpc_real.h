// Arithmetic type of the solve path.  The device code and the runtime are compiled twice:
// fp64 (namespace mhpc, the reference's precision) and, with -DMHPC_FP32, fp32 (namespace
// mhpc32); mhpc_capi.cpp dispatches on the problem descriptor's
// precision.  The kernel-level parity hooks exist in fp64 only.
#pragma once

#ifndef MHPC_FP32
#define MHPC_NS mhpc
#define MHPC_REAL double
#else
#define MHPC_NS mhpc32
#define MHPC_REAL float
#endif

namespace MHPC_NS {
using real = MHPC_REAL;
}  // namespace MHPC_NS
