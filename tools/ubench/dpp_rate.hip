// Issue rate / latency of v_fmac_f64_dpp row_newbcast vs plain v_fmac_f64 on gfx950: one wave,
// a loop of ACC independent accumulator chains, cycles per instruction from s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8(x) x x x x x x x x
template <int MODE>
__global__ void k(double* out, long long* cyc, int iters) {
  double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
         a6 = a0 + 6, a7 = a0 + 7, s = 1.0000001, m = 0.9999999;
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
    if (MODE == 0)  // plain, 8 independent chains
      asm volatile(R8("v_fmac_f64_e32 %0, %8, %9\n v_fmac_f64_e32 %1, %8, %9\n v_fmac_f64_e32 %2, %8, %9\n v_fmac_f64_e32 %3, %8, %9\n v_fmac_f64_e32 %4, %8, %9\n v_fmac_f64_e32 %5, %8, %9\n v_fmac_f64_e32 %6, %8, %9\n v_fmac_f64_e32 %7, %8, %9\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s), "v"(m));
    if (MODE == 1)  // dpp, 8 independent chains
      asm volatile(R8("v_fmac_f64_dpp %0, %8, %9 row_newbcast:1\n v_fmac_f64_dpp %1, %8, %9 row_newbcast:2\n v_fmac_f64_dpp %2, %8, %9 row_newbcast:3\n v_fmac_f64_dpp %3, %8, %9 row_newbcast:4\n v_fmac_f64_dpp %4, %8, %9 row_newbcast:5\n v_fmac_f64_dpp %5, %8, %9 row_newbcast:6\n v_fmac_f64_dpp %6, %8, %9 row_newbcast:7\n v_fmac_f64_dpp %7, %8, %9 row_newbcast:8\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s), "v"(m));
    if (MODE == 2)  // plain, 4 chains (dependency distance 4)
      asm volatile(R8("v_fmac_f64_e32 %0, %8, %9\n v_fmac_f64_e32 %1, %8, %9\n v_fmac_f64_e32 %2, %8, %9\n v_fmac_f64_e32 %3, %8, %9\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s), "v"(m));
    if (MODE == 3)  // dpp, 4 chains
      asm volatile(R8("v_fmac_f64_dpp %0, %8, %9 row_newbcast:1\n v_fmac_f64_dpp %1, %8, %9 row_newbcast:2\n v_fmac_f64_dpp %2, %8, %9 row_newbcast:3\n v_fmac_f64_dpp %3, %8, %9 row_newbcast:4\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s), "v"(m));
    if (MODE == 4)  // dpp, 3 chains
      asm volatile(R8("v_fmac_f64_dpp %0, %8, %9 row_newbcast:1\n v_fmac_f64_dpp %1, %8, %9 row_newbcast:2\n v_fmac_f64_dpp %2, %8, %9 row_newbcast:3\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s), "v"(m));
    if (MODE == 5)  // plain, 1 chain (latency)
      asm volatile(R8("v_fmac_f64_e32 %0, %8, %9\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s), "v"(m));
    if (MODE == 6)  // mov_b64_dpp + fmac pairs, 8 chains
      asm volatile(R8("v_mov_b64_dpp v[200:201], %8 row_newbcast:1\n v_fmac_f64_e32 %0, v[200:201], %9\n v_mov_b64_dpp v[202:203], %8 row_newbcast:2\n v_fmac_f64_e32 %1, v[202:203], %9\n v_mov_b64_dpp v[204:205], %8 row_newbcast:3\n v_fmac_f64_e32 %2, v[204:205], %9\n v_mov_b64_dpp v[206:207], %8 row_newbcast:4\n v_fmac_f64_e32 %3, v[206:207], %9\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s), "v"(m) : "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207");
    if (MODE == 7)  // v_mul_f64 plain 8 chains
      asm volatile(R8("v_mul_f64 %0, %0, %9\n v_mul_f64 %1, %1, %9\n v_mul_f64 %2, %2, %9\n v_mul_f64 %3, %3, %9\n v_mul_f64 %4, %4, %9\n v_mul_f64 %5, %5, %9\n v_mul_f64 %6, %6, %9\n v_mul_f64 %7, %7, %9\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s), "v"(m));
    if (MODE == 8)  // s_nop 1 cost: 8 plain fmacs with an s_nop 1 every 4
      asm volatile(R8("s_nop 1\n v_fmac_f64_e32 %0, %8, %9\n v_fmac_f64_e32 %1, %8, %9\n v_fmac_f64_e32 %2, %8, %9\n v_fmac_f64_e32 %3, %8, %9\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s), "v"(m));
  }
  long long t1 = clock64();
  out[blockIdx.x * 64 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  double* out; long long* cyc;
  hipMalloc(&out, 1024 * 64 * 8); hipMalloc(&cyc, 1024 * 8);
  const int iters = 2000;
  const int ins[9] = {64, 64, 32, 32, 24, 8, 64, 64, 32};
  const char* names[9] = {"plain 8ch", "dpp 8ch", "plain 4ch", "dpp 4ch", "dpp 3ch", "plain 1ch",
                          "mov_dpp+fmac 4ch (per pair)", "mul 8ch", "plain 4ch + s_nop1/4"};
  for (int grid : {1, 256, 1024}) {
    for (int mode = 0; mode < 9; ++mode) {
      auto launch = [&]() {
        switch (mode) {
          case 0: hipLaunchKernelGGL(k<0>, dim3(grid), dim3(64), 0, 0, out, cyc, iters); break;
          case 1: hipLaunchKernelGGL(k<1>, dim3(grid), dim3(64), 0, 0, out, cyc, iters); break;
          case 2: hipLaunchKernelGGL(k<2>, dim3(grid), dim3(64), 0, 0, out, cyc, iters); break;
          case 3: hipLaunchKernelGGL(k<3>, dim3(grid), dim3(64), 0, 0, out, cyc, iters); break;
          case 4: hipLaunchKernelGGL(k<4>, dim3(grid), dim3(64), 0, 0, out, cyc, iters); break;
          case 5: hipLaunchKernelGGL(k<5>, dim3(grid), dim3(64), 0, 0, out, cyc, iters); break;
          case 6: hipLaunchKernelGGL(k<6>, dim3(grid), dim3(64), 0, 0, out, cyc, iters); break;
          case 7: hipLaunchKernelGGL(k<7>, dim3(grid), dim3(64), 0, 0, out, cyc, iters); break;
          case 8: hipLaunchKernelGGL(k<8>, dim3(grid), dim3(64), 0, 0, out, cyc, iters); break;
        }
      };
      launch(); hipDeviceSynchronize(); launch(); hipDeviceSynchronize();
      long long c[1024]; hipMemcpy(c, cyc, grid * 8, hipMemcpyDeviceToHost);
      double avg = 0; for (int i = 0; i < grid; ++i) avg += c[i]; avg /= grid;
      printf("grid %4d  %-28s %6.2f cycles/instr\n", grid, names[mode], avg / ((double)iters * ins[mode]));
    }
  }
  return 0;
}
