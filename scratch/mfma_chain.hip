// fp64 MFMA issue rate of ONE wave per SIMD against the number of independent accumulator chains
// (the fused leaf's 64 x 16 tasks keep 4): operands in registers, 1 workgroup of 4 waves per CU
// (a large dynamic LDS request keeps a second one off the CU).  Prints cycles per MFMA per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
template <int NACC>
__global__ __launch_bounds__(256) void k_chain(double* out, int iters, double seed) {
  extern __shared__ double lds[];
  const int l = threadIdx.x & 63;
  double a[4], b[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    a[s] = seed * (l + s + 1);
    b[s] = seed / (l + s + 2);
  }
  d4 acc[NACC];
#pragma unroll
  for (int c = 0; c < NACC; ++c) acc[c] = (d4){0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int c = 0; c < NACC; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[(s + c) & 3], acc[c], 0, 0, 0);
  }
  double t = 0;
#pragma unroll
  for (int c = 0; c < NACC; ++c) t += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  if (t == 12345.678) lds[l] = t;  // keeps the LDS request and the chains alive
  out[blockIdx.x * 256 + threadIdx.x] = t;
}
template <int NACC>
void run(double* out, hipEvent_t e0, hipEvent_t e1, int wps = 1) {
  const int iters = 4096 / NACC;  // the same MFMA count per wave for every NACC
  const size_t lds = wps == 1 ? 100 * 1024 : 70 * 1024;  // one or two workgroups (waves per SIMD) per CU
  hipFuncSetAttribute((const void*)k_chain<NACC>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k_chain<NACC>, dim3(256 * wps), dim3(256), lds, 0, out, iters, 1e-3);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k_chain<NACC>, dim3(256 * wps), dim3(256), lds, 0, out, iters, 1e-3);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double mfma_per_simd = 4.0 * 4096 * wps;  // MFMAs per SIMD (wps waves per SIMD)
  printf("waves/SIMD=%d NACC=%2d  %.3f ms  %.1f ns per MFMA per SIMD (%.1f cycles at 2.4 GHz)  err=%s\n", wps, NACC, ms,
         ms * 1e6 / mfma_per_simd, ms * 1e6 / mfma_per_simd * 2.4, hipGetErrorString(hipGetLastError()));
}
int main() {
  double* out;
  hipMalloc(&out, 512 * 256 * sizeof(double));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  run<1>(out, e0, e1);
  run<2>(out, e0, e1);
  run<4>(out, e0, e1);
  run<8>(out, e0, e1);
  run<16>(out, e0, e1);
  run<4>(out, e0, e1, 2);
  run<16>(out, e0, e1, 2);
  return 0;
}
