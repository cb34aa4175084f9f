// Do fp64 MFMA and fp64 VALU FMA run concurrently on a gfx950 SIMD?  One 8-wave workgroup per CU
// (LDS request keeps it alone), 2 waves per SIMD: waves 0-3 run MFMA chains, waves 4-7 run VALU
// v_fma_f64 chains, either role alone (the other waves exit at once) or both at once.
//   hipcc --offload-arch=gfx950 -O3 -o scratch/pipes_bench scratch/pipes_bench.hip && scratch/pipes_bench
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int MODE>  // 1: MFMA waves only, 2: VALU waves only, 3: both
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_pipes(const double* src, double* out, int iters) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const bool mf = w < 4;
  if (mf && !(MODE & 1)) return;
  if (!mf && !(MODE & 2)) return;
  double acc_out = 0.0;
  if (mf) {
    double a = src[l], b = src[64 + l];
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    for (int i = 0; i < iters; ++i) {
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
    }
    acc_out = c0[0] + c1[1] + c2[2] + c3[3];
  } else {
    double x[16];
    const double m = src[128 + l], s = src[192 + l];
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = src[l] + k;
    for (int i = 0; i < iters; ++i) {
      // 16 independent FMAs x 8 = 128 FMAs per lane per iteration = 64 MFMA-equivalents of flops? no:
      // one MFMA 16x16x4 = 1024 FMAs per wave = 16 v_fma_f64 (64 lanes); 64 v_fma_f64 here = 4 MFMAs
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int k = 0; k < 16; ++k) x[k] = fma(x[k], m, s);
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) acc_out += x[k];
  }
  out[blockIdx.x * 512 + threadIdx.x] = acc_out;
}

template <int MODE>
double run(const double* src, double* out, int iters, float& ms) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k_pipes<MODE>, dim3(256), dim3(512), 100 * 1024, 0, src, out, iters);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_pipes<MODE>, dim3(256), dim3(512), 100 * 1024, 0, src, out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= 5;
  // flops: MFMA waves 4 MFMAs x 2048 per iteration; VALU waves 64 v_fma_f64 x 64 lanes x 2
  const double fm = (MODE & 1) ? 4.0 * 4 * 2048.0 * iters : 0.0;
  const double fv = (MODE & 2) ? 4.0 * 64 * 64 * 2.0 * iters : 0.0;
  return (fm + fv) * 256 / (ms * 1e-3) / 1e12;
}

int main() {
  double *src, *out;
  (void)hipMalloc(&src, 256 * 8);
  (void)hipMalloc(&out, 256 * 512 * 8);
  double h[256];
  for (int i = 0; i < 256; ++i) h[i] = 1e-3 * ((i * 37) % 101) / 101.0;
  h[128] = 0.999;
  (void)hipMemcpy(src, h, sizeof(h), hipMemcpyHostToDevice);
  (void)hipFuncSetAttribute((const void*)k_pipes<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024);
  (void)hipFuncSetAttribute((const void*)k_pipes<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024);
  (void)hipFuncSetAttribute((const void*)k_pipes<3>, hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024);
  const int iters = 40000;
  float m1, m2, m3;
  const double t1 = run<1>(src, out, iters, m1);
  const double t2 = run<2>(src, out, iters, m2);
  const double t3 = run<3>(src, out, iters, m3);
  printf("{\"mfma_only\": {\"ms\": %.3f, \"tflops\": %.2f}, \"valu_only\": {\"ms\": %.3f, \"tflops\": %.2f}, "
         "\"both\": {\"ms\": %.3f, \"tflops\": %.2f}, \"err\": \"%s\"}\n",
         m1, t1, m2, t2, m3, t3, hipGetErrorString(hipGetLastError()));
  return 0;
}
