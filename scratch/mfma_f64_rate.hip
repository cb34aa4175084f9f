// Issue cost of the two fp64 MFMA shapes on gfx950: cycles per instruction for one wave per SIMD
// and for two waves per SIMD, 8 independent accumulator chains per wave.
// build: hipcc --offload-arch=gfx950 -O3 mfma_f64_rate.hip -o mfma_f64_rate
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int IT = 4096;
__global__ void k16(double* out, long long* cyc, double x) {
  d4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = (d4){x, x, x, x};
  double a = x + threadIdx.x, b = x * 0.5;
  long long t0 = wall_clock64();
  long long c0 = clock64();
  for (int it = 0; it < IT; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  long long c1 = clock64();
  double s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = c1 - c0;
  (void)t0;
}
__global__ void k4(double* out, long long* cyc, double x) {
  double acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = x;
  double a = x + threadIdx.x, b = x * 0.5;
  long long c0 = clock64();
  for (int it = 0; it < IT; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 0, 0, 0);
  }
  long long c1 = clock64();
  double s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = c1 - c0;
}
int main() {
  double* out;
  long long* cyc;
  hipMalloc(&out, 1024 * 512 * sizeof(double));
  hipMalloc(&cyc, 1024 * sizeof(long long));
  long long h[1024];
  for (int waves = 4; waves <= 8; waves += 4) {
    for (int kind = 0; kind < 2; ++kind) {
      for (int rep = 0; rep < 2; ++rep) {
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0);
        if (kind == 0) hipLaunchKernelGGL(k16, dim3(256), dim3(64 * waves), 0, 0, out, cyc, 1.0);
        else hipLaunchKernelGGL(k4, dim3(256), dim3(64 * waves), 0, 0, out, cyc, 1.0);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        hipMemcpy(h, cyc, 256 * sizeof(long long), hipMemcpyDeviceToHost);
        double avg = 0;
        for (int i = 0; i < 256; ++i) avg += h[i];
        avg /= 256;
        const double n = (double)IT * 8;
        printf("%s waves/WG %d: %.1f cycles per instruction per wave (clock64), %.3f ms, %.2f TF/s\n",
               kind == 0 ? "16x16x4f64" : "4x4x4f64  ", waves, avg / n, ms,
               256.0 * waves * n * (kind == 0 ? 2048.0 : 512.0) / (ms * 1e-3) / 1e12);
      }
    }
  }
  return 0;
}
