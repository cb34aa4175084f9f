// Sustained fp64 MFMA rate with random operands (DVFS-loaded clock), operands in registers.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <random>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void k(const double* src, double* out, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  double a[4], b[4];
  for (int i = 0; i < 4; ++i) { a[i] = src[(t * 8 + i) & 4095]; b[i] = src[(t * 8 + 4 + i) & 4095]; }
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = (d4){0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[(s + i) & 3], acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[t] = s;
}

int main() {
  std::vector<double> h(4096);
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> U(-1, 1);
  for (auto& x : h) x = U(g) * 1e-3;
  double *src, *out;
  hipMalloc(&src, 4096 * 8);
  hipMalloc(&out, 256 * 4096 * 8);
  hipMemcpy(src, h.data(), 4096 * 8, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int blocks : {256, 1024, 2048}) {
    const int iters = 20000;
    hipLaunchKernelGGL(k<8>, dim3(blocks), dim3(256), 0, 0, src, out, iters);
    hipEventRecord(e0);
    const int reps = 5;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k<8>, dim3(blocks), dim3(256), 0, 0, src, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double fl = 2048.0 * 4 * 8 * (double)iters * blocks * 4 * reps;
    printf("sustained f64 mfma random operands blocks=%d (waves/SIMD=%d): %.1f ms  %.2f TFLOP/s\n", blocks, blocks / 256,
           ms, fl / ms / 1e9);
  }
  return 0;
}
