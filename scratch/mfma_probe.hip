// Probe: f64 MFMA 16x16x4 operand/result layout and throughput on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void layout_kernel(const double* A, const double* B, double* out) {
  int l = threadIdx.x;
  double a = A[(l & 15) * 4 + (l >> 4)];   // A[i=l&15][k=l>>4], A is 16x4 row-major
  double b = B[(l >> 4) * 16 + (l & 15)];  // B[k=l>>4][j=l&15], B is 4x16 row-major
  d4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}

template <int NACC>
__global__ void rate_kernel(double* out, int iters, double s) {
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = (d4){0, 0, 0, 0};
  double a = threadIdx.x * 1e-3 + s, b = 1.0 - threadIdx.x * 1e-4;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double t = 0;
  for (int i = 0; i < NACC; ++i) t += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

__global__ void valu_kernel(double* out, int iters, double s) {
  double x0 = threadIdx.x * 1e-3 + s, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
  const double m = 0.999999, c = 1e-7;
  for (int it = 0; it < iters; ++it) {
    x0 = fma(x0, m, c); x1 = fma(x1, m, c); x2 = fma(x2, m, c); x3 = fma(x3, m, c);
    x4 = fma(x4, m, c); x5 = fma(x5, m, c); x6 = fma(x6, m, c); x7 = fma(x7, m, c);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}

int main() {
  std::vector<double> A(64), B(64), out(256);
  for (int i = 0; i < 16; ++i) for (int k = 0; k < 4; ++k) A[i * 4 + k] = i * 4 + k + 1;        // distinct
  for (int k = 0; k < 4; ++k) for (int j = 0; j < 16; ++j) B[k * 16 + j] = (k == 0 ? 1 : 0) * (j == 0 ? 1 : 0) + (k + 1) * 1000.0 * (j + 1);
  double *dA, *dB, *dO;
  hipMalloc(&dA, 512); hipMalloc(&dB, 512); hipMalloc(&dO, 256 * 8 * 1024);
  hipMemcpy(dA, A.data(), 512, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), 512, hipMemcpyHostToDevice);
  layout_kernel<<<1, 64>>>(dA, dB, dO);
  hipMemcpy(out.data(), dO, 256 * 8, hipMemcpyDeviceToHost);
  // reference D[i][j] = sum_k A[i][k] B[k][j]
  int bad_guide = 0, bad_alt = 0;
  for (int l = 0; l < 64; ++l) for (int r = 0; r < 4; ++r) {
    int j = l & 15;
    int i_guide = (l >> 4) + 4 * r;       // guide: row=(lane>>4)+4*reg
    int i_alt = (l >> 4) * 4 + r;         // f32 16x16x4 style
    double ref_g = 0, ref_a = 0;
    for (int k = 0; k < 4; ++k) { ref_g += A[i_guide * 4 + k] * B[k * 16 + j]; ref_a += A[i_alt * 4 + k] * B[k * 16 + j]; }
    if (ref_g != out[l * 4 + r]) bad_guide++;
    if (ref_a != out[l * 4 + r]) bad_alt++;
  }
  printf("layout: mismatches guide-map(row=(l>>4)+4r)=%d alt-map(row=4(l>>4)+r)=%d\n", bad_guide, bad_alt);

  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  int iters = 20000;
  for (int wpb = 1; wpb <= 8; wpb *= 2) {
    int blocks = 256 * 4 / wpb * 2;  // 2 waves / SIMD overall
    rate_kernel<4><<<blocks, 64 * wpb>>>(dO, 10, 0.0);
    hipEventRecord(e0);
    rate_kernel<4><<<blocks, 64 * wpb>>>(dO, iters, 0.0);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double flops = (double)blocks * wpb * iters * 4 * 2048.0;
    printf("mfma f64 4acc blocks=%d wpb=%d: %.3f ms  %.2f TFLOP/s\n", blocks, wpb, ms, flops / ms / 1e9);
  }
  {
    int blocks = 1024, wpb = 4;
    hipEventRecord(e0);
    rate_kernel<1><<<blocks, 64 * wpb>>>(dO, iters, 0.0);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double flops = (double)blocks * wpb * iters * 1 * 2048.0;
    printf("mfma f64 1acc (dependent) blocks=%d: %.3f ms  %.2f TFLOP/s\n", blocks, ms, flops / ms / 1e9);
    hipEventRecord(e0);
    rate_kernel<1><<<256, 64>>>(dO, iters, 0.0);
    hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("mfma f64 1acc 1 wave/CU: %.3f ms -> %.1f ns per dependent mfma\n", ms, ms * 1e6 / iters);
    hipEventRecord(e0);
    rate_kernel<4><<<256, 64>>>(dO, iters, 0.0);
    hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("mfma f64 4acc 1 wave/CU: %.3f ms -> %.1f ns per mfma\n", ms, ms * 1e6 / iters / 4);
  }
  for (int occ = 1; occ <= 8; occ *= 2) {
    int blocks = 256 * occ;
    hipEventRecord(e0);
    valu_kernel<<<blocks, 256>>>(dO, iters, 0.0);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double flops = (double)blocks * 256 * iters * 8 * 2.0;
    printf("valu fma f64 blocks=%d: %.3f ms  %.2f TFLOP/s\n", blocks, ms, flops / ms / 1e9);
  }
  return 0;
}
