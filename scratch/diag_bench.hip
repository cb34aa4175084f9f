// isolate the latency of the 64x64 diag (potf2 + inverse) kernel phases
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cmath>
constexpr int TS = 64, NTHR = 256, DS = 65;
__device__ __forceinline__ double wave_sum(double v) { for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o); return v; }

template <int VAR>
__global__ __launch_bounds__(NTHR) void k_diag(const double* Kin, double* Lout, int ld) {
  __shared__ double Ls[TS * DS];
  __shared__ double colbuf[2][TS];
  __shared__ double piv[TS];
  __shared__ double red[4];
  __shared__ double rowbuf[2][TS];
  const int slot = blockIdx.x, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const double* A = Kin + (size_t)slot * ld * ld;
  for (int e = tid; e < TS * TS; e += NTHR) { const int r = e & 63, c = e >> 6; Ls[c * DS + r] = (r >= c) ? A[(size_t)c * ld + r] : 0.0; }
  __syncthreads();
  double a[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) a[q] = Ls[lane * DS + 16 * w + q];
  if (VAR & 1) {
    for (int k = 0; k < TS; ++k) {
      double* cb = colbuf[k & 1];
      if (lane == k) {
#pragma unroll
        for (int q = 0; q < 16; ++q) cb[16 * w + q] = a[q];
      }
      __syncthreads();
      const double akk = cb[k];
      const double pk = (akk > 0.0) ? akk : 1.0;
      if (tid == 0) piv[k] = pk;
      double t;
      if (VAR & 4) t = (lane > k) ? cb[lane] * __builtin_amdgcn_rcp(pk) : 0.0;  // approx (timing only)
      else t = (lane > k) ? cb[lane] / pk : 0.0;
#pragma unroll
      for (int q = 0; q < 16; ++q) a[q] = fma(-cb[16 * w + q], t, a[q]);
    }
  }
  __syncthreads();
  {
    const double sc = sqrt(piv[lane] + 1.0), isc = 1.0 / sc;
#pragma unroll
    for (int q = 0; q < 16; ++q) { const int r = 16 * w + q; Ls[lane * DS + r] = (r > lane) ? a[q] * isc : (r == lane ? sc : 0.0); }
    if (w == 0) { const double s = wave_sum(log(sc)); if (lane == 0) red[0] = s; }
  }
  __syncthreads();
  double x[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) x[q] = (16 * w + q == lane) ? 1.0 : 0.0;
  if (VAR & 2) {
    for (int kb = 0; kb < 4; ++kb) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int k = 16 * kb + q;
        double* rb = rowbuf[k & 1];
        if (w == kb) { x[q] = x[q] / Ls[k * DS + k]; rb[lane] = x[q]; }
        __syncthreads();
        const double xr = rb[lane];
        if (w > kb) {
#pragma unroll
          for (int q2 = 0; q2 < 16; ++q2) x[q2] = fma(-Ls[k * DS + 16 * w + q2], xr, x[q2]);
        } else if (w == kb) {
#pragma unroll
          for (int q2 = q + 1; q2 < 16; ++q2) x[q2] = fma(-Ls[k * DS + 16 * w + q2], xr, x[q2]);
        }
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 16; ++q) Ls[lane * DS + 16 * w + q] = x[q];
  __syncthreads();
  double* Lo = Lout + (size_t)slot * ld * ld;
  for (int e = tid; e < TS * TS; e += NTHR) { const int r = e & 63, c = e >> 6; Lo[(size_t)c * ld + r] = Ls[c * DS + r] + red[0]; }
}
__global__ void k_empty(double* p) { if (threadIdx.x == 1000) p[0] = 1; }

int main() {
  const int B = 48, ld = 2048;
  double *K, *L;
  hipMalloc(&K, (size_t)B * ld * ld * 8); hipMalloc(&L, (size_t)B * ld * ld * 8);
  std::vector<double> h(64 * 64);
  for (int i = 0; i < 64; ++i) for (int j = 0; j < 64; ++j) h[i * 64 + j] = (i == j ? 70.0 : 0.0) + 1.0 / (1 + i + j);
  for (int s = 0; s < B; ++s) hipMemcpy2D(K + (size_t)s * ld * ld, ld * 8, h.data(), 64 * 8, 64 * 8, 64, hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto run = [&](auto kern, const char* name) {
    hipLaunchKernelGGL(kern, dim3(B), dim3(NTHR), 0, 0, K, L, ld);
    hipEventRecord(e0);
    for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(kern, dim3(B), dim3(NTHR), 0, 0, K, L, ld);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("%-28s %8.2f us/launch\n", name, ms * 1000 / 20);
  };
  {
    hipLaunchKernelGGL(k_empty, dim3(B), dim3(NTHR), 0, 0, L);
    hipEventRecord(e0);
    for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(k_empty, dim3(B), dim3(NTHR), 0, 0, L);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("%-28s %8.2f us/launch\n", "empty", ms * 1000 / 20);
  }
  run(k_diag<0>, "load+store only");
  run(k_diag<1>, "potf2 only");
  run(k_diag<2>, "inverse only");
  run(k_diag<3>, "potf2 + inverse");
  run(k_diag<5>, "potf2(rcp) only");
  printf("err=%s\n", hipGetErrorString(hipGetLastError()));
}
