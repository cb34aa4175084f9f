// fp64 MFMA wave-tile size study: 64x64 per wave (library core, 2 waves/SIMD) against 128x64 and
// 128x128 per wave (accumulators in AGPRs, 1-2 waves/SIMD) on the hot path's batched shapes
// (C = A B^T over panels of column-major ld=2048 matrices, one 1024x1024 output panel per slot,
// 192 slots, XCD slot mapping as the library).  Prints TF/s per variant and K.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double d4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ d4 mfma(double a, double b, d4 c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }

template <int WM, int WN, int SD>
struct Frag { double a[SD][WM], b[SD][WN]; };
template <int WM, int WN, int SD>
__device__ __forceinline__ void fload(Frag<WM, WN, SD>& f, const double* pa, const double* pb, size_t sa, size_t sb) {
#pragma unroll
  for (int s = 0; s < SD; ++s) {
#pragma unroll
    for (int a = 0; a < WM; ++a) f.a[s][a] = pa[s * sa + 16 * a];
#pragma unroll
    for (int b = 0; b < WN; ++b) f.b[s][b] = pb[s * sb + 16 * b];
  }
}
template <int WM, int WN, int SD>
__device__ __forceinline__ void fmma(d4 (&acc)[WM][WN], const Frag<WM, WN, SD>& f) {
#pragma unroll
  for (int s = 0; s < SD; ++s)
#pragma unroll
    for (int a = 0; a < WM; ++a)
#pragma unroll
      for (int b = 0; b < WN; ++b) acc[a][b] = mfma(f.b[s][b], f.a[s][a], acc[a][b]);
}
// stage = SD sub-steps of depth 4; two register stages in ping-pong
template <int WM, int WN, int SD>
__device__ __forceinline__ void core(d4 (&acc)[WM][WN], const double* A, size_t lda, const double* B, size_t ldb, int K) {
  const int nst = __builtin_amdgcn_readfirstlane(K / (4 * SD));
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const double* pa = A + lr + (size_t)lk * lda;
  const double* pb = B + lr + (size_t)lk * ldb;
  const size_t sa = 4 * lda, sb = 4 * ldb;
  Frag<WM, WN, SD> f0, f1;
  fload(f0, pa, pb, sa, sb);
  for (int it = 0; it < nst; it += 2) {
    fload(f1, pa + (size_t)(it + 1) * SD * sa, pb + (size_t)(it + 1) * SD * sb, sa, sb);
    fmma(acc, f0);
    const int n2 = (it + 2 < nst) ? it + 2 : nst - 1;
    fload(f0, pa + (size_t)n2 * SD * sa, pb + (size_t)n2 * SD * sb, sa, sb);
    fmma(acc, f1);
  }
}

// the same core with scheduling barriers between the four phases: the prefetch of stage it+1 stays
// in flight across the MFMAs of stage it (the compiler otherwise sinks the loads and waits on all)
template <int WM, int WN, int SD>
__device__ __forceinline__ void core_sb(d4 (&acc)[WM][WN], const double* A, size_t lda, const double* B, size_t ldb, int K) {
  const int nst = __builtin_amdgcn_readfirstlane(K / (4 * SD));
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const double* pa = A + lr + (size_t)lk * lda;
  const double* pb = B + lr + (size_t)lk * ldb;
  const size_t sa = 4 * lda, sb = 4 * ldb;
  Frag<WM, WN, SD> f0, f1;
  fload(f0, pa, pb, sa, sb);
  for (int it = 0; it < nst; it += 2) {
    fload(f1, pa + (size_t)(it + 1) * SD * sa, pb + (size_t)(it + 1) * SD * sb, sa, sb);
    __builtin_amdgcn_sched_barrier(0);
    fmma(acc, f0);
    __builtin_amdgcn_sched_barrier(0);
    const int n2 = (it + 2 < nst) ? it + 2 : nst - 1;
    fload(f0, pa + (size_t)n2 * SD * sa, pb + (size_t)n2 * SD * sb, sa, sb);
    __builtin_amdgcn_sched_barrier(0);
    fmma(acc, f1);
    __builtin_amdgcn_sched_barrier(0);
  }
}


// R register stages of depth 4 SD in a ring: stage it + R - 1 is loaded while stage it runs
template <int WM, int WN, int SD, int R>
__device__ __forceinline__ void core_ring(d4 (&acc)[WM][WN], const double* A, size_t lda, const double* B, size_t ldb, int K) {
  const int nst = __builtin_amdgcn_readfirstlane(K / (4 * SD));
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const double* pa = A + lr + (size_t)lk * lda;
  const double* pb = B + lr + (size_t)lk * ldb;
  const size_t sa = 4 * lda, sb = 4 * ldb;
  Frag<WM, WN, SD> f[R];
#pragma unroll
  for (int r = 0; r < R - 1; ++r) {
    const int n = r < nst ? r : nst - 1;
    fload(f[r], pa + (size_t)n * SD * sa, pb + (size_t)n * SD * sb, sa, sb);
  }
  for (int it = 0; it < nst; it += R) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int nx = it + r + R - 1, n = nx < nst ? nx : nst - 1;
      fload(f[(r + R - 1) % R], pa + (size_t)n * SD * sa, pb + (size_t)n * SD * sb, sa, sb);
      __builtin_amdgcn_sched_barrier(0);
      if (it + r < nst) fmma(acc, f[r]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// WG = 4 waves (2 x 2), wave tile (16 WM) x (16 WN); WG tile (32 WM) x (32 WN).
template <int WM, int WN, int SD, bool SB = false, int R = 0>
__device__ __forceinline__ void body(const double* P, double* C, int T, int nbr, int K, int S) {
  const int x = blockIdx.x & 7, q = blockIdx.x >> 3;
  const int slot = (q / T) * 8 + x, u = q % T;
  if (slot >= S) return;
  const int bi = u % nbr, bj = u / nbr;
  const double* M = P + (size_t)slot * 2048 * 2048;
  const int w = threadIdx.x >> 6, wr = w >> 1, wc = w & 1;
  d4 acc[WM][WN];
#pragma unroll
  for (int a = 0; a < WM; ++a)
#pragma unroll
    for (int b = 0; b < WN; ++b) acc[a][b] = (d4){0, 0, 0, 0};
  const int r0 = 1024 + bi * 32 * WM + 16 * WM * wr, c0 = bj * 32 * WN + 16 * WN * wc;
  if constexpr (R > 0) core_ring<WM, WN, SD, R>(acc, M + r0, 2048, M + c0, 2048, K);
  else if constexpr (SB) core_sb<WM, WN, SD>(acc, M + r0, 2048, M + c0, 2048, K);
  else core<WM, WN, SD>(acc, M + r0, 2048, M + c0, 2048, K);
  double* Cs = C + (size_t)slot * 1024 * 1024;
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
#pragma unroll
  for (int a = 0; a < WM; ++a)
#pragma unroll
    for (int b = 0; b < WN; ++b)
#pragma unroll
      for (int qq = 0; qq < 4; ++qq)
        Cs[(size_t)(c0 + 16 * b + lk + 4 * qq) * 1024 + (r0 - 1024) + 16 * a + lr] = acc[a][b][qq];
}
#define KERN(NAME, WM, WN, SD, OCC)                                                                   \
  __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, OCC))) void NAME(         \
      const double* P, double* C, int T, int nbr, int K, int S) {                                     \
    body<WM, WN, SD>(P, C, T, nbr, K, S);                                                             \
  }
KERN(k_64x64_sd4_o2, 4, 4, 4, 2)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_64x64_sb_o2(
    const double* P, double* C, int T, int nbr, int K, int S) {
  body<4, 4, 4, true>(P, C, T, nbr, K, S);
}
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_64x64_sb2_o2(
    const double* P, double* C, int T, int nbr, int K, int S) {
  body<4, 4, 2, true>(P, C, T, nbr, K, S);
}
#define RING(NAME, SD, R)                                                                             \
  __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void NAME(             \
      const double* P, double* C, int T, int nbr, int K, int S) {                                     \
    body<4, 4, SD, false, R>(P, C, T, nbr, K, S);                                                     \
  }
RING(k_ring_sd2_r3, 2, 3)
RING(k_ring_sd1_r4, 1, 4)
RING(k_ring_sd1_r3, 1, 3)
RING(k_ring_sd2_r2, 2, 2)
KERN(k_128x64_sd2_o2, 8, 4, 2, 2)
KERN(k_128x64_sd4_o1, 8, 4, 4, 1)
KERN(k_128x128_sd2_o1, 8, 8, 2, 1)
KERN(k_128x128_sd1_o1, 8, 8, 1, 1)

int main() {
  const int S = 192;
  const size_t mat = 2048ull * 2048;
  double* P;
  if (hipMalloc(&P, S * mat * 8) != hipSuccess) return 1;
  std::vector<double> h(mat);
  for (size_t i = 0; i < mat; ++i) h[i] = ((i * 2654435761ull) % 1000) / 1000.0 - 0.5;
  for (int s = 0; s < S; ++s) (void)hipMemcpy(P + s * mat, h.data(), mat * 8, hipMemcpyHostToDevice);
  double* C;
  if (hipMalloc(&C, (size_t)S * 1024 * 1024 * 8) != hipSuccess) return 1;
  std::vector<double> ref((size_t)1024 * 1024), got((size_t)1024 * 1024);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  struct V { const char* name; const void* f; int WM, WN; };
  V vs[] = {{"64x64 sd4 o2 (no barriers)", (const void*)k_64x64_sd4_o2, 4, 4},
            {"64x64 sd2 o2 sb (library)", (const void*)k_64x64_sb2_o2, 4, 4},
            {"ring sd2 r2", (const void*)k_ring_sd2_r2, 4, 4},
            {"ring sd2 r3", (const void*)k_ring_sd2_r3, 4, 4},
            {"ring sd1 r4", (const void*)k_ring_sd1_r4, 4, 4},
            {"ring sd1 r3", (const void*)k_ring_sd1_r3, 4, 4}};
  for (int K : {1024, 512, 256, 128}) {
    bool first = true;
    for (auto& v : vs) {
      const int nbr = 1024 / (32 * v.WM), nbc = 1024 / (32 * v.WN), T = nbr * nbc;
      const int grid = 8 * ((S + 7) / 8) * T;
      int Tm = T, nb = nbr, Km = K, Sm = S;
      void* a2[] = {&P, &C, &Tm, &nb, &Km, &Sm};
      (void)hipMemset(C, 0, (size_t)S * 1024 * 1024 * 8);
      (void)hipLaunchKernel(v.f, dim3(grid), dim3(256), a2, 0, 0);
      (void)hipDeviceSynchronize();
      // slot 77's panel against the first variant's
      (void)hipMemcpy(first ? ref.data() : got.data(), C + (size_t)77 * 1024 * 1024, ref.size() * 8, hipMemcpyDeviceToHost);
      double md = 0.0;
      if (!first)
        for (size_t i = 0; i < ref.size(); ++i) md = fmax(md, fabs(ref[i] - got[i]));
      first = false;
      (void)hipEventRecord(e0);
      const int reps = 5;
      for (int r = 0; r < reps; ++r) (void)hipLaunchKernel(v.f, dim3(grid), dim3(256), a2, 0, 0);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      ms /= reps;
      const double fl = 2.0 * 1024 * 1024 * (double)K * S;
      printf("K=%4d %-24s grid=%6d %8.3f ms %6.2f TF/s  maxdiff %.3g\n", K, v.name, grid, ms, fl / ms / 1e9, md);
      fflush(stdout);
    }
  }
  printf("err=%s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
