// Is the library's 64 x 64 fp64 wave core (mma_64x64: two register stages of depth 8, group
// barriers interleaving one load per two MFMAs, 2 waves/SIMD) bound by operand latency or by its
// instruction stream?  The same core, timed on 192 batched 1024 x 1024 x K panels (ld 2048), with
// operands from (a) each slot's own panels (the library's case: L2 misses to MALL / HBM), (b) one
// 64-row panel pair shared by every wave on the chip (L2-hot), (c) no loads at all (the stage
// registers rotate; same MFMA stream and loop).  Against the steady-state ceiling of
// scratch/mfma_ceiling.hip (64 cycles per MFMA per SIMD at 2 waves/SIMD: 77.2 TF/s at 2.39 GHz).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double d4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ d4 mfma(double a, double b, d4 c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }
constexpr int QM = 4, QN = 4, SD = 2;
struct F4 {
  double a[SD][QM], b[SD][QN];
};
template <bool LOAD>
__device__ __forceinline__ void fload(F4& f, const double* pa, const double* pb, ptrdiff_t sa, ptrdiff_t sb) {
#pragma unroll
  for (int s = 0; s < SD; ++s) {
#pragma unroll
    for (int a = 0; a < QM; ++a) f.a[s][a] = LOAD ? pa[s * sa + 16 * a] : f.a[s][a] * 0.999;
#pragma unroll
    for (int b = 0; b < QN; ++b) f.b[s][b] = LOAD ? pb[s * sb + 16 * b] : f.b[s][b] * 1.001;
  }
}
__device__ __forceinline__ void fmma(d4 (&acc)[QM][QN], const F4& f) {
#pragma unroll
  for (int s = 0; s < SD; ++s)
#pragma unroll
    for (int a = 0; a < QM; ++a)
#pragma unroll
      for (int b = 0; b < QN; ++b) acc[a][b] = mfma(f.b[s][b], f.a[s][a], acc[a][b]);
}
template <bool LOAD>
__device__ __forceinline__ void core(d4 (&acc)[QM][QN], const double* A, size_t lda, const double* B, size_t ldb, int K) {
  const int nst = __builtin_amdgcn_readfirstlane(K / (4 * SD));
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const double* pa = A + lr + (ptrdiff_t)lk * lda;
  const double* pb = B + lr + (ptrdiff_t)lk * ldb;
  const ptrdiff_t sa = 4 * (ptrdiff_t)lda, sb = 4 * (ptrdiff_t)ldb;
  F4 f0, f1;
  fload<true>(f0, pa, pb, sa, sb);
  f1 = f0;
  for (int it = 0; it < nst; it += 2) {
    __builtin_amdgcn_sched_barrier(0);
    fload<LOAD>(f1, pa + (ptrdiff_t)(it + 1) * SD * sa, pb + (ptrdiff_t)(it + 1) * SD * sb, sa, sb);
    fmma(acc, f0);
#pragma unroll
    for (int g = 0; g < SD * (QM + QN); ++g) {
      __builtin_amdgcn_sched_group_barrier(LOAD ? 0x020 : 0x002, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    const int n2 = (it + 2 < nst) ? it + 2 : nst - 1;
    fload<LOAD>(f0, pa + (ptrdiff_t)n2 * SD * sa, pb + (ptrdiff_t)n2 * SD * sb, sa, sb);
    fmma(acc, f1);
#pragma unroll
    for (int g = 0; g < SD * (QM + QN); ++g) {
      __builtin_amdgcn_sched_group_barrier(LOAD ? 0x020 : 0x002, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}
// MODE 0: own panels; 1: one shared L2-hot 64-row panel pair; 2: no loads in the loop
template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_core(const double* P, double* C, int T,
                                                                                          int nbr, int K, int S) {
  const int x = blockIdx.x & 7, q = blockIdx.x >> 3;
  const int slot = (q / T) * 8 + x, u = q % T;
  if (slot >= S) return;
  const int bi = u % nbr, bj = u / nbr;
  const double* M = P + (MODE == 1 ? 0 : (size_t)slot * 2048 * 2048);
  const int w = threadIdx.x >> 6, wr = w >> 1, wc = w & 1;
  d4 acc[QM][QN];
#pragma unroll
  for (int a = 0; a < QM; ++a)
#pragma unroll
    for (int b = 0; b < QN; ++b) acc[a][b] = (d4){0, 0, 0, 0};
  const int r0 = 1024 + bi * 128 + 64 * wr, c0 = bj * 128 + 64 * wc;
  const int ra = MODE == 1 ? 1024 : r0, cb = MODE == 1 ? 0 : c0;
  core<MODE != 2>(acc, M + ra, 2048, M + cb, 2048, K);
  double* Cs = C + (size_t)slot * 1024 * 1024;
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
#pragma unroll
  for (int a = 0; a < QM; ++a)
#pragma unroll
    for (int b = 0; b < QN; ++b)
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) Cs[(size_t)(c0 + 16 * b + lk + 4 * qq) * 1024 + (r0 - 1024) + 16 * a + lr] = acc[a][b][qq];
}

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
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  struct V {
    const char* name;
    const void* f;
  };
  V vs[] = {{"own panels (library case)", (const void*)k_core<0>},
            {"one shared panel (L2-hot)", (const void*)k_core<1>},
            {"no loads in the loop", (const void*)k_core<2>}};
  for (int K : {1024, 256}) {
    for (auto& v : vs) {
      const int nbr = 8, T = 64;
      const int grid = 8 * ((S + 7) / 8) * T;
      int Tm = T, nb = nbr, Km = K, Sm = S;
      void* a2[] = {&P, &C, &Tm, &nb, &Km, &Sm};
      for (int r = 0; r < 20; ++r) (void)hipLaunchKernel(v.f, dim3(grid), dim3(256), a2, 0, 0);  // warm-up
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0);
      const int reps = 10;
      for (int r = 0; r < reps; ++r) (void)hipLaunchKernel(v.f, dim3(grid), dim3(256), a2, 0, 0);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      ms /= reps;
      const double fl = 2.0 * 1024 * 1024 * (double)K * S;
      printf("K=%4d %-28s %8.3f ms %6.2f TF/s\n", K, v.name, ms, fl / ms / 1e9);
      fflush(stdout);
    }
  }
  printf("err=%s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
