// fp64 MFMA direct-from-L2 GEMM cores: wave-tile / staging / occupancy variants on the GP hot
// path's batched shapes (C = A B^T, panels of column-major ld=2048 matrices, one output panel
// per slot).  Prints TF/s per variant and shape.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double d4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ d4 mfma(double a, double b, d4 c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }

template <int WM, int WN>
struct Frag { double a[4][WM], b[4][WN]; };
template <int WM, int WN>
__device__ __forceinline__ void fload(Frag<WM, WN>& f, const double* pa, const double* pb, size_t sa, size_t sb) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
#pragma unroll
    for (int a = 0; a < WM; ++a) f.a[s][a] = pa[s * sa + 16 * a];
#pragma unroll
    for (int b = 0; b < WN; ++b) f.b[s][b] = pb[s * sb + 16 * b];
  }
}
template <int WM, int WN>
__device__ __forceinline__ void fmma(d4 (&acc)[WM][WN], const Frag<WM, WN>& f) {
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int a = 0; a < WM; ++a)
#pragma unroll
      for (int b = 0; b < WN; ++b) acc[a][b] = mfma(f.b[s][b], f.a[s][a], acc[a][b]);
}
template <int WM, int WN, int DB>
__device__ __forceinline__ void core(d4 (&acc)[WM][WN], const double* A, size_t lda, const double* B, size_t ldb, int K) {
  const int nst = __builtin_amdgcn_readfirstlane(K >> 4);
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const double* pa = A + lr + (size_t)lk * lda;
  const double* pb = B + lr + (size_t)lk * ldb;
  const size_t sa = 4 * lda, sb = 4 * ldb;
  if constexpr (DB == 0) {
    for (int it = 0; it < nst; ++it) {
      Frag<WM, WN> f;
      fload(f, pa + (size_t)it * 4 * sa, pb + (size_t)it * 4 * sb, sa, sb);
      fmma(acc, f);
    }
  } else {
    Frag<WM, WN> f0, f1;
    fload(f0, pa, pb, sa, sb);
    for (int it = 0; it < nst; it += 2) {
      fload(f1, pa + (size_t)(it + 1) * 4 * sa, pb + (size_t)(it + 1) * 4 * sb, sa, sb);
      fmma(acc, f0);
      const int n2 = (it + 2 < nst) ? it + 2 : nst - 1;
      fload(f0, pa + (size_t)n2 * 4 * sa, pb + (size_t)n2 * 4 * sb, sa, sb);
      fmma(acc, f1);
    }
  }
}

// WG = 4 waves (2 x 2), wave tile (16 WM) x (16 WN); WG tile (32 WM) x (32 WN).
// grid: 8-XCD slot mapping as the library (slot s on blocks b = s mod 8).
template <int WM, int WN, int DB>
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
  core<WM, WN, DB>(acc, M + r0, 2048, M + c0, 2048, K);
  // store into C (per slot 1024 x 1024 column-major, ld 1024)
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
#define KERN(NAME, WM, WN, DB, OCC)                                                                   \
  __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, OCC))) void NAME(         \
      const double* P, double* C, int T, int nbr, int K, int S) {                                     \
    body<WM, WN, DB>(P, C, T, nbr, K, S);                                                             \
  }
KERN(k_a_4x2_s1_o4, 4, 2, 0, 4)
KERN(k_b_4x4_s1_o2, 4, 4, 0, 2)
KERN(k_c_4x4_db_o2, 4, 4, 1, 2)
KERN(k_d_2x2_s1_o8, 2, 2, 0, 8)
KERN(k_d2_2x2_s1_o6, 2, 2, 0, 6)
KERN(k_e_4x2_db_o3, 4, 2, 1, 3)
KERN(k_f_2x4_s1_o4, 2, 4, 0, 4)
KERN(k_g_4x1_s1_o6, 4, 1, 0, 6)

// TRSM-like: 16 x 16 output tiles per slot, unit = 4 rows x 1 column (waves = rows), K = (tj+1) 64.
// fold = 0: units ordered by column descending (longest first); fold = 1: a unit does column j and
// then column 15 - j (equal total K per workgroup).
template <int FOLD>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_tri(const double* P, double* C, int T, int S) {
  const int x = blockIdx.x & 7, q = blockIdx.x >> 3;
  const int slot = (q / T) * 8 + x, u = q % T;
  if (slot >= S) return;
  const double* M = P + (size_t)slot * 2048 * 2048;
  double* Cs = C + (size_t)slot * 1024 * 1024;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const int CU = FOLD ? 8 : 16;
  const int pi = u / CU, pj = u - pi * CU;
  const int ti = 4 * pi + w;
  for (int pass = 0; pass < (FOLD ? 2 : 1); ++pass) {
    const int tj = FOLD ? (pass == 0 ? 15 - pj : pj) : 15 - pj;
    d4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = (d4){0, 0, 0, 0};
    core<4, 4, 1>(acc, M + 1024 + ti * 64, 2048, M + tj * 64, 2048, (tj + 1) * 64);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) Cs[(size_t)(tj * 64 + 16 * b + lk + 4 * qq) * 1024 + ti * 64 + 16 * a + lr] = acc[a][b][qq];
  }
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
  struct V { const char* name; const void* f; int WM, WN; };
  V vs[] = {{"4x2 s1 o4 (library)", (const void*)k_a_4x2_s1_o4, 4, 2}, {"4x4 s1 o2", (const void*)k_b_4x4_s1_o2, 4, 4},
            {"4x4 db o2", (const void*)k_c_4x4_db_o2, 4, 4},        {"2x2 s1 o8", (const void*)k_d_2x2_s1_o8, 2, 2},
            {"2x2 s1 o6", (const void*)k_d2_2x2_s1_o6, 2, 2},       {"4x2 db o3", (const void*)k_e_4x2_db_o3, 4, 2},
            {"2x4 s1 o4", (const void*)k_f_2x4_s1_o4, 2, 4},        {"4x1 s1 o6", (const void*)k_g_4x1_s1_o6, 4, 1}};
  for (int K : {1024, 512, 256}) {
    for (auto& v : vs) {
      const int nbr = 1024 / (32 * v.WM), nbc = 1024 / (32 * v.WN), T = nbr * nbc;
      const int grid = 8 * ((S + 7) / 8) * T;
      void* args[] = {&P, &C, (void*)&T, (void*)&nbr, &K, (void*)&S};
      int Tm = T, nb = nbr, Km = K, Sm = S;
      void* a2[] = {&P, &C, &Tm, &nb, &Km, &Sm};
      (void)args;
      (void)hipLaunchKernel(v.f, dim3(grid), dim3(256), a2, 0, 0);
      (void)hipEventRecord(e0);
      const int reps = 5;
      for (int r = 0; r < reps; ++r) (void)hipLaunchKernel(v.f, dim3(grid), dim3(256), a2, 0, 0);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      ms /= reps;
      const double fl = 2.0 * 1024 * 1024 * (double)K * S;
      printf("K=%4d %-22s grid=%6d %8.3f ms %6.2f TF/s\n", K, v.name, grid, ms, fl / ms / 1e9);
    }
  }
  for (int fold = 0; fold < 2; ++fold) {
    int T = fold ? 4 * 8 : 4 * 16, Sm = S;
    const int grid = 8 * ((S + 7) / 8) * T;
    const void* f = fold ? (const void*)k_tri<1> : (const void*)k_tri<0>;
    void* a2[] = {&P, &C, &T, &Sm};
    (void)hipLaunchKernel(f, dim3(grid), dim3(256), a2, 0, 0);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) (void)hipLaunchKernel(f, dim3(grid), dim3(256), a2, 0, 0);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    const double fl = 2.0 * 1024 * 64 * 64.0 * (16 * 17 / 2) * S;
    printf("TRSM-like tri K fold=%d grid=%6d %8.3f ms %6.2f TF/s\n", fold, grid, ms, fl / ms / 1e9);
  }
  printf("err=%s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
