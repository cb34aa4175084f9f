// fp64 MFMA GEMM cores on the GP hot path's batched shapes (C = A B^T, panels of column-major
// ld=2048 matrices, 192 slots, random operands): the library's register-direct 64x64 wave core
// (each wave streams its own A and B panels from L2) against an LDS-staged workgroup core (the
// 4 waves of a UR x UC unit share one A panel of 64 UR rows and one B panel of 64 UC rows,
// double-buffered global_load_lds stages of KS columns).  Prints ms and TF/s per variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double d4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ d4 mfma(double a, double b, d4 c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }

struct Frag4 { double a[4][4], b[4][4]; };
__device__ __forceinline__ void f4load(Frag4& f, const double* pa, const double* pb, size_t sa, size_t sb) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
#pragma unroll
    for (int a = 0; a < 4; ++a) f.a[s][a] = pa[s * sa + 16 * a];
#pragma unroll
    for (int b = 0; b < 4; ++b) f.b[s][b] = pb[s * sb + 16 * b];
  }
}
__device__ __forceinline__ void f4mma(d4 (&acc)[4][4], const Frag4& f) {
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = mfma(f.b[s][b], f.a[s][a], acc[a][b]);
}
// library core (gprx_kernels.hip mma_64x64)
__device__ __forceinline__ void core_reg(d4 (&acc)[4][4], const double* A, size_t lda, const double* B, size_t ldb, int K) {
  const int nst = __builtin_amdgcn_readfirstlane(K >> 4);
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const double* pa = A + lr + (size_t)lk * lda;
  const double* pb = B + lr + (size_t)lk * ldb;
  const size_t sa = 4 * lda, sb = 4 * ldb;
  Frag4 f0, f1;
  f4load(f0, pa, pb, sa, sb);
  for (int it = 0; it < nst; it += 2) {
    f4load(f1, pa + (size_t)(it + 1) * 4 * sa, pb + (size_t)(it + 1) * 4 * sb, sa, sb);
    f4mma(acc, f0);
    const int n2 = (it + 2 < nst) ? it + 2 : nst - 1;
    f4load(f0, pa + (size_t)n2 * 4 * sa, pb + (size_t)n2 * 4 * sb, sa, sb);
    f4mma(acc, f1);
  }
}

// ---- LDS-staged block core ------------------------------------------------------------------
// Unit UR x UC waves; wave (wr, wc) computes rows 64 wr.. of the A panel against rows 64 wc.. of
// the B panel.  Stage = KS columns of both panels in LDS, column stride AR + 16 / BR + 16 doubles
// (the 16-double pad shifts consecutive columns by 32 banks: the two k rows a ds_read_b64 lane
// group touches never share a bank).  Each global_load_lds moves one 1 KiB run (128 rows) of
// one column; the waves take the (KS (UR + UC) / 2) runs of a stage round robin.
template <int UR, int UC, int KS>
struct Blk {
  static constexpr int AR = 64 * UR, BR = 64 * UC, AST = AR + 16, BST = BR + 16;
  static constexpr int STG = KS * (AST + BST);              // doubles per stage
  static constexpr int RUNS = KS * (UR + UC) / 2;           // 1 KiB runs per stage
  static constexpr int LDS = 2 * STG;                       // double-buffered
};
template <int UR, int UC, int KS>
__device__ __forceinline__ void blk_issue(const double* A, size_t lda, const double* B, size_t ldb, int k0, double* buf) {
  using P = Blk<UR, UC, KS>;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < P::RUNS / 4; ++j) {
    const int run = 4 * j + w;
    const double* src;
    double* dst;
    if (run < KS * UR / 2) {  // A: column c = run / (UR/2), 128-row half h
      const int c = run / (UR / 2), h = run - c * (UR / 2);
      src = A + (size_t)(k0 + c) * lda + 128 * h;
      dst = buf + c * P::AST + 128 * h;
    } else {
      const int rb = run - KS * UR / 2;
      const int c = rb / (UC / 2), h = rb - c * (UC / 2);
      src = B + (size_t)(k0 + c) * ldb + 128 * h;
      dst = buf + KS * P::AST + c * P::BST + 128 * h;
    }
    __builtin_amdgcn_global_load_lds((const void*)(src + 2 * l), (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
  }
}
template <int UR, int UC, int KS>
__device__ __forceinline__ void blk_core(d4 (&acc)[4][4], const double* A, size_t lda, const double* B, size_t ldb, int K,
                                         double* lds, bool compute) {
  using P = Blk<UR, UC, KS>;
  const int nst = K / KS;
  const int w = threadIdx.x >> 6, wr = w / UC, wc = w - wr * UC;
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  blk_issue<UR, UC, KS>(A, lda, B, ldb, 0, lds);
  for (int it = 0; it < nst; ++it) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    double* cur = lds + (it & 1) * P::STG;
    if (it + 1 < nst) blk_issue<UR, UC, KS>(A, lda, B, ldb, (it + 1) * KS, lds + ((it + 1) & 1) * P::STG);
    if (compute) {
      const double* pa = cur + 64 * wr + lr + lk * P::AST;
      const double* pb = cur + KS * P::AST + 64 * wc + lr + lk * P::BST;
#pragma unroll
      for (int s = 0; s < KS / 4; ++s) {
        double fa[4], fb[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) fa[a] = pa[4 * s * P::AST + 16 * a];
#pragma unroll
        for (int b = 0; b < 4; ++b) fb[b] = pb[4 * s * P::BST + 16 * b];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) acc[a][b] = mfma(fb[b], fa[a], acc[a][b]);
      }
    }
  }
}

__device__ __forceinline__ void store(double* Cs, int r0, int c0, const d4 (&acc)[4][4]) {
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) Cs[(size_t)(c0 + 16 * b + lk + 4 * qq) * 1024 + r0 + 16 * a + lr] = acc[a][b][qq];
}
__device__ __forceinline__ void zero(d4 (&acc)[4][4]) {
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = (d4){0, 0, 0, 0};
}

// C(1024 x 1024) = A B^T with A rows 1024.. and B rows 0.. of each slot's 2048 x 2048 matrix;
// unit UR x UC tiles of 64; slot s on blocks b = s mod 8
template <int UR, int UC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_reg(const double* P, double* C, int K, int S) {
  constexpr int NBR = 16 / UR, NBC = 16 / UC, T = NBR * NBC;
  const int x = blockIdx.x & 7, q = blockIdx.x >> 3;
  const int slot = (q / T) * 8 + x, u = q % T;
  if (slot >= S) return;
  const int bi = u % NBR, bj = u / NBR;
  const double* M = P + (size_t)slot * 2048 * 2048;
  const int w = threadIdx.x >> 6, wr = w / UC, wc = w - wr * UC;
  d4 acc[4][4];
  zero(acc);
  const int r0 = 64 * (UR * bi + wr), c0 = 64 * (UC * bj + wc);
  core_reg(acc, M + 1024 + r0, 2048, M + c0, 2048, K);
  store(C + (size_t)slot * 1024 * 1024, r0, c0, acc);
}
template <int UR, int UC, int KS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_lds(const double* P, double* C, int K, int S) {
  constexpr int NBR = 16 / UR, NBC = 16 / UC, T = NBR * NBC;
  __shared__ __attribute__((aligned(16))) double lds[Blk<UR, UC, KS>::LDS];
  const int x = blockIdx.x & 7, q = blockIdx.x >> 3;
  const int slot = (q / T) * 8 + x, u = q % T;
  if (slot >= S) return;
  const int bi = u % NBR, bj = u / NBR;
  const double* M = P + (size_t)slot * 2048 * 2048;
  const int w = threadIdx.x >> 6, wr = w / UC, wc = w - wr * UC;
  d4 acc[4][4];
  zero(acc);
  blk_core<UR, UC, KS>(acc, M + 1024 + 64 * UR * bi, 2048, M + 64 * UC * bj, 2048, K, lds, true);
  store(C + (size_t)slot * 1024 * 1024, 64 * (UR * bi + wr), 64 * (UC * bj + wc), acc);
}

__global__ void k_fill(double* P, size_t n, unsigned long long seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned long long z = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    P[i] = (double)(z >> 11) * (1.0 / 9007199254740992.0) - 0.5;
  }
}

int main() {
  const int S = 192;
  const size_t mat = 2048ull * 2048;
  double *P, *C, *C2;
  if (hipMalloc(&P, S * mat * 8) != hipSuccess) return 1;
  if (hipMalloc(&C, (size_t)S * 1024 * 1024 * 8) != hipSuccess) return 1;
  if (hipMalloc(&C2, (size_t)S * 1024 * 1024 * 8) != hipSuccess) return 1;
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, P, S * mat, 12345ull);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  struct V { const char* name; const void* f; int UR, UC; };
  V vs[] = {{"reg 2x2 (library)", (const void*)k_reg<2, 2>, 2, 2},
            {"reg 4x1", (const void*)k_reg<4, 1>, 4, 1},
            {"lds 2x2 ks16", (const void*)k_lds<2, 2, 16>, 2, 2},
            {"lds 2x2 ks8", (const void*)k_lds<2, 2, 8>, 2, 2},
            {"lds 4x1 ks8", (const void*)k_lds<4, 1, 8>, 4, 1},
            {"lds 2x2 ks32", (const void*)k_lds<2, 2, 32>, 2, 2}};
  std::vector<double> h1((size_t)1024 * 1024), h2((size_t)1024 * 1024);
  for (int K : {1024, 512, 256, 128}) {
    for (auto& v : vs) {
      const int T = (16 / v.UR) * (16 / v.UC);
      const int grid = 8 * ((S + 7) / 8) * T;
      int Km = K, Sm = S;
      double* out = (&v == &vs[0]) ? C : C2;
      void* a2[] = {&P, &out, &Km, &Sm};
      (void)hipLaunchKernel(v.f, dim3(grid), dim3(256), a2, 0, 0);
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0);
      const int reps = 5;
      for (int r = 0; r < reps; ++r) (void)hipLaunchKernel(v.f, dim3(grid), dim3(256), a2, 0, 0);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      ms /= reps;
      double maxd = 0.0;
      if (out == C2) {  // same products as the library core (summation order differs: none here)
        (void)hipMemcpy(h1.data(), C + (size_t)7 * 1024 * 1024, h1.size() * 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(h2.data(), C2 + (size_t)7 * 1024 * 1024, h2.size() * 8, hipMemcpyDeviceToHost);
        for (size_t i = 0; i < h1.size(); ++i) maxd = fmax(maxd, fabs(h1[i] - h2[i]));
      }
      const double fl = 2.0 * 1024 * 1024 * (double)K * S;
      printf("K=%4d %-20s grid=%6d %8.3f ms %6.2f TF/s  maxdiff %.3g\n", K, v.name, grid, ms, fl / ms / 1e9, maxd);
    }
  }
  printf("err=%s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
