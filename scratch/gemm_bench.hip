// Microbenchmark of fp64 MFMA tile-GEMM cores for the GP hot path: C = A B^T, A/B row panels of
// column-major 2048x2048 matrices, many independent tiles (batched), K deep.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cstdlib>
typedef double d4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ d4 mfma(double a, double b, d4 c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }

// ---------------- V0: direct global fragments (current library core) ----------------
__device__ __forceinline__ void mma_abt(d4 (&acc)[2][2], const double* __restrict__ A, size_t lda,
                                        const double* __restrict__ B, size_t ldb, int K) {
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const double* pa = A + lr + (size_t)lk * lda;
  const double* pb = B + lr + (size_t)lk * ldb;
  const size_t sa = 4 * lda, sb = 4 * ldb;
  double a0[4], a1[4], b0[4], b1[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) { a0[s] = pa[s * sa]; a1[s] = pa[s * sa + 16]; b0[s] = pb[s * sb]; b1[s] = pb[s * sb + 16]; }
  const int nst = K >> 4;
  for (int it = 1; it < nst; ++it) {
    pa += 4 * sa; pb += 4 * sb;
    double na0[4], na1[4], nb0[4], nb1[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) { na0[s] = pa[s * sa]; na1[s] = pa[s * sa + 16]; nb0[s] = pb[s * sb]; nb1[s] = pb[s * sb + 16]; }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      acc[0][0] = mfma(b0[s], a0[s], acc[0][0]); acc[0][1] = mfma(b1[s], a0[s], acc[0][1]);
      acc[1][0] = mfma(b0[s], a1[s], acc[1][0]); acc[1][1] = mfma(b1[s], a1[s], acc[1][1]);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) { a0[s] = na0[s]; a1[s] = na1[s]; b0[s] = nb0[s]; b1[s] = nb1[s]; }
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    acc[0][0] = mfma(b0[s], a0[s], acc[0][0]); acc[0][1] = mfma(b1[s], a0[s], acc[0][1]);
    acc[1][0] = mfma(b0[s], a1[s], acc[1][0]); acc[1][1] = mfma(b1[s], a1[s], acc[1][1]);
  }
}

__global__ __launch_bounds__(256) void k_v0(const double* P, double* C, int T, int nblk, int K) {
  const int slot = blockIdx.x / T, t = blockIdx.x % T;
  const int bi = t % nblk, bj = (t / nblk) % nblk;
  const double* M = P + (size_t)slot * 2048 * 2048;
  const int w = threadIdx.x >> 6, wr = w >> 1, wc = w & 1;
  d4 acc[2][2];
  for (int a = 0; a < 2; ++a) for (int b = 0; b < 2; ++b) acc[a][b] = (d4){0, 0, 0, 0};
  mma_abt(acc, M + bi * 64 + 32 * wr, 2048, M + bj * 64 + 32 * wc, 2048, K);
  const int l = threadIdx.x & 63;
  double s = 0;
  for (int a = 0; a < 2; ++a) for (int b = 0; b < 2; ++b) for (int q = 0; q < 4; ++q) s += acc[a][b][q];
  C[(size_t)blockIdx.x * 256 + threadIdx.x] = s;
}

// ---------------- LDS-staged cores ----------------
// WG = 4 waves (2x2). Wave tile = (16*WM) x (16*WN). WG tile RA = 32*WM rows of A, RB = 32*WN rows of B.
// Stage = KS k-columns. LDS image per stage: [k][row] with row stride SA = RA + 16 (doubles).
template <int WM, int WN, int KS>
struct Core {
  static constexpr int RA = 32 * WM, RB = 32 * WN;
  static constexpr int SA = RA + 16, SB = RB + 16;
  static constexpr int STAGE = KS * (SA + SB);           // doubles per stage
  static constexpr int LA = RA * KS / 2 / 256;           // dwordx4 per thread for A per stage
  static constexpr int LB = RB * KS / 2 / 256;
  static_assert(LA >= 1 && LB >= 1, "stage too small");

  __device__ static void run(d4 (&acc)[WM][WN], const double* __restrict__ A, size_t lda,
                             const double* __restrict__ B, size_t ldb, int K, double* lds) {
    const int tid = threadIdx.x, w = tid >> 6, wr = w >> 1, wc = w & 1;
    const int l = tid & 63, lr = l & 15, lk = l >> 4;
    // global load mapping: element pair (row 2*(e % (R/2)), col e / (R/2)), e = tid + 256*i
    double2 ra[LA], rb[LB];
    auto gload = [&](int k0) {
#pragma unroll
      for (int i = 0; i < LA; ++i) {
        const int e = tid + 256 * i, c = e / (RA / 2), r = 2 * (e % (RA / 2));
        ra[i] = *(const double2*)(A + (size_t)(k0 + c) * lda + r);
      }
#pragma unroll
      for (int i = 0; i < LB; ++i) {
        const int e = tid + 256 * i, c = e / (RB / 2), r = 2 * (e % (RB / 2));
        rb[i] = *(const double2*)(B + (size_t)(k0 + c) * ldb + r);
      }
    };
    auto swrite = [&](double* buf) {
#pragma unroll
      for (int i = 0; i < LA; ++i) {
        const int e = tid + 256 * i, c = e / (RA / 2), r = 2 * (e % (RA / 2));
        *(double2*)(buf + c * SA + r) = ra[i];
      }
      double* bb = buf + KS * SA;
#pragma unroll
      for (int i = 0; i < LB; ++i) {
        const int e = tid + 256 * i, c = e / (RB / 2), r = 2 * (e % (RB / 2));
        *(double2*)(bb + c * SB + r) = rb[i];
      }
    };
    auto compute = [&](const double* buf) {
      const double* pa = buf + lk * SA + wr * 16 * WM + lr;
      const double* pb = buf + KS * SA + lk * SB + wc * 16 * WN + lr;
#pragma unroll
      for (int s = 0; s < KS / 4; ++s) {
        double af[WM], bf[WN];
#pragma unroll
        for (int a = 0; a < WM; ++a) af[a] = pa[s * 4 * SA + 16 * a];
#pragma unroll
        for (int b = 0; b < WN; ++b) bf[b] = pb[s * 4 * SB + 16 * b];
#pragma unroll
        for (int a = 0; a < WM; ++a)
#pragma unroll
          for (int b = 0; b < WN; ++b) acc[a][b] = mfma(bf[b], af[a], acc[a][b]);
      }
    };
    const int nst = K / KS;
    gload(0);
    swrite(lds);
    __syncthreads();
    for (int st = 0; st < nst; ++st) {
      double* cur = lds + (st & 1) * STAGE;
      double* nxt = lds + ((st + 1) & 1) * STAGE;
      if (st + 1 < nst) gload((st + 1) * KS);
      compute(cur);
      if (st + 1 < nst) swrite(nxt);
      __syncthreads();
    }
  }
};

template <int WM, int WN, int KS>
__global__ __launch_bounds__(256) void k_lds(const double* P, double* C, int T, int nblkA, int nblkB, int K) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  using CO = Core<WM, WN, KS>;
  const int slot = blockIdx.x / T, t = blockIdx.x % T;
  const int bi = t % nblkA, bj = (t / nblkA) % nblkB;
  const double* M = P + (size_t)slot * 2048 * 2048;
  d4 acc[WM][WN];
  for (int a = 0; a < WM; ++a) for (int b = 0; b < WN; ++b) acc[a][b] = (d4){0, 0, 0, 0};
  CO::run(acc, M + bi * CO::RA, 2048, M + bj * CO::RB, 2048, K, lds);
  double s = 0;
  for (int a = 0; a < WM; ++a) for (int b = 0; b < WN; ++b) for (int q = 0; q < 4; ++q) s += acc[a][b][q];
  C[(size_t)blockIdx.x * 256 + threadIdx.x] = s;
}


// ---------------- direct variants: wave tile WM x WN (16-blocks), WG 2x2 waves, prefetch depth PF stages of 16 ----
template <int WM, int WN, int PF>
__device__ __forceinline__ void mma_dir(d4 (&acc)[WM][WN], const double* __restrict__ A, size_t lda,
                                        const double* __restrict__ B, size_t ldb, int K) {
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const double* pa = A + lr + (size_t)lk * lda;
  const double* pb = B + lr + (size_t)lk * ldb;
  const size_t sa = 4 * lda, sb = 4 * ldb;
  double af[PF + 1][4][WM], bf[PF + 1][4][WN];
  const int nst = K >> 4;
#pragma unroll
  for (int p = 0; p < PF; ++p)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int a = 0; a < WM; ++a) af[p][s][a] = pa[(p * 4 + s) * sa + 16 * a];
#pragma unroll
      for (int b = 0; b < WN; ++b) bf[p][s][b] = pb[(p * 4 + s) * sb + 16 * b];
    }
  for (int it = 0; it < nst; it += PF + 1) {
    // stages it .. it+PF: slot p holds stage it+p for p < PF; load stage it+PF into slot PF
#pragma unroll
    for (int q = 0; q <= PF; ++q) {
      const int ld_st = it + q + PF;   // stage to load now
      const int slot_ld = (q + PF) % (PF + 1);
      if (ld_st < nst) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
#pragma unroll
          for (int a = 0; a < WM; ++a) af[slot_ld][s][a] = pa[((size_t)ld_st * 4 + s) * sa + 16 * a];
#pragma unroll
          for (int b = 0; b < WN; ++b) bf[slot_ld][s][b] = pb[((size_t)ld_st * 4 + s) * sb + 16 * b];
        }
      }
      if (it + q < nst) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int a = 0; a < WM; ++a)
#pragma unroll
            for (int b = 0; b < WN; ++b) acc[a][b] = mfma(bf[q][s][b], af[q][s][a], acc[a][b]);
      }
    }
  }
}
template <int WM, int WN, int PF>
__global__ __launch_bounds__(256) void k_dir(const double* P, double* C, int T, int nblkA, int nblkB, int K) {
  const int slot = blockIdx.x / T, t = blockIdx.x % T;
  const int bi = t % nblkA, bj = (t / nblkA) % nblkB;
  const double* M = P + (size_t)slot * 2048 * 2048;
  const int w = threadIdx.x >> 6, wr = w >> 1, wc = w & 1;
  d4 acc[WM][WN];
  for (int a = 0; a < WM; ++a) for (int b = 0; b < WN; ++b) acc[a][b] = (d4){0, 0, 0, 0};
  mma_dir<WM, WN, PF>(acc, M + bi * 32 * WM + 16 * WM * wr, 2048, M + bj * 32 * WN + 16 * WN * wc, 2048, K);
  double s = 0;
  for (int a = 0; a < WM; ++a) for (int b = 0; b < WN; ++b) for (int q = 0; q < 4; ++q) s += acc[a][b][q];
  C[(size_t)blockIdx.x * 256 + threadIdx.x] = s;
}

// host reference check for one tile of V0 vs LDS (sum of acc) is implicit: compare C sums
int main(int argc, char** argv) {
  const int S = 48;
  size_t mat = 2048ull * 2048;
  double* P; hipMalloc(&P, S * mat * 8);
  std::vector<double> h(mat);
  for (size_t i = 0; i < mat; ++i) h[i] = ((i * 2654435761ull) % 1000) / 1000.0 - 0.5;
  for (int s = 0; s < S; ++s) hipMemcpy(P + s * mat, h.data(), mat * 8, hipMemcpyHostToDevice);
  double* C; hipMalloc(&C, 64ull << 20);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int K : {256, 1024, 2048}) {
    // V0
    {
      int T = 16; int nb = 32; int grid = S * T;
      hipLaunchKernelGGL(k_v0, dim3(grid), dim3(256), 0, 0, P, C, T, nb, K);
      hipEventRecord(e0);
      for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_v0, dim3(grid), dim3(256), 0, 0, P, C, T, nb, K);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 5;
      printf("K=%4d V0 direct 64x64  grid=%5d: %7.3f ms %6.2f TF\n", K, grid, ms, 2.0 * grid * 64 * 64 * K / ms / 1e9);
    }
#define RUNL(WM, WN, KS, T)                                                                                  \
    {                                                                                                        \
      using CO = Core<WM, WN, KS>;                                                                           \
      int grid = S * T; size_t sh = 2 * CO::STAGE * 8;                                                       \
      auto kf = k_lds<WM, WN, KS>;                                                                           \
      hipFuncSetAttribute((const void*)kf, hipFuncAttributeMaxDynamicSharedMemorySize, sh);                  \
      hipLaunchKernelGGL(kf, dim3(grid), dim3(256), sh, 0, P, C, T, 2048 / CO::RA, 2048 / CO::RB, K);        \
      hipEventRecord(e0);                                                                                    \
      for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kf, dim3(grid), dim3(256), sh, 0, P, C, T, 2048 / CO::RA, 2048 / CO::RB, K); \
      hipEventRecord(e1); hipEventSynchronize(e1);                                                           \
      float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 5;                                                   \
      printf("K=%4d LDS %3dx%3d KS=%2d grid=%5d lds=%6zu: %7.3f ms %6.2f TF\n", K, CO::RA, CO::RB, KS, grid, sh, ms, \
             2.0 * grid * CO::RA * CO::RB * K / ms / 1e9);                                                   \
    }

#define RUND(WM, WN, PF, T)                                                                                  \
    {                                                                                                        \
      int grid = S * T;                                                                                      \
      auto kf = k_dir<WM, WN, PF>;                                                                           \
      int nA = 2048 / (32 * WM), nB = 2048 / (32 * WN);                                                      \
      hipLaunchKernelGGL(kf, dim3(grid), dim3(256), 0, 0, P, C, T, nA, nB, K);                               \
      hipEventRecord(e0);                                                                                    \
      for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kf, dim3(grid), dim3(256), 0, 0, P, C, T, nA, nB, K);   \
      hipEventRecord(e1); hipEventSynchronize(e1);                                                           \
      float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 5;                                                   \
      printf("K=%4d DIR wave %dx%d PF=%d grid=%5d: %7.3f ms %6.2f TF\n", K, 16*WM, 16*WN, PF, grid, ms,     \
             2.0 * grid * 32*WM * 32*WN * K / ms / 1e9);                                                     \
    }
    RUND(2, 2, 1, 16)
    RUND(2, 2, 2, 16)
    RUND(2, 2, 1, 64)
    RUND(2, 4, 1, 8)
    RUND(2, 4, 1, 32)
    RUND(4, 2, 1, 32)
    RUND(4, 4, 1, 16)
    RUND(4, 4, 1, 4)
    RUND(2, 4, 2, 32)
  }
  hipError_t err = hipGetLastError();
  printf("err=%s\n", hipGetErrorString(err));
  return 0;
}
