// fp64 MFMA GEMM cores, round 2: global_load_lds (LDS-DMA) staged 128x128 workgroup tiles,
// triple-buffered with counted vmcnt, vs the direct 64x32-per-wave core used by the library.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cmath>
typedef double d4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ d4 mfma(double a, double b, d4 c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }

// ---------------- direct 64x32 wave core (library) ----------------
__device__ __forceinline__ void mma_64x32(d4 (&acc)[4][2], const double* __restrict__ A, size_t lda,
                                          const double* __restrict__ B, size_t ldb, int K) {
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const double* pa = A + lr + (size_t)lk * lda;
  const double* pb = B + lr + (size_t)lk * ldb;
  const size_t sa = 4 * lda, sb = 4 * ldb;
  double af[4][4], bf[4][2];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
#pragma unroll
    for (int a = 0; a < 4; ++a) af[s][a] = pa[s * sa + 16 * a];
#pragma unroll
    for (int b = 0; b < 2; ++b) bf[s][b] = pb[s * sb + 16 * b];
  }
  const int nst = K >> 4;
  for (int it = 1; it < nst; ++it) {
    pa += 4 * sa; pb += 4 * sb;
    double na[4][4], nb[4][2];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int a = 0; a < 4; ++a) na[s][a] = pa[s * sa + 16 * a];
#pragma unroll
      for (int b = 0; b < 2; ++b) nb[s][b] = pb[s * sb + 16 * b];
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = mfma(bf[s][b], af[s][a], acc[a][b]);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int a = 0; a < 4; ++a) af[s][a] = na[s][a];
#pragma unroll
      for (int b = 0; b < 2; ++b) bf[s][b] = nb[s][b];
    }
  }
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) acc[a][b] = mfma(bf[s][b], af[s][a], acc[a][b]);
}

// grid: S slots x T units; unit u -> (rows block bi = u % nbA, col block bj = u / nbA); K range [k0, k0+K)
// tri: K = (bj+1)*64 (triangular-like) else K fixed
__global__ __launch_bounds__(256) void k_dir(const double* P, double* C, int T, int nbA, int K, int tri) {
  const int x = blockIdx.x & 7, q = blockIdx.x >> 3;
  const int slot = (q / T) * 8 + x, u = q % T;
  const int bi = u % nbA, bj = u / nbA;
  const double* M = P + (size_t)slot * 2048 * 2048;
  const int w = threadIdx.x >> 6, wr = w >> 1, wc = w & 1;
  const int Kb = tri ? (bj + 1) * 64 : K;
  d4 acc[4][2];
  for (int a = 0; a < 4; ++a) for (int b = 0; b < 2; ++b) acc[a][b] = (d4){0, 0, 0, 0};
  mma_64x32(acc, M + 1024 + bi * 128 + 64 * wr, 2048, M + bj * 64 + 32 * wc, 2048, Kb);
  double s = 0;
  for (int a = 0; a < 4; ++a) for (int b = 0; b < 2; ++b) for (int q2 = 0; q2 < 4; ++q2) s += acc[a][b][q2];
  C[(size_t)blockIdx.x * 256 + threadIdx.x] = s;
}

// ---------------- LDS-DMA 128x128 core ----------------
// WG 4 waves (2x2), wave tile 64x64 (4x4 accumulators).  Stage = 16 k columns: A 128x16 and B 128x16
// doubles, each column (128 doubles = 1 KB) one global_load_lds_dwordx4 wave instruction.
// NB stages ring in one LDS array.
template <int NB>
__device__ __forceinline__ void mma_128x128_lds(d4 (&acc)[4][4], const double* __restrict__ A, size_t lda,
                                                const double* __restrict__ B, size_t ldb, int K, double* lds) {
  const int tid = threadIdx.x, w = tid >> 6, wr = w >> 1, wc = w & 1;
  const int l = tid & 63, lr = l & 15, lk = l >> 4;
  constexpr int STAGE = 2 * 16 * 128;  // doubles
  const int nst = K >> 4;
  // this wave loads columns 4w..4w+3 of A and of B in every stage
  auto issue = [&](int st) {
    double* buf = lds + (st % NB) * STAGE;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int kk = st * 16 + 4 * w + c;
      __builtin_amdgcn_global_load_lds((const void*)(A + (size_t)kk * lda + 2 * l),
                                       (__attribute__((address_space(3))) void*)(buf + (4 * w + c) * 128), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(B + (size_t)kk * ldb + 2 * l),
                                       (__attribute__((address_space(3))) void*)(buf + 16 * 128 + (4 * w + c) * 128), 16, 0, 0);
    }
  };
  for (int p = 0; p < NB - 1 && p < nst; ++p) issue(p);
  for (int st = 0; st < nst; ++st) {
    // wait for own loads of stage st: outstanding allowed = loads of later issued stages
    const int ahead = (nst - 1 - st) < (NB - 2) ? (nst - 1 - st) : (NB - 2);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // all waves' stage-st data landed; all done with stage st-1
    if (st + NB - 1 < nst) issue(st + NB - 1);  // into the buffer of stage st-1
    const double* buf = lds + (st % NB) * STAGE;
    const double* pa = buf + lk * 128 + 64 * wr + lr;
    const double* pb = buf + 16 * 128 + lk * 128 + 64 * wc + lr;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      double af[4], bf[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) af[a] = pa[s * 4 * 128 + 16 * a];
#pragma unroll
      for (int b = 0; b < 4; ++b) bf[b] = pb[s * 4 * 128 + 16 * b];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = mfma(bf[b], af[a], acc[a][b]);
    }
  }
}

template <int NB>
__global__ __launch_bounds__(256) void k_lds(const double* P, double* C, int T, int nbA, int K, int tri) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int x = blockIdx.x & 7, q = blockIdx.x >> 3;
  const int slot = (q / T) * 8 + x, u = q % T;
  const int bi = u % nbA, bj = u / nbA;
  const double* M = P + (size_t)slot * 2048 * 2048;
  const int Kb = tri ? (bj + 1) * 128 : K;
  d4 acc[4][4];
  for (int a = 0; a < 4; ++a) for (int b = 0; b < 4; ++b) acc[a][b] = (d4){0, 0, 0, 0};
  mma_128x128_lds<NB>(acc, M + 1024 + bi * 128, 2048, M + bj * 128, 2048, Kb, lds);
  double s = 0;
  for (int a = 0; a < 4; ++a) for (int b = 0; b < 4; ++b) for (int q2 = 0; q2 < 4; ++q2) s += acc[a][b][q2];
  C[(size_t)blockIdx.x * 256 + threadIdx.x] = s;
}

// correctness check kernel: one 128x128 tile written out, compare direct vs lds on host
template <int NB>
__global__ __launch_bounds__(256) void k_lds_store(const double* A, const double* B, double* C, int K) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int w = threadIdx.x >> 6, wr = w >> 1, wc = w & 1, l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  d4 acc[4][4];
  for (int a = 0; a < 4; ++a) for (int b = 0; b < 4; ++b) acc[a][b] = (d4){0, 0, 0, 0};
  mma_128x128_lds<NB>(acc, A, 128, B, 128, K, lds);
  for (int a = 0; a < 4; ++a) for (int b = 0; b < 4; ++b) for (int q = 0; q < 4; ++q)
    C[(64 * wc + 16 * b + lk + 4 * q) * 128 + 64 * wr + 16 * a + lr] = acc[a][b][q];
}

int main() {
  const int S = 48;
  size_t mat = 2048ull * 2048;
  double* P; hipMalloc(&P, S * mat * 8);
  std::vector<double> h(mat);
  for (size_t i = 0; i < mat; ++i) h[i] = ((i * 2654435761ull) % 1000) / 1000.0 - 0.5;
  for (int s = 0; s < S; ++s) hipMemcpy(P + s * mat, h.data(), mat * 8, hipMemcpyHostToDevice);
  double* C; hipMalloc(&C, 256ull << 20);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  // correctness of the LDS core
  {
    const int K = 256;
    std::vector<double> hA(128 * K), hB(128 * K), hC(128 * 128), ref(128 * 128, 0.0);
    for (int i = 0; i < 128 * K; ++i) { hA[i] = (i % 17) - 8; hB[i] = (i % 13) - 6 + 0.5 * (i % 3); }
    for (int r = 0; r < 128; ++r) for (int c = 0; c < 128; ++c) { double s = 0; for (int k = 0; k < K; ++k) s += hA[k * 128 + r] * hB[k * 128 + c]; ref[c * 128 + r] = s; }
    double *dA, *dB, *dC; hipMalloc(&dA, 128 * K * 8); hipMalloc(&dB, 128 * K * 8); hipMalloc(&dC, 128 * 128 * 8);
    hipMemcpy(dA, hA.data(), 128 * K * 8, hipMemcpyHostToDevice); hipMemcpy(dB, hB.data(), 128 * K * 8, hipMemcpyHostToDevice);
    size_t sh = 3 * 2 * 16 * 128 * 8;
    hipFuncSetAttribute((const void*)k_lds_store<3>, hipFuncAttributeMaxDynamicSharedMemorySize, sh);
    hipLaunchKernelGGL(k_lds_store<3>, dim3(1), dim3(256), sh, 0, dA, dB, dC, K);
    hipMemcpy(hC.data(), dC, 128 * 128 * 8, hipMemcpyDeviceToHost);
    double err = 0; for (int i = 0; i < 128 * 128; ++i) err = fmax(err, fabs(hC[i] - ref[i]));
    printf("lds core correctness: max err %.3e\n", err);
  }
  for (int tri = 0; tri <= 1; ++tri)
  for (int K : {512, 1024}) {
    {
      int nbA = 8, T = nbA * 16;  // 1024x1024 output per slot in 128x64 units
      int grid = S * T;
      hipLaunchKernelGGL(k_dir, dim3(grid), dim3(256), 0, 0, P, C, T, nbA, K, tri);
      hipEventRecord(e0);
      for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k_dir, dim3(grid), dim3(256), 0, 0, P, C, T, nbA, K, tri);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 3;
      double fl = 0; for (int bj = 0; bj < 16; ++bj) fl += 2.0 * 128 * 64 * (tri ? (bj + 1) * 64 : K) * nbA;
      fl *= S;
      printf("tri=%d K=%4d DIRECT 128x64 units grid=%5d: %7.3f ms %6.2f TF\n", tri, K, grid, ms, fl / ms / 1e9);
    }
#define RUNL(NB)                                                                                            \
    {                                                                                                       \
      int nbA = 8, T = nbA * 8; int grid = S * T; size_t sh = NB * 2 * 16 * 128 * 8;                        \
      hipFuncSetAttribute((const void*)k_lds<NB>, hipFuncAttributeMaxDynamicSharedMemorySize, sh);          \
      hipLaunchKernelGGL(k_lds<NB>, dim3(grid), dim3(256), sh, 0, P, C, T, nbA, K, tri);                   \
      hipEventRecord(e0);                                                                                   \
      for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k_lds<NB>, dim3(grid), dim3(256), sh, 0, P, C, T, nbA, K, tri); \
      hipEventRecord(e1); hipEventSynchronize(e1);                                                          \
      float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 3;                                                  \
      double fl = 0; for (int bj = 0; bj < 8; ++bj) fl += 2.0 * 128 * 128 * (tri ? (bj + 1) * 128 : K) * nbA; \
      fl *= S;                                                                                              \
      printf("tri=%d K=%4d LDS-DMA 128x128 NB=%d grid=%5d: %7.3f ms %6.2f TF\n", tri, K, NB, grid, ms, fl / ms / 1e9); \
    }
    RUNL(2)
    RUNL(3)
    RUNL(4)
  }
  printf("err=%s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
