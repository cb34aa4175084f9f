// One copy of L^-1: can a GEMM read one operand "k-packed" (element (row, k) at X[k + row ld], the
// transpose of the library's (row, k) at X[row + k ld]) as fast as the library's register-direct
// 64x64 core reads both operands row-contiguous?  A packed lane loads two consecutive k with one
// 16-B load (k = 8 st + 2 lk + s for sub-step s); the other operand then walks k in the same order.
// C = A B^T over one 1024 x 1024 output panel per slot, 240 slots, ld = 2048, XCD slot mapping as
// the library.  Prints TF/s per variant and K, and the max difference against the regular variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ d4 mfma(double a, double b, d4 c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }

struct Fr {
  double a[2][4], b[2][4];
};
// operand modes: 0 row-contiguous, k = 4s + lk (library); 1 row-contiguous, k = 2 lk + s;
// 2 k-packed (16-B load of k = 2 lk, 2 lk + 1)
struct Op {
  const double* p;
  ptrdiff_t st, sub, blk;
};
template <int M>
__device__ __forceinline__ Op op_ptr(const double* X, ptrdiff_t ld) {
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  if (M == 0) return Op{X + lr + lk * ld, 8 * ld, 4 * ld, 16};
  if (M == 1) return Op{X + lr + 2 * lk * ld, 8 * ld, ld, 16};
  return Op{X + 2 * lk + lr * ld, 8, 1, 16 * ld};
}
template <int M>
__device__ __forceinline__ void op_load(double (&f)[2][4], const Op& o, int st) {
  const double* p = o.p + (ptrdiff_t)st * o.st;
  if constexpr (M == 2) {
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const d2 v = *(const d2*)(p + a * o.blk);
      f[0][a] = v.x;
      f[1][a] = v.y;
    }
  } else {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int a = 0; a < 4; ++a) f[s][a] = p[s * o.sub + a * o.blk];
  }
}
__device__ __forceinline__ void fr_mma(d4 (&acc)[4][4], const Fr& f) {
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = mfma(f.b[s][b], f.a[s][a], acc[a][b]);
}
template <int NL>
__device__ __forceinline__ void groups() {
  constexpr int nm = 32, q = nm / NL, r = nm % NL;
#pragma unroll
  for (int g = 0; g < r; ++g) {
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, q + 1, 0);
  }
#pragma unroll
  for (int g = r; g < NL; ++g) {
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, q, 0);
  }
}
template <int MA, int MB>
__device__ __forceinline__ void core(d4 (&acc)[4][4], const double* A, const double* B, ptrdiff_t ld, int K) {
  const int nst = __builtin_amdgcn_readfirstlane(K / 8);
  const Op pa = op_ptr<MA>(A, ld), pb = op_ptr<MB>(B, ld);
  constexpr int NL = (MA == 2 ? 4 : 8) + (MB == 2 ? 4 : 8);
  Fr f0, f1;
  op_load<MA>(f0.a, pa, 0);
  op_load<MB>(f0.b, pb, 0);
  for (int it = 0; it < nst; it += 2) {
    __builtin_amdgcn_sched_barrier(0);
    op_load<MA>(f1.a, pa, it + 1);
    op_load<MB>(f1.b, pb, it + 1);
    fr_mma(acc, f0);
    groups<NL>();
    __builtin_amdgcn_sched_barrier(0);
    const int n2 = (it + 2 < nst) ? it + 2 : nst - 1;
    op_load<MA>(f0.a, pa, n2);
    op_load<MB>(f0.b, pb, n2);
    fr_mma(acc, f1);
    groups<NL>();
    __builtin_amdgcn_sched_barrier(0);
  }
}
// WG = 4 waves (2 x 2) of 64 x 64 tiles.  Regular A: rows 1024.. of P (col-major); packed A: the
// same elements read from PT = P^T.
template <int MA, int MB>
__device__ __forceinline__ void body(const double* P, const double* PT, double* C, int T, int K, int S) {
  const int x = blockIdx.x & 7, q = blockIdx.x >> 3;
  const int slot = (q / T) * 8 + x, u = q % T;
  if (slot >= S) return;
  const int bi = u % 8, bj = u / 8;
  const size_t mat = 2048ull * 2048;
  const int w = threadIdx.x >> 6, wr = w >> 1, wc = w & 1;
  d4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = (d4){0, 0, 0, 0};
  const int r0 = 1024 + bi * 128 + 64 * wr, c0 = bj * 128 + 64 * wc;
  const double* A = MA == 2 ? PT + slot * mat + (size_t)r0 * 2048 : P + slot * mat + r0;
  const double* B = MB == 2 ? PT + slot * mat + (size_t)c0 * 2048 : P + slot * mat + c0;
  core<MA, MB>(acc, A, B, 2048, K);
  double* Cs = C + (size_t)slot * 1024 * 1024;
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int qq = 0; qq < 4; ++qq)
        Cs[(size_t)(c0 + 16 * b + lk + 4 * qq) * 1024 + (r0 - 1024) + 16 * a + lr] = acc[a][b][qq];
}
#define KERN(NAME, MA, MB)                                                                            \
  __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void NAME(             \
      const double* P, const double* PT, double* C, int T, int K, int S) {                            \
    body<MA, MB>(P, PT, C, T, K, S);                                                                  \
  }
KERN(k_reg, 0, 0)
KERN(k_reg_k2, 1, 1)
KERN(k_pa, 2, 1)
KERN(k_pb, 1, 2)
KERN(k_pab, 2, 2)

int main() {
  const int S = 240;
  const size_t mat = 2048ull * 2048;
  double *P, *PT;
  if (hipMalloc(&P, S * mat * 8) != hipSuccess) return 1;
  if (hipMalloc(&PT, S * mat * 8) != hipSuccess) return 1;
  std::vector<double> h(mat), ht(mat);
  for (size_t i = 0; i < mat; ++i) h[i] = ((i * 2654435761ull) % 1000) / 1000.0 - 0.5;
  for (size_t r = 0; r < 2048; ++r)
    for (size_t c = 0; c < 2048; ++c) ht[c + r * 2048] = h[r + c * 2048];
  for (int s = 0; s < S; ++s) {
    (void)hipMemcpy(P + s * mat, h.data(), mat * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(PT + s * mat, ht.data(), mat * 8, hipMemcpyHostToDevice);
  }
  double* C;
  if (hipMalloc(&C, (size_t)S * 1024 * 1024 * 8) != hipSuccess) return 1;
  std::vector<double> ref((size_t)1024 * 1024), got((size_t)1024 * 1024);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  struct V {
    const char* name;
    const void* f;
  };
  V vs[] = {{"regular (library)", (const void*)k_reg},
            {"regular, k = 2lk+s", (const void*)k_reg_k2},
            {"A packed", (const void*)k_pa},
            {"B packed", (const void*)k_pb},
            {"A and B packed", (const void*)k_pab}};
  for (int K : {1024, 512, 256}) {
    bool first = true;
    for (int rep = 0; rep < 2; ++rep)
      for (auto& v : vs) {
        const int T = 64, grid = 8 * ((S + 7) / 8) * T;
        int Tm = T, Km = K, Sm = S;
        void* a2[] = {&P, &PT, &C, &Tm, &Km, &Sm};
        (void)hipMemset(C, 0, (size_t)S * 1024 * 1024 * 8);
        (void)hipLaunchKernel(v.f, dim3(grid), dim3(256), a2, 0, 0);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(first ? ref.data() : got.data(), C + (size_t)77 * 1024 * 1024, ref.size() * 8,
                        hipMemcpyDeviceToHost);
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
        printf("K=%4d %-22s %8.3f ms %6.2f TF/s  maxdiff %.3g\n", K, v.name, ms, fl / ms / 1e9, md);
        fflush(stdout);
      }
  }
  printf("err=%s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
