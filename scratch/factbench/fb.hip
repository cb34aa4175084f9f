// Microbenchmark of the 16 x 16 diagonal-block factor+inverse on one wave (k_leaf9's diag_w1 step
// loop), cycles per block from s_memtime.  Variants (template V):
//   0: dpp_f64 (two 32-bit DPP moves) + 2 fma, sqrt chain (diag_tile_fast<1>)
//   1: v_fmac_f64_dpp, sqrt chain
//   2: v_fmac_f64_dpp, reciprocal chain (sqrt beside)
//   3: as 2 without the inverse (a only)
//   4: as 2 without updates beyond column j+1 (the bare pivot chain)
// grid: one workgroup per CU of 64 threads (+ optional MFMA-streaming partner wave on the same SIMD)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
typedef double d4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ double readlane_d(double v, int lane) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_readlane((int)b, lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ void sqrt_rsqrt(double p, double& s, double& r) {
  r = __builtin_amdgcn_rsq(p);
  r = r * fma(-0.5 * p * r, r, 1.5);
  r = r * fma(-0.5 * p * r, r, 1.5);
  s = p * r;
  s = fma(0.5 * r, fma(-s, s, p), s);
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
template <int M>
__device__ __forceinline__ void fmac_bcast(double& acc, double src, double f) {
  asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(src), "v"(f), "i"(M));
}
template <int V, int J, int M>
__device__ __forceinline__ void upd(double (&a)[16], double (&y)[16], double au, double aj, double fa, double fy, double yj) {
  if constexpr (M < 16) {
    if constexpr (V == 0) {
      const double b = dpp_f64<0x150 + M>(aj);
      a[M] = fma(-aj, b, a[M]);
      y[M] = fma(-b, yj, y[M]);
    } else if constexpr (V == 4) {
      if (M == J + 1) fmac_bcast<M>(a[M], au, fa);
    } else {
      fmac_bcast<M>(a[M], au, fa);
      if constexpr (V != 3) fmac_bcast<M>(y[M], au, fy);
    }
    upd<V, J, M + 1>(a, y, au, aj, fa, fy, yj);
  }
}
template <int J>
__device__ __forceinline__ double bcast_c(double v) { return __builtin_amdgcn_mov_dpp(v, 0x150 + J, 0xF, 0xF, true); }
// variant 5/6: d = this lane's running diagonal A[i][i] - sum_k u_ik^2 / p_k; pivot J = d of lane J
template <int V, int J>
__device__ __forceinline__ void step5(double (&a)[16], double (&y)[16], double& d, int lr, int& fl) {
  if constexpr (J < 16) {
    const double au = a[J];
    const double p = bcast_c<J>(d);
    const double pk = (p > 0.0) ? p : 1.0;
    fl = (fl < 0 && !(p > 0.0)) ? J : fl;
    const double r0 = __builtin_amdgcn_rcp(pk);
    const double e = fma(-pk, r0, 1.0);
    const double ip = fma(r0, fma(e, e, e), r0);
    d = fma(-au * au, ip, d);  // the next pivots (lane m: column J's contribution to A[m][m])
    const double yu = y[J];
    if constexpr (V == 6) {
      if constexpr (J + 1 < 16) fmac_bcast<J + 1>(a[J + 1], au, -au * ip);
    } else {
      upd<2, J, J + 1>(a, y, au, au, -au * ip, -yu * ip, yu);
    }
    double ljj, rj;
    sqrt_rsqrt(pk, ljj, rj);
    a[J] = (lr > J) ? au * rj : (lr == J ? ljj : 0.0);
    y[J] = yu * rj;
    step5<V, J + 1>(a, y, d, lr, fl);
  }
}
// variant 7: as 5 with the columns kept unscaled (no square root in the step); scaled at the end
template <int J>
__device__ __forceinline__ void step7(double (&a)[16], double (&y)[16], double& d, double& pv, int lr, int& fl) {
  if constexpr (J < 16) {
    const double au = a[J], yu = y[J];
    const double p = bcast_c<J>(d);
    const double pk = (p > 0.0) ? p : 1.0;
    fl = (fl < 0 && !(p > 0.0)) ? J : fl;
    pv = (lr == J) ? pk : pv;
    const double r0 = __builtin_amdgcn_rcp(pk);
    const double e = fma(-pk, r0, 1.0);
    const double ip = fma(r0, fma(e, e, e), r0);
    d = fma(-au * au, ip, d);
    upd<2, J, J + 1>(a, y, au, au, -au * ip, -yu * ip, yu);
    step7<J + 1>(a, y, d, pv, lr, fl);
  }
}
template <int J>
__device__ __forceinline__ void scale7(double (&a)[16], double (&y)[16], double rl, double sl, int lr) {
  if constexpr (J < 16) {
    const double rJ = bcast_c<J>(rl);
    a[J] = (lr > J) ? a[J] * rJ : (lr == J ? sl : 0.0);
    y[J] = y[J] * rJ;
    scale7<J + 1>(a, y, rl, sl, lr);
  }
}
template <int V, int J>
__device__ __forceinline__ void step(double (&a)[16], double (&y)[16], int lr) {
  if constexpr (J < 16) {
    const double au = a[J];
    const double p = readlane_d(au, J);
    const double pk = (p > 0.0) ? p : 1.0;
    if constexpr (V <= 1) {
      double ljj, rj;
      sqrt_rsqrt(pk, ljj, rj);
      const double lij = au * rj;
      a[J] = (lr > J) ? lij : (lr == J ? ljj : 0.0);
      const double xj = y[J] * rj;
      y[J] = xj;
      upd<V, J, J + 1>(a, y, au, a[J], -lij * rj, -xj * rj, xj);
      if constexpr (V == 0)
        for (int m = J; m < 16; ++m) asm volatile("" : "+v"(y[m]));
    } else {
      double ip = __builtin_amdgcn_rcp(pk);
      ip = fma(ip, fma(-pk, ip, 1.0), ip);
      ip = fma(ip, fma(-pk, ip, 1.0), ip);
      const double yu = y[J];
      upd<V, J, J + 1>(a, y, au, au, -au * ip, -yu * ip, yu);
      double ljj, rj;
      sqrt_rsqrt(pk, ljj, rj);
      a[J] = (lr > J) ? au * rj : (lr == J ? ljj : 0.0);
      y[J] = yu * rj;
    }
    step<V, J + 1>(a, y, lr);
  }
}
template <int V>
__global__ __launch_bounds__(128) void kfact(const double* in, double* out, unsigned long long* cyc, int reps, int partner) {
  __shared__ double T[16 * 17];
  const int l = threadIdx.x & 63, lr = l & 15, w = threadIdx.x >> 6;
  if (w == 1) {  // MFMA stream on the same SIMD? (waves 0 and 1 of a workgroup: SIMD placement unknown; see stats)
    if (!partner) return;
    d4 acc = {0, 0, 0, 0};
    double x = in[l];
    for (int i = 0; i < reps * 400; ++i) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, acc, 0, 0, 0);
    if (acc[0] == 12345.0) out[0] = acc[1];
    return;
  }
  for (int e = l; e < 256; e += 64) T[(e >> 4) * 17 + (e & 15)] = in[blockIdx.x * 256 + e] + ((e >> 4) == (e & 15) ? 32.0 : 0.0);
  __builtin_amdgcn_wave_barrier();
  double sum = 0.0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
    double a[16], y[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      a[k] = T[k * 17 + lr];
      y[k] = (k == lr) ? 1.0 : 0.0;
    }
    if constexpr (V == 7) {
      double d = T[lr * 17 + lr], pv = 1.0;
      int fl = -1;
      step7<0>(a, y, d, pv, lr, fl);
      double sl, rl;
      sqrt_rsqrt(pv, sl, rl);
      scale7<0>(a, y, rl, sl, lr);
      sum += fl;
    } else if constexpr (V >= 5) {
      double d = T[lr * 17 + lr];
      int fl = -1;
      step5<V, 0>(a, y, d, lr, fl);
      sum += fl;
    } else {
      step<V, 0>(a, y, lr);
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) sum += a[k] + y[k];
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + l] = sum;
  if (l == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
  const int nb = 256, reps = 200;
  double *in, *out;
  unsigned long long* cyc;
  hipMalloc(&in, nb * 256 * 8);
  hipMalloc(&out, nb * 64 * 8);
  hipMalloc(&cyc, nb * 8);
  std::vector<double> h(nb * 256);
  for (size_t i = 0; i < h.size(); ++i) h[i] = 0.01 * ((i * 2654435761u) % 1000) / 1000.0;
  hipMemcpy(in, h.data(), h.size() * 8, hipMemcpyHostToDevice);
  std::vector<unsigned long long> c(nb);
  auto run = [&](auto kern, const char* name, int partner) {
    hipLaunchKernelGGL(kern, dim3(nb), dim3(partner ? 128 : 64), 0, 0, in, out, cyc, reps, partner);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(kern, dim3(nb), dim3(partner ? 128 : 64), 0, 0, in, out, cyc, reps, partner);
    hipDeviceSynchronize();
    hipMemcpy(c.data(), cyc, nb * 8, hipMemcpyDeviceToHost);
    std::vector<unsigned long long> s(c);
    std::sort(s.begin(), s.end());
    printf("%-40s partner %d  cycles/block median %.0f  min %.0f\n", name, partner, (double)s[nb / 2] / reps, (double)s[0] / reps);
  };
  for (int p = 0; p < 2; ++p) {
    run(kfact<0>, "0 dpp mov32 + fma, sqrt chain", p);
    run(kfact<1>, "1 fmac_dpp, sqrt chain", p);
    run(kfact<2>, "2 fmac_dpp, rcp chain", p);
    run(kfact<3>, "3 fmac_dpp, rcp chain, no inverse", p);
    run(kfact<4>, "4 bare pivot chain (rcp)", p);
    run(kfact<5>, "5 running diagonal, DPP pivot, rcp3", p);
    run(kfact<6>, "6 as 5, bare chain", p);
    run(kfact<7>, "7 unscaled steps, one rsqrt, scale at end", p);
  }
  return 0;
}
