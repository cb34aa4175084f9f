// Steady-state fp64 MFMA ceiling of one MI355X (v_mfma_f64_16x16x4_f64, 2048 flops per wave
// instruction): operands in registers, random (or zero) data, >= 2 s of back-to-back warm-up
// launches, then timed launches of >= 50 ms each.  Every wave stamps s_memtime (shader cycles) and
// s_memrealtime (100 MHz) around its loop into a buffer of its own, so the result gives both the
// cycles per MFMA per SIMD and the clock the chip holds under that load (MI355X_MICROARCH.md 'DVFS
// give-back' item 6).  Variants: 1 / 2 waves per SIMD, 4 / 16 independent accumulator chains.
//   hipcc --offload-arch=gfx950 -O3 -o mfma_ceiling mfma_ceiling.hip && ./mfma_ceiling [json]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <random>
#include <vector>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC, int WPS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPS, WPS))) void k_ceiling(const double* src, double* out, unsigned long long* st, int iters) {
  extern __shared__ double lds[];
  const int t = blockIdx.x * 256 + threadIdx.x, l = threadIdx.x & 63;
  double a[4], b[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    a[s] = src[(t * 8 + s) & 4095];
    b[s] = src[(t * 8 + 4 + s) & 4095];
  }
  d4 acc[NACC];
#pragma unroll
  for (int c = 0; c < NACC; ++c) acc[c] = (d4){a[c & 3], b[c & 3], 0, 0};
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_sched_barrier(0);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int c = 0; c < NACC; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[(s + c) & 3], acc[c], 0, 0, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_sched_barrier(0);
  double s = 0;
#pragma unroll
  for (int c = 0; c < NACC; ++c) s += (acc[c][0] + acc[c][1]) + (acc[c][2] + acc[c][3]);
  if (s == 12345.678) lds[l] = s;  // keeps the LDS request (residency) and the chains alive
  out[t] = s;
  if (l == 0) {
    const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    st[4 * w + 0] = t0;
    st[4 * w + 1] = t1;
    st[4 * w + 2] = r0;
    st[4 * w + 3] = r1;
  }
}

template <int NACC, int WPS>
void run1(const double* src, double* out, unsigned long long* dst, int wps, bool zero, const double* zsrc, FILE* js, bool& first) {
  // wps workgroups (4 waves, one per SIMD) per CU: the LDS request keeps a further one off
  const size_t lds = (160 * 1024) / (wps + 1) + 1024;
  (void)hipFuncSetAttribute((const void*)k_ceiling<NACC, WPS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const int blocks = 256 * wps;
  // ~60 ms per launch at ~27 ns per MFMA per SIMD: 2.2 M MFMAs per SIMD
  const int per_iter = 4 * NACC, iters = (int)(2.2e6 / per_iter / wps);
  const double* s = zero ? zsrc : src;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto w0 = std::chrono::steady_clock::now();
  int nwarm = 0;
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - w0).count() < 2.5) {
    for (int k = 0; k < 8; ++k) hipLaunchKernelGGL((k_ceiling<NACC, WPS>), dim3(blocks), dim3(256), lds, 0, s, out, dst, iters);
    hipDeviceSynchronize();
    nwarm += 8;
  }
  const int reps = 5;
  hipEventRecord(e0);
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_ceiling<NACC, WPS>), dim3(blocks), dim3(256), lds, 0, s, out, dst, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const int nw = blocks * 4;
  std::vector<unsigned long long> h(4 * (size_t)nw);
  hipMemcpy(h.data(), dst, h.size() * 8, hipMemcpyDeviceToHost);
  std::vector<double> clk;
  unsigned long long r_lo = ~0ull, r_hi = 0;
  for (int w = 0; w < nw; ++w) {
    const double dt = (double)(h[4 * w + 1] - h[4 * w]), dr = (double)(h[4 * w + 3] - h[4 * w + 2]);
    clk.push_back(dt / dr * 0.1);  // GHz
    r_lo = std::min(r_lo, h[4 * w + 2]);
    r_hi = std::max(r_hi, h[4 * w + 3]);
  }
  std::sort(clk.begin(), clk.end());
  const double med_clk = clk[nw / 2];
  const double flops = 2048.0 * per_iter * (double)iters * nw * reps;
  const double tf = flops / (ms * 1e-3) / 1e12;
  // cycles per MFMA per SIMD over the last launch's envelope (first wave start to last wave end on
  // the 100 MHz realtime counter, at the median clock): the wps waves of a SIMD need not all be
  // resident at once, so one wave's own interval divided by wps (round 4's conversion) overstated
  // the rate above the spec peak at 3, 4 and 8 waves per SIMD
  const double span_cyc = (double)(r_hi - r_lo) / 0.1 * med_clk;  // ns -> cycles
  const double mfma_per_simd = (double)per_iter * iters * nw / 1024.0;
  const double med_cyc = span_cyc / mfma_per_simd;
  const double tf_clk = 2048.0 * 1024 * med_clk * 1e9 / med_cyc / 1e12;  // from the stamps
  printf("[build wpe %d] waves/SIMD=%d chains=%2d %s  %.1f ms/launch  %.2f TF/s (events)  clock %.3f GHz (p10 %.3f p90 %.3f)  "
         "%.2f cycles/MFMA/SIMD  %.2f TF/s (stamps)  warm-up %d launches  %s\n",
         WPS, wps, NACC, zero ? "zeros " : "random", ms / reps, tf, med_clk, clk[nw / 10], clk[nw * 9 / 10], med_cyc, tf_clk,
         nwarm, hipGetErrorString(hipGetLastError()));
  if (js) {
    fprintf(js,
            "%s  {\"build_waves_per_eu\": %d, \"accumulators\": \"%s\", \"waves_per_simd\": %d, \"chains\": %d, \"operands\": \"%s\", \"ms_per_launch\": %.3f, \"tflops_events\": %.3f, "
            "\"clock_ghz_median\": %.4f, \"clock_ghz_p10\": %.4f, \"clock_ghz_p90\": %.4f, \"cycles_per_mfma_per_simd\": %.3f, "
            "\"tflops_stamps\": %.3f, \"warmup_launches\": %d}",
            first ? "" : ",\n", WPS, WPS == 1 ? "agpr" : "vgpr", wps, NACC, zero ? "zeros" : "random", ms / reps, tf, med_clk, clk[nw / 10], clk[nw * 9 / 10],
            med_cyc, tf_clk, nwarm);
    first = false;
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main(int argc, char** argv) {
  std::vector<double> h(4096);
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> U(-1, 1);
  for (auto& x : h) x = U(g) * 1e-3;  // small: the chains stay finite over millions of steps
  double *src, *zsrc, *out;
  unsigned long long* st;
  hipMalloc(&src, 4096 * 8);
  hipMalloc(&zsrc, 4096 * 8);
  hipMalloc(&out, 8 * 256 * 256 * 8);
  hipMalloc(&st, 8 * 256 * 4 * 4 * 8);
  hipMemcpy(src, h.data(), 4096 * 8, hipMemcpyHostToDevice);
  hipMemset(zsrc, 0, 4096 * 8);
  FILE* js = argc > 1 ? fopen(argv[1], "w") : nullptr;
  if (js) fprintf(js, "{\"kernel\": \"v_mfma_f64_16x16x4_f64, operands in registers\", \"runs\": [\n");
  bool first = true;
  run1<4, 1>(src, out, st, 1, false, zsrc, js, first);
  run1<16, 1>(src, out, st, 1, false, zsrc, js, first);
  run1<16, 1>(src, out, st, 1, true, zsrc, js, first);
  run1<1, 1>(src, out, st, 1, false, zsrc, js, first);
  // compiled for 2 waves per SIMD (accumulators in VGPRs, no AGPRs), launched at one
  run1<4, 2>(src, out, st, 1, false, zsrc, js, first);
  run1<16, 2>(src, out, st, 1, false, zsrc, js, first);
  run1<4, 2>(src, out, st, 2, false, zsrc, js, first);
  run1<8, 2>(src, out, st, 2, false, zsrc, js, first);
  run1<16, 2>(src, out, st, 2, false, zsrc, js, first);
  run1<4, 3>(src, out, st, 3, false, zsrc, js, first);
  run1<4, 4>(src, out, st, 4, false, zsrc, js, first);
  run1<8, 4>(src, out, st, 4, false, zsrc, js, first);
  run1<2, 8>(src, out, st, 8, false, zsrc, js, first);
  if (js) {
    fprintf(js, "\n]}\n");
    fclose(js);
  }
  return 0;
}
