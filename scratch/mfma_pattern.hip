// Where does the 64x64 wave core lose ~6% of the fp64 MFMA rate when no loads are in its loop
// (profiles/r04_core_latency.txt: 72.2 TF/s vs the 77.4 ceiling)?  Operands in registers,
// 2 waves per SIMD, 16 accumulators (4 x 4 blocks of 16 x 16), variants of the operand pattern.
//   hipcc --offload-arch=gfx950 -O3 -o scratch/mfma_pattern scratch/mfma_pattern.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ d4 mfma(double a, double b, d4 c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }

// V: 0 one A / one B register for every MFMA; 1 four A x four B (the core's blocks, one k-step per
// iteration); 2 as 1 with every operand rewritten by a VALU op each iteration (stands in for the
// loads landing); 3 as 1 with two operand sets alternating (the core's f0 / f1 ping-pong, 2 k-steps
// per iteration); 4 as 3 with the library's sched_group_barrier interleave of 5 MFMA / 4 VALU
template <int V>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_pat(const double* src, double* out, int iters) {
  const int l = threadIdx.x & 63;
  d4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = (d4){0, 0, 0, 0};
  double A[2][4], B[2][4];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      A[s][a] = src[(s * 8 + a) * 64 + l];
      B[s][a] = src[(s * 8 + 4 + a) * 64 + l];
    }
  int ip[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) ip[q] = q + l;
  for (int i = 0; i < iters; ++i) {
    if constexpr (V == 0) {
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) acc[a][b] = mfma(B[0][0], A[0][0], acc[a][b]);
    } else if constexpr (V == 1) {
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) acc[a][b] = mfma(B[0][b], A[0][a], acc[a][b]);
    } else if constexpr (V == 2) {
#pragma unroll
      for (int r = 0; r < 2; ++r) {
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) acc[a][b] = mfma(B[0][b], A[0][a], acc[a][b]);
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          A[0][a] = A[0][a] * 0.999;
          B[0][a] = B[0][a] * 0.999;
        }
      }
    } else if constexpr (V == 5 || V == 6) {  // V1 + 8 (V5) / 16 (V6) integer VALU ops per 16 MFMAs
#pragma unroll
      for (int r = 0; r < 2; ++r) {
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) acc[a][b] = mfma(B[0][b], A[0][a], acc[a][b]);
#pragma unroll
        for (int q = 0; q < (V == 5 ? 8 : 16); ++q) asm volatile("v_add_u32 %0, %0, %1" : "+v"(ip[q & 7]) : "v"(l));
      }
    } else {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) acc[a][b] = mfma(B[s][b], A[s][a], acc[a][b]);
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          A[s][a] = A[s][a] * 0.999;
          B[s][a] = B[s][a] * 0.999;
        }
        if constexpr (V == 4) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
  }
  double t = 0.0;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) t += acc[a][b][0] + acc[a][b][3];
#pragma unroll
  for (int q = 0; q < 8; ++q) t += ip[q];
  out[blockIdx.x * 256 + threadIdx.x] = t;
}

// V7: the library core's pattern: 2 stages of 8 A + 8 B fragment loads (global, 64-bit VGPR
// addresses advanced per stage) in ping-pong with 32 MFMAs each, over an L2-resident panel;
// V8: the same with buffer loads (32-bit lane offset in a VGPR, stage offset in an SGPR)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
}
template <int V>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_core(const double* P, double* out, int iters) {
  constexpr int LD = 256;  // panel: 256 x 64 doubles (128 KB), column-major, L2-resident
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  d4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = (d4){0, 0, 0, 0};
  double fa[2][2][4], fb[2][2][4];  // [buffer][substep][block]
  const __amdgpu_buffer_rsrc_t r = rsrc(P, LD * 64 * 8);
  const int vo = (lr + lk * LD) * 8;
  auto load = [&](int buf, int st) {
    const int stage = st & 3;  // wrap over the panel's 64 columns (8 per stage)
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        if constexpr (V == 7) {
          const double* p = P + lr + lk * LD + (stage * 8 + 4 * s) * LD;
          fa[buf][s][a] = p[16 * a];
          fb[buf][s][a] = p[64 + 16 * a];
        } else {
          const int so = (stage * 8 + 4 * s) * LD * 8;
          fa[buf][s][a] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, vo + 128 * a, so, 0));
          fb[buf][s][a] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, vo + 512 + 128 * a, so, 0));
        }
      }
  };
  auto mm = [&](int buf) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = mfma(fb[buf][s][b], fa[buf][s][a], acc[a][b]);
  };
  load(0, 0);
  for (int it = 0; it < iters; it += 2) {
    __builtin_amdgcn_sched_barrier(0);
    load(1, it + 1);
    mm(0);
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    load(0, it + 2);
    mm(1);
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  double t = 0.0;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) t += acc[a][b][0] + acc[a][b][3];
  out[blockIdx.x * 256 + threadIdx.x] = t;
}
template <int V>
void run_core(const double* src, double* out, int iters, const char* name) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k_core<V>, dim3(512), dim3(256), 0, 0, src, out, iters);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_core<V>, dim3(512), dim3(256), 0, 0, src, out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= 5;
  const double fl = 512.0 * 4 * 32 * 2048.0 * iters;  // 32 MFMAs per stage, one stage per iteration
  printf("%-48s %8.3f ms  %6.2f TF/s\n", name, ms, fl / (ms * 1e-3) / 1e12);
}

template <int V>
void run(const double* src, double* out, int iters, const char* name) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k_pat<V>, dim3(512), dim3(256), 0, 0, src, out, iters);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_pat<V>, dim3(512), dim3(256), 0, 0, src, out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= 5;
  const double fl = 512.0 * 4 * 32 * 2048.0 * iters;  // 32 MFMAs per iteration per wave
  printf("%-48s %8.3f ms  %6.2f TF/s\n", name, ms, fl / (ms * 1e-3) / 1e12);
}

int main() {
  double *src, *out;
  (void)hipMalloc(&src, 16 * 64 * 8);
  (void)hipMalloc(&out, 512 * 256 * 8);
  double h[16 * 64];
  for (int i = 0; i < 16 * 64; ++i) h[i] = 1e-3 * ((i * 37) % 101) / 101.0;
  (void)hipMemcpy(src, h, sizeof(h), hipMemcpyHostToDevice);
  const int it = 20000;
  run<0>(src, out, it, "V0 one A, one B register");
  run<1>(src, out, it, "V1 4 A x 4 B registers");
  run<2>(src, out, it, "V2 V1 + operands rewritten by VALU");
  run<3>(src, out, it, "V3 two operand sets alternating + VALU");
  run<4>(src, out, it, "V4 V3 + sched_group_barrier interleave");
  run<5>(src, out, it, "V5 V1 + 8 int VALU per 16 MFMAs");
  run<6>(src, out, it, "V6 V1 + 16 int VALU per 16 MFMAs");
  double* panel;
  (void)hipMalloc(&panel, 256 * 64 * 8);
  (void)hipMemset(panel, 0, 256 * 64 * 8);
  run_core<7>(panel, out, it, "V7 core: global loads, 64-bit VGPR addresses");
  run_core<8>(panel, out, it, "V8 core: buffer loads, SGPR stage offsets");
  printf("err=%s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
