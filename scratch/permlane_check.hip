// v + v(lane ^ 16) and v + v(lane ^ 32) by v_permlane16/32_swap against __shfl_xor, bit for bit
//   hipcc --offload-arch=gfx950 -O3 -o scratch/permlane_check scratch/permlane_check.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
__device__ double sx16(double v) {
  const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return __hiloint2double((int)h[0], (int)l[0]) + __hiloint2double((int)h[1], (int)l[1]);
}
__device__ double sx32(double v) {
  const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return __hiloint2double((int)h[0], (int)l[0]) + __hiloint2double((int)h[1], (int)l[1]);
}
__global__ void k(const double* in, double* out) {
  const int l = threadIdx.x;
  const double v = in[l];
  out[l] = v + __shfl_xor(v, 16);
  out[64 + l] = sx16(v);
  out[128 + l] = v + __shfl_xor(v, 32);
  out[192 + l] = sx32(v);
  double a = v; a += __shfl_xor(a, 16); a += __shfl_xor(a, 32);
  double b = sx32(sx16(v));
  out[256 + l] = a;
  out[320 + l] = b;
}
int main() {
  double h[64], o[384];
  unsigned s = 12345;
  for (int i = 0; i < 64; ++i) { s = s * 1103515245u + 12345u; h[i] = ((s >> 8) / 16777216.0 - 0.5) * (1 << (i % 17)); }
  double *di, *dout;
  (void)hipMalloc(&di, sizeof(h)); (void)hipMalloc(&dout, sizeof(o));
  (void)hipMemcpy(di, h, sizeof(h), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, di, dout);
  (void)hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost);
  int bad16 = 0, bad32 = 0, badc = 0;
  for (int i = 0; i < 64; ++i) {
    bad16 += memcmp(&o[i], &o[64 + i], 8) != 0;
    bad32 += memcmp(&o[128 + i], &o[192 + i], 8) != 0;
    badc += memcmp(&o[256 + i], &o[320 + i], 8) != 0;
  }
  printf("xor16 mismatches %d, xor32 mismatches %d, chained %d, err=%s\n", bad16, bad32, badc, hipGetErrorString(hipGetLastError()));
  return bad16 + bad32 + badc;
}
