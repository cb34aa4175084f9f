// Which SIMD does wave w of a workgroup land on, and which workgroups share a CU?  B blocks of 256
// threads with 68 KB of dynamic LDS (k_node8h's shape); every wave records its hardware ids and
// realtime stamps around a ~40 us busy loop.  hipcc --offload-arch=gfx950 -O3 hwid_probe.hip -o hwid_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ __launch_bounds__(512) void probe(unsigned* out, int spin) {
  extern __shared__ double lds[];
  const int w = threadIdx.x >> 6; const int NW = blockDim.x >> 6;
  unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));       // HW_REG_HW_ID, 32 bits
  unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11));     // HW_REG_XCC_ID
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  double x = threadIdx.x;
  for (int i = 0; i < spin; ++i) x = __builtin_fma(x, 1.0000001, 1e-9);
  lds[threadIdx.x] = x;
  __syncthreads();
  unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0) {
    unsigned* o = out + ((size_t)blockIdx.x * NW + w) * 8;
    o[0] = blockIdx.x; o[1] = w; o[2] = hw; o[3] = xcc;
    o[4] = (unsigned)t0; o[5] = (unsigned)(t0 >> 32); o[6] = (unsigned)t1; o[7] = (unsigned)(t1 >> 32) + (lds[threadIdx.x + 1] > 1e300);
  }
}
int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 1024, spin = argc > 2 ? atoi(argv[2]) : 20000;
  const int NT = argc > 3 ? atoi(argv[3]) : 256, NWV = NT / 64;
  unsigned* d;
  hipMalloc(&d, (size_t)B * NWV * 8 * 4);
  hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(probe, dim3(B), dim3(NT), NT == 512 ? 150000 : 67608, 0, d, spin);
  hipDeviceSynchronize();
  std::vector<unsigned> h((size_t)B * NWV * 8);
  hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
  for (int i = 0; i < B * NWV; ++i) {
    const unsigned* o = &h[(size_t)i * 8];
    const unsigned hw = o[2];
    printf("%u %u simd %u wave %u cu %u sh %u se %u xcc %u t0 %llu t1 %llu\n", o[0], o[1], (hw >> 4) & 3, hw & 15, (hw >> 8) & 15,
           (hw >> 12) & 1, (hw >> 13) & 7, o[3] & 15, (unsigned long long)o[4] | ((unsigned long long)o[5] << 32),
           (unsigned long long)o[6] | ((unsigned long long)o[7] << 32));
  }
  return 0;
}
