// Does per-lane scratch (private segment) memory keep its contents while another process uses
// the same GPU?  Each lane fills a dynamically indexed private array (forced to scratch), waits,
// reads it back and counts mismatches.  Run it alone and beside a second GPU process.
//   hipcc --offload-arch=gfx950 -O2 -o scratch/scratch_probe scratch/scratch_probe.hip
//   scratch/scratch_probe SECONDS
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(256) void k_scratch(unsigned long long* bad, int salt, int spin) {
  volatile double buf[96];  // volatile + runtime indices: lives in scratch
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  for (int i = 0; i < 96; ++i) buf[(i * 37 + salt) % 96] = (double)(t * 131u + (unsigned)i * 7u + (unsigned)salt);
  for (int s = 0; s < spin; ++s) __builtin_amdgcn_s_sleep(8);
  unsigned long long n = 0;
  for (int i = 0; i < 96; ++i)
    if (buf[(i * 37 + salt) % 96] != (double)(t * 131u + (unsigned)i * 7u + (unsigned)salt)) ++n;
  if (n) atomicAdd(bad, n);
}

int main(int argc, char** argv) {
  const double secs = argc > 1 ? atof(argv[1]) : 10.0;
  unsigned long long* d = nullptr;
  if (hipMalloc(&d, sizeof(*d)) != hipSuccess) return 1;
  (void)hipMemset(d, 0, sizeof(*d));
  const auto t0 = std::chrono::steady_clock::now();
  long launches = 0;
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < secs) {
    for (int k = 0; k < 16; ++k, ++launches) hipLaunchKernelGGL(k_scratch, dim3(4096), dim3(256), 0, 0, d, (int)(launches % 96), 64);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
  }
  unsigned long long h = 0;
  (void)hipMemcpy(&h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("{\"launches\": %ld, \"lanes_per_launch\": %d, \"mismatched_words\": %llu}\n", launches, 4096 * 256, h);
  return h ? 3 : 0;
}
