// Phase timing of the 64x64 diagonal tile factor (diag_tile<NW>) at B=192 (one workgroup per slot):
// the 4-wave kernel, the 1-wave variant in a 64-thread workgroup, and an instrumented 1-wave copy
// (scratch/diag_probe_body.inc, generated from the production body) with s_memrealtime probes.
#include "../gpr.jl_amd/csrc/gprx_kernels.hip"
#include <cstdio>
namespace gprx {
__global__ void k_nothing(int* p) { if (p && threadIdx.x == 1000) p[0] = 1; }
__global__ __launch_bounds__(256) void k_diag_twice(DevBatch db, int jt) { diag_tile_fast(db, blockIdx.x, jt); __syncthreads(); diag_tile_fast(db, blockIdx.x, jt + 1); }
}
using namespace gprx;
int main() {
  const int B = 192, N = 256;
  DevBatch db{};
  db.B = B; db.N = N; db.Npad = N; db.nt = N / 64; db.ld = N; db.mat = (size_t)N * N; db.d = 1;
  std::vector<double> h((size_t)B * N * N);
  for (int s = 0; s < B; ++s)
    for (int c = 0; c < N; ++c)
      for (int r = 0; r < N; ++r) h[(size_t)s * N * N + (size_t)c * N + r] = (r == c ? N + 1.0 : 0.5 / (1.0 + abs(r - c)));
  hipMalloc(&db.K, h.size() * 8); hipMalloc(&db.Linv, h.size() * 8); hipMalloc(&db.Mt, h.size() * 8);
  hipMalloc(&db.Y, (size_t)B * N * 8); hipMalloc(&db.zp, (size_t)B * 2 * db.nt * N * 8);
  hipMalloc(&db.logdet_part, (size_t)B * db.nt * 8); hipMalloc(&db.status, B * 4); hipMalloc(&db.info, B * 4);
  hipMemset(db.Y, 0, (size_t)B * N * 8); hipMemset(db.status, 0, B * 4);
  unsigned long long* tp;
  hipMalloc(&tp, 64 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  auto run = [&](const char* name, auto launch) {
    hipMemcpy(db.K, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    launch();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 20; ++r) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-28s %8.2f us per launch\n", name, ms * 1000 / 20);
  };
  run("diag (k_diag_f)", [&] { hipLaunchKernelGGL(k_diag_f, dim3(B), dim3(256), 0, 0, db, 1); });
  run("diag x2 in one kernel", [&] { hipLaunchKernelGGL(k_diag_twice, dim3(B), dim3(256), 0, 0, db, 1); });
  run("empty kernel", [&] { hipLaunchKernelGGL(k_nothing, dim3(1), dim3(64), 0, 0, (int*)nullptr); });
  int st[B];
  hipMemcpy(st, db.status, B * 4, hipMemcpyDeviceToHost);
  printf("status0=%d err=%s\n", st[0], hipGetErrorString(hipGetLastError()));
  return 0;
}
