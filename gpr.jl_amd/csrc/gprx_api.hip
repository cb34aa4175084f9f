// gprx_api.hip -- C ABI (include/gprx.h) over the gfx950 kernels: context/stream ownership,
// batch workspaces in HBM, the per-evaluation launch sequence, status mapping, profiling.
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "../../include/gprx.h"
#include "gprx_internal.h"

using gprx::DevBatch;
using gprx::TS;

namespace {

struct KStat {
  double ms = 0.0, flops = 0.0, bytes = 0.0;
  int64_t n = 0;
};
struct PendingEv {
  std::string name;
  std::string level;  // optional second key, e.g. "potrf_syrk/n32" (per recursion level)
  hipEvent_t a, b;
  double flops, bytes;
};

}  // namespace

struct gprx_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;
  std::string err;
  int dist_mode = GPRX_DIST_DIRECT;  // the Gram of GaussianProcesses cov_ij (distij) [ext]
  bool prof = false;
  std::map<std::string, KStat> stats;
  std::vector<hipEvent_t> evpool;
  std::vector<PendingEv> pending;
  // recursion nodes of <= this many tiles run fused in k_leaf; 0 = auto: 4 for batches of >= 32
  // slots (fewer launches), 1 below that (GPRX_OPT_LEAF_TILES)
  int leaf_tiles = 0;
  // recursion nodes of <= this many tiles use the 64 x 32 pair-unit GEMM; 0 = auto (set_geometry:
  // 4 for batches of >= 32 slots, every node below that) (GPRX_OPT_SMALL_N)
  int small_n = 0;
  int node_waves = 0;  // GPRX_OPT_NODE_WAVES: 0 auto, 8 (k_node8), 4 (k_node8h)
  // replay each batch's launch sequence as a hipGraph (GPRX_OPT_GRAPHS).  Off by default: measured
  // equal to direct launches at B=1..192 (the launches are queued far ahead of the GPU).
  bool use_graphs = false;
  std::set<gprx_batch*> batches;      // live batches (destroyed with the context)
  void* rbuf = nullptr;               // rollout argument buffer (device), grown on demand
  size_t rcap = 0;
};

struct gprx_batch {
  gprx_ctx* ctx = nullptr;
  DevBatch db{};
  std::vector<void*> allocs;
  double* h_params = nullptr;  // pinned
  double* h_out = nullptr;     // pinned, B*(d+3)
  double* h_mu = nullptr;      // pinned, B*Mpad
  double* h_var = nullptr;
  int* h_status = nullptr;  // pinned, 2B (status, info)
  int* opt_active = nullptr;  // device, B: the optimiser's per-round evaluation mask (DevBatch::active)
  double* opt_trace = nullptr;  // caller's host buffer for gprx_batch_set_opt_trace (diagnostics)
  int opt_trace_rounds = 0;
  bool factored = false;
  bool have_train = false;
  bool have_test = false;
  // captured evaluation graphs, one per (want_grad, want_pred); valid while the key matches
  hipGraphExec_t gexec[4] = {};
  DevBatch gkey[4];
  int gkey_ctx[4][3] = {};
  bool gvalid[4] = {};
};

struct gprx_gp {
  gprx_batch* batch = nullptr;
  int M_cap = 0;
};

namespace {

int set_err(gprx_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

#define HIPCHK(ctx, expr)                                                                          \
  do {                                                                                             \
    hipError_t e_ = (expr);                                                                        \
    if (e_ != hipSuccess) {                                                                        \
      (void)hipGetLastError(); /* not sticky for the context's next call */                        \
      return set_err((ctx), e_ == hipErrorOutOfMemory ? GPRX_OUT_OF_MEMORY : GPRX_DEVICE_ERROR,     \
                     std::string(#expr) + ": " + hipGetErrorString(e_));                           \
    }                                                                                              \
  } while (0)

hipEvent_t ev_get(gprx_ctx* c) {
  if (!c->evpool.empty()) {
    hipEvent_t e = c->evpool.back();
    c->evpool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

// Launch helper: optional HIP-event bracket per launch, on the context stream.
template <class F>
void timed(gprx_ctx* c, hipStream_t st, const char* name, double flops, double bytes, F&& f, int level = 0) {
  if (!c->prof) {
    f();
    return;
  }
  hipEvent_t a = ev_get(c), b = ev_get(c);
  (void)hipEventRecord(a, st);
  f();
  (void)hipEventRecord(b, st);
  c->pending.push_back({name, level ? std::string(name) + "/n" + std::to_string(level) : std::string(), a, b, flops, bytes});
}

void collect(gprx_ctx* c) {
  for (auto& p : c->pending) {
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, p.a, p.b);
    for (int k = 0; k < 2; ++k) {
      if (k == 1 && p.level.empty()) break;
      KStat& s = c->stats[k ? p.level : p.name];
      s.ms += ms;
      s.n += 1;
      s.flops += p.flops;
      s.bytes += p.bytes;
    }
    c->evpool.push_back(p.a);
    c->evpool.push_back(p.b);
  }
  c->pending.clear();
}

template <class T>
int dalloc(gprx_batch* b, T** p, size_t count) {
  void* q = nullptr;
  if (count == 0) count = 1;
  hipError_t e = hipMalloc(&q, count * sizeof(T));
  if (e != hipSuccess) {
    (void)hipGetLastError();  // clear the runtime's sticky error: later calls check hipGetLastError
    *p = nullptr;
    return set_err(b->ctx, e == hipErrorOutOfMemory ? GPRX_OUT_OF_MEMORY : GPRX_DEVICE_ERROR,
                   std::string("hipMalloc: ") + hipGetErrorString(e));
  }
  b->allocs.push_back(q);
  *p = (T*)q;
  return GPRX_OK;
}

void free_test(gprx_batch* b);

// The GEMM cores, the Gram and the LINV21 store address their operands through buffer resources of
// 0x7ffffff0 bytes from a tile origin, with 32-bit byte offsets (gprx_kernels.hip buffer_rsrc,
// core_ptr): a K walk spans up to Npad columns of ld = Npad (the factorisation) or Npad rows of
// ld = Mpad (the prediction variance's K*^T).  Beyond that range a load would silently read 0, so
// such sizes are refused (N <= 16320 at M <= Npad).
constexpr size_t BUF_LIMIT = 0x7ffffff0;
bool sizes_addressable(size_t Npad, size_t Mpad) { return Npad * std::max(Npad, Mpad) * sizeof(double) < BUF_LIMIT; }
size_t pad64(size_t n) { return (n + TS - 1) / TS * TS; }

// Device bytes of a batch's test-point buffers (alloc_test) and of the whole batch
// (gprx_batch_create); the same expressions as the allocations
size_t test_bytes(size_t B, size_t d, size_t Npad, size_t Mpad) {
  const size_t nt = Npad / TS;
  return sizeof(double) * (B * Mpad * d + B * Npad * Mpad + 2 * B * nt * Mpad + 2 * B * Mpad);
}
size_t batch_bytes(size_t B, int d, size_t Npad, size_t Mpad) {
  const size_t nt = Npad / TS, mat = Npad * Npad, xs = (size_t)(d | 1);
  int ngu = 0, nimg = 0;
  const size_t nlj = (size_t)std::max(gprx::lauum_plan((int)nt, d, &ngu, &nimg, nullptr), 0);
  const size_t dbl = B * Npad * d + B * Npad * xs + B * Npad + 5 * B * mat + B * Npad + B * 2 * nt * Npad + B * Npad +
                     B * (d + 4) + B * (d + 2) + B * nt + B * (size_t)ngu * (d + 2) + B * (d + 3);
  const size_t ints = 2 * B + 2 * gprx::LU * nlj + B;
  return dbl * sizeof(double) + ints * sizeof(int) + test_bytes(B, d, Npad, Mpad);
}

int alloc_test(gprx_batch* b, int M_max) {
  DevBatch& db = b->db;
  db.M = 0;
  db.Mpad = ((M_max + TS - 1) / TS) * TS;
  if (db.Mpad == 0) db.Mpad = TS;
  if (!sizes_addressable(db.Npad, db.Mpad))
    return set_err(b->ctx, GPRX_INVALID_ARGUMENT, "test points: Npad * max(Npad, Mpad) * 8 exceeds the 2 GiB buffer range");
  db.mt = db.Mpad / TS;
  const size_t B = db.B;
  int rc;
  if ((rc = dalloc(b, &db.Xs, B * db.Mpad * db.d))) return rc;
  if ((rc = dalloc(b, &db.KsT, B * (size_t)db.Npad * db.Mpad))) return rc;
  if ((rc = dalloc(b, &db.mu_part, B * db.nt * (size_t)db.Mpad))) return rc;
  if ((rc = dalloc(b, &db.var_part, B * db.nt * (size_t)db.Mpad))) return rc;
  if ((rc = dalloc(b, &db.out_mu, B * db.Mpad))) return rc;
  if ((rc = dalloc(b, &db.out_var, B * db.Mpad))) return rc;
  if (hipHostMalloc((void**)&b->h_mu, B * db.Mpad * sizeof(double)) != hipSuccess ||
      hipHostMalloc((void**)&b->h_var, B * db.Mpad * sizeof(double)) != hipSuccess) {
    (void)hipGetLastError();
    return GPRX_OUT_OF_MEMORY;
  }
  (void)hipMemset(db.Xs, 0, B * db.Mpad * db.d * sizeof(double));
  return GPRX_OK;
}

void release_ptr(gprx_batch* b, void* p) {
  for (auto it = b->allocs.begin(); it != b->allocs.end(); ++it)
    if (*it == p) {
      (void)hipFree(p);
      b->allocs.erase(it);
      return;
    }
}

void free_test(gprx_batch* b) {
  DevBatch& db = b->db;
  void* ps[] = {db.Xs, db.KsT, db.mu_part, db.var_part, db.out_mu, db.out_var};
  for (void* p : ps)
    if (p) release_ptr(b, p);
  db.Xs = db.KsT = db.mu_part = db.var_part = db.out_mu = db.out_var = nullptr;
  if (b->h_mu) (void)hipHostFree(b->h_mu);
  if (b->h_var) (void)hipHostFree(b->h_var);
  b->h_mu = b->h_var = nullptr;
}

int copy_in(gprx_ctx* c, void* dst, const void* src, size_t bytes, int mem) {
  HIPCHK(c, hipMemcpyAsync(dst, src, bytes, mem == GPRX_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                           c->stream));
  return GPRX_OK;
}

// Recursive Cholesky + inverse over tile range [o, o+n) (tile units), all slots in lock step.
// upd: the node lies in the trailing block of an ancestor (its tiles were updated into S); the top
// child inherits the parent's flag, the bottom child follows the parent's SYRK
void factor_rec(gprx_ctx* c, hipStream_t st, const DevBatch& db, int o, int n, int upd) {
  const double T = TS, Bd = db.B;
  const int leaf = c->leaf_tiles > 0 ? c->leaf_tiles : (db.B >= 32 ? 4 : 1);
  if (n > 1 && n <= leaf) {
    const double m = n * T;
    timed(c, st, "leaf", Bd * (m * m * m / 3.0 + m * m * m / 3.0), Bd * 8.0 * 3.0 * m * m,
          [&] { gprx::launch_leaf(db, o, n, upd, st); }, n);
    return;
  }
#ifndef GPRX_NODE8
#define GPRX_NODE8 1
#endif
  if (GPRX_NODE8 && n == 8 && leaf == 4 && db.B >= 32) {  // the whole node in one launch (k_node8)
    const double m = 4 * T;
    // the 4-wave form (two slots per CU, bit-identical) on request only: measured slower at every
    // batch size ("Two slots per CU"): a paired slot's fp64 VALU chain and MFMAs share
    // the SIMD's one fp64 pipe with the other slot's, so the pair runs at half speed
    const bool four = c->node_waves == 4;
    timed(c, st, four ? "node8h" : "node8", Bd * (4.0 * m * m * m / 3.0 + 4.0 * m * m * m),
          Bd * 8.0 * (16.0 * m * m + 6.5 * m * m), [&] { gprx::launch_node8(db, o, upd, st, four); }, n);
    return;
  }
  if (n == 1) {
    timed(c, st, "diag", Bd * (T * T * T / 3.0 + T * T * T / 3.0), Bd * 8.0 * 3.0 * T * T,
          [&] { gprx::launch_diag(db, o, upd, st); });
    return;
  }
  const int h = n / 2;
  const double m1 = h * T, m2 = (n - h) * T;
  factor_rec(c, st, db, o, h, upd);
  gprx::GemmGeom g{gprx::OP_TRSM, o, h, n, upd};
  const double f_trsm = Bd * m2 * m1 * m1, f_syrk = Bd * m2 * m2 * m1, f_tt = Bd * m2 * m1 * m1,
               f_linv = Bd * m1 * m2 * m2;
  const double b_trsm = Bd * 8.0 * (2.0 * m2 * m1 + m1 * m1 / 2.0), b_syrk = Bd * 8.0 * (m2 * m1 + m2 * m2),
               b_tt = Bd * 8.0 * (2.0 * m2 * m1 + m1 * m1 / 2.0), b_linv = Bd * 8.0 * (3.0 * m2 * m1 + m2 * m2 / 2.0);
  timed(c, st, "potrf_trsm", f_trsm, b_trsm, [&] { gprx::launch_gemm(db, g, st); }, n);
  gprx::GemmGeom gs{gprx::OP_SYRK, o, h, n, upd}, gt{gprx::OP_TT, o, h, n, upd};
  // T^T = L11^-T L21^T needs only rec(A11) and the TRSM: it runs in the SYRK's launch
  timed(c, st, "syrk_tt", f_syrk + f_tt, b_syrk + b_tt, [&] { gprx::launch_gemm(db, gs, st, gt); }, n);
  factor_rec(c, st, db, o + h, n - h, 1);
  g.op = gprx::OP_LINV21;
  timed(c, st, "trtri_linv21", f_linv, b_linv, [&] { gprx::launch_gemm(db, g, st); }, n);
}

void predict_cross(gprx_ctx* c, hipStream_t st, const DevBatch& db) {
  const double N = db.N, M = db.M, d = db.d, B = db.B;
  timed(c, st, "pred_cross", B * 3.0 * N * M * d, B * 8.0 * (N * db.Mpad + (N + M) * d),
        [&] { gprx::launch_pred_cross(db, st); });
}
void predict_var(gprx_ctx* c, hipStream_t st, const DevBatch& db) {
  if (!db.want_var) return;
  const double N = db.N, M = db.M, B = db.B;
  gprx::GemmGeom g{gprx::OP_PREDVAR, 0, 0, 0};
  timed(c, st, "pred_var", B * N * N * M, B * 8.0 * (N * N / 2 + N * db.Mpad), [&] { gprx::launch_gemm(db, g, st); });
}
void predict_mean_final(gprx_ctx* c, hipStream_t st, const DevBatch& db) {
  const double B = db.B;
  timed(c, st, "pred_final", B * 2.0 * db.nt * db.Mpad, B * 16.0 * db.nt * db.Mpad,
        [&] { gprx::launch_pred_final(db, st); });
}
void predict_group(gprx_ctx* c, hipStream_t st, const DevBatch& db) {
  predict_cross(c, st, db);
  predict_var(c, st, db);
  predict_mean_final(c, st, db);
}

// Whole evaluation of a batch (or a slot range of it) on stream `st`.
void eval_group(gprx_ctx* c, hipStream_t st, const DevBatch& db, bool want_grad, bool want_pred) {
  const double Bd = db.B, nt = db.nt, Np = db.Npad, d = db.d;
  timed(c, st, "gram", Bd * 3.0 * db.N * (double)db.N * d / 2.0, Bd * 8.0 * (Np * Np / 2.0 + Np * d),
        [&] { gprx::launch_gram(db, st); });
  factor_rec(c, st, db, 0, db.nt, 0);
  timed(c, st, "alpha", Bd * Np * nt, Bd * 8.0 * Np * nt, [&] { gprx::launch_alpha(db, st, 0); });
  timed(c, st, "alpha", Bd * Np * Np, Bd * 8.0 * Np * Np / 2.0, [&] { gprx::launch_alpha(db, st, 1); });
  if (want_grad)
    timed(c, st, "lauum_grad", Bd * (Np * Np * Np / 3.0 + Np * Np * d + 4.0 * Np * Np),
          Bd * 8.0 * (Np * Np + Np * (db.xs + 2.0)),  // minimum: Mt upper, Kf lower, Xc, alpha once
          [&] { gprx::launch_lauum_grad(db, st); });
  timed(c, st, "finalize", Bd * 2.0 * db.N, Bd * 16.0 * db.N, [&] { gprx::launch_finalize(db, want_grad ? 1 : 0, st); });
  if (want_pred) predict_group(c, st, db);
}

// One evaluation as a replayed hipGraph: ~40-50 dependent launches per evaluation become one
// graph launch (captured on first use; re-captured when the batch geometry, the test set or a
// kernel variant changes).  Used when profiling is off and the batch is one slot group.
int run_graph(gprx_batch* b, bool want_grad, bool want_pred) {
  gprx_ctx* c = b->ctx;
  const DevBatch& db = b->db;
  const int gi = (want_grad ? 1 : 0) + (want_pred ? 2 : 0);
  const bool same = b->gvalid[gi] && memcmp(&b->gkey[gi], &db, sizeof(DevBatch)) == 0 &&
                    b->gkey_ctx[gi][0] == c->leaf_tiles && b->gkey_ctx[gi][1] == c->small_n &&
                    b->gkey_ctx[gi][2] == c->node_waves;
  if (!same) {
    if (b->gvalid[gi]) (void)hipGraphExecDestroy(b->gexec[gi]);
    b->gvalid[gi] = false;
    hipGraph_t graph = nullptr;
    HIPCHK(c, hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    eval_group(c, c->stream, db, want_grad, want_pred);
    const hipError_t le = hipGetLastError();
    const hipError_t ce = hipStreamEndCapture(c->stream, &graph);
    if (le != hipSuccess || ce != hipSuccess) {
      if (graph) (void)hipGraphDestroy(graph);
      return set_err(c, GPRX_DEVICE_ERROR, std::string("graph capture: ") + hipGetErrorString(le != hipSuccess ? le : ce));
    }
    const hipError_t ie = hipGraphInstantiate(&b->gexec[gi], graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    HIPCHK(c, ie);
    memcpy(&b->gkey[gi], &db, sizeof(DevBatch));
    b->gkey_ctx[gi][0] = c->leaf_tiles;
    b->gkey_ctx[gi][1] = c->small_n;
    b->gkey_ctx[gi][2] = c->node_waves;
    b->gvalid[gi] = true;
  }
  HIPCHK(c, hipGraphLaunch(b->gexec[gi], c->stream));
  return GPRX_OK;
}

// One evaluation on the context stream: direct launches, or the captured graph when enabled.
// factor = false: prediction only, from the last factorisation.
int run_eval(gprx_batch* b, bool want_grad, bool want_pred, bool factor) {
  gprx_ctx* c = b->ctx;
  if (factor && c->use_graphs && !c->prof) return run_graph(b, want_grad, want_pred);
  if (factor) eval_group(c, c->stream, b->db, want_grad, want_pred);
  else if (want_pred) predict_group(c, c->stream, b->db);
  HIPCHK(c, hipGetLastError());
  return GPRX_OK;
}

// Per-call launch geometry from the context options and the batch size.
void set_geometry(const gprx_ctx* c, DevBatch& db) {
  db.small_n = c->small_n > 0 ? c->small_n : (db.B >= 32 ? 4 : 64);  // small batches: more, smaller units
}

}  // namespace

extern "C" {

int gprx_abi_version(void) { return GPRX_ABI_VERSION; }

int gprx_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

const char* gprx_status_string(int s) {
  switch (s) {
    case GPRX_OK: return "ok";
    case GPRX_NOT_POSITIVE_DEFINITE: return "not positive definite";
    case GPRX_INVALID_ARGUMENT: return "invalid argument";
    case GPRX_DEVICE_ERROR: return "device error";
    case GPRX_OUT_OF_MEMORY: return "out of memory";
    case GPRX_NOT_READY: return "not ready";
  }
  return "unknown";
}

int gprx_ctx_create(int device, gprx_ctx** out) {
  if (!out) return GPRX_INVALID_ARGUMENT;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return GPRX_DEVICE_ERROR;
  if (device < 0 || device >= n) return GPRX_INVALID_ARGUMENT;
  gprx_ctx* c = new gprx_ctx();
  c->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return GPRX_DEVICE_ERROR;
  }
  {  // kernel attributes of this device, once, before any context on it can launch
    static std::mutex m;
    static std::map<int, std::unique_ptr<std::once_flag>> once;
    std::once_flag* f;
    {
      std::lock_guard<std::mutex> g(m);
      auto& p = once[device];
      if (!p) p.reset(new std::once_flag());
      f = p.get();
    }
    std::call_once(*f, [] { gprx::set_kernel_attributes(); });
  }
  *out = c;
  return GPRX_OK;
}

void gprx_ctx_destroy(gprx_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  while (!c->batches.empty()) gprx_batch_destroy(*c->batches.begin());  // handles become invalid
  for (auto& p : c->pending) {
    (void)hipEventDestroy(p.a);
    (void)hipEventDestroy(p.b);
  }
  for (auto e : c->evpool) (void)hipEventDestroy(e);
  if (c->rbuf) (void)hipFree(c->rbuf);
  (void)hipStreamDestroy(c->stream);
  delete c;
}

const char* gprx_ctx_last_error(const gprx_ctx* c) { return c ? c->err.c_str() : "null context"; }

int gprx_ctx_set_dist_mode(gprx_ctx* c, int mode) {
  if (!c || (mode != GPRX_DIST_EXPANDED && mode != GPRX_DIST_DIRECT)) return GPRX_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> g(c->mu);
  c->dist_mode = mode;
  return GPRX_OK;
}

int gprx_ctx_device(const gprx_ctx* c) { return c ? c->device : -1; }

int gprx_ctx_set_option(gprx_ctx* c, int option, int value) {
  if (!c) return GPRX_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> g(c->mu);
  switch (option) {
    case GPRX_OPT_LEAF_TILES:
      if (value < 0 || value > 8) return set_err(c, GPRX_INVALID_ARGUMENT, "leaf tiles: 0 (auto) .. 8");
      c->leaf_tiles = value;
      return GPRX_OK;
    case GPRX_OPT_SMALL_N:
      if (value < 0) return set_err(c, GPRX_INVALID_ARGUMENT, "small_n: >= 0 (0 = auto)");
      c->small_n = value;
      return GPRX_OK;
    case GPRX_OPT_GRAPHS:
      c->use_graphs = value != 0;
      return GPRX_OK;
    case GPRX_OPT_NODE_WAVES:
      if (value != 0 && value != 4 && value != 8) return set_err(c, GPRX_INVALID_ARGUMENT, "node waves: 0 (auto), 4 or 8");
      c->node_waves = value;
      return GPRX_OK;
  }
  return set_err(c, GPRX_INVALID_ARGUMENT, "unknown option");
}

int gprx_ctx_set_profiling(gprx_ctx* c, int enable) {
  if (!c) return GPRX_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> g(c->mu);
  c->prof = enable != 0;
  return GPRX_OK;
}

int gprx_ctx_kernel_stats(gprx_ctx* c, const char* kernel, double* total_ms, int64_t* launches, double* algo_flops,
                          double* algo_bytes) {
  if (!c || !kernel) return GPRX_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> g(c->mu);
  auto it = c->stats.find(kernel);
  KStat s = it == c->stats.end() ? KStat() : it->second;
  if (total_ms) *total_ms = s.ms;
  if (launches) *launches = s.n;
  if (algo_flops) *algo_flops = s.flops;
  if (algo_bytes) *algo_bytes = s.bytes;
  return GPRX_OK;
}

int gprx_ctx_reset_stats(gprx_ctx* c) {
  if (!c) return GPRX_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> g(c->mu);
  c->stats.clear();
  return GPRX_OK;
}

static void batch_free(gprx_batch* b);

int gprx_batch_create(gprx_ctx* c, int B, int d, int N, int M_max, gprx_batch** out) {
  if (!c || !out) return GPRX_INVALID_ARGUMENT;
  *out = nullptr;
  if (B < 1 || d < 1 || d > gprx::DMAX || N < 1 || M_max < 0)
    return set_err(c, GPRX_INVALID_ARGUMENT, "gprx_batch_create: need B>=1, 1<=d<=64, N>=1, M_max>=0");
  if (!sizes_addressable(pad64(N), std::max<size_t>(pad64(M_max), TS)))
    return set_err(c, GPRX_INVALID_ARGUMENT,
                   "gprx_batch_create: Npad * max(Npad, Mpad) * 8 must stay below the 2 GiB buffer range (N <= 16320)");
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return GPRX_DEVICE_ERROR;
  gprx_batch* b = new gprx_batch();
  b->ctx = c;
  c->batches.insert(b);
  DevBatch& db = b->db;
  db.B = B;
  db.d = d;
  db.N = N;
  db.Npad = ((N + TS - 1) / TS) * TS;
  db.nt = db.Npad / TS;
  db.ntl = db.nt * (db.nt + 1) / 2;
  db.ld = db.Npad;
  db.mat = (size_t)db.Npad * db.Npad;
  db.pst = d + 4;
  db.gps = d + 2;
  db.nlj = gprx::lauum_plan(db.nt, d, &db.ngu, &db.nimg, nullptr);
  const size_t Bs = B;
  int rc = GPRX_OK;
  auto fail = [&](int r) {  // under c->mu: unlink here, free without re-locking
    c->batches.erase(b);
    batch_free(b);
    return r;
  };
  if (db.nlj < 1) return fail(set_err(c, GPRX_INVALID_ARGUMENT, "gprx_batch_create: lauum plan failed"));
  if ((rc = dalloc(b, &db.X, Bs * db.Npad * d))) return fail(rc);
  db.xs = d | 1;
  if ((rc = dalloc(b, &db.Xc, Bs * db.Npad * db.xs))) return fail(rc);
  if ((rc = dalloc(b, &db.Y, Bs * db.Npad))) return fail(rc);
  if ((rc = dalloc(b, &db.K, Bs * db.mat))) return fail(rc);
  if ((rc = dalloc(b, &db.S, Bs * db.mat))) return fail(rc);
  if ((rc = dalloc(b, &db.Lw, Bs * db.mat))) return fail(rc);
  if ((rc = dalloc(b, &db.Linv, Bs * db.mat))) return fail(rc);
  if ((rc = dalloc(b, &db.Mt, Bs * db.mat))) return fail(rc);
  if ((rc = dalloc(b, &db.z, Bs * db.Npad))) return fail(rc);
  if ((rc = dalloc(b, &db.zp, Bs * 2 * db.nt * (size_t)db.Npad))) return fail(rc);
  if ((rc = dalloc(b, &db.alpha, Bs * db.Npad))) return fail(rc);
  if ((rc = dalloc(b, &db.params, Bs * db.pst))) return fail(rc);
  if ((rc = dalloc(b, &db.theta, Bs * (d + 2)))) return fail(rc);
  if ((rc = dalloc(b, &db.logdet_part, Bs * db.nt))) return fail(rc);
  if ((rc = dalloc(b, &db.grad_part, Bs * db.ngu * db.gps))) return fail(rc);
  if ((rc = dalloc(b, &db.out, Bs * (d + 3)))) return fail(rc);
  if ((rc = dalloc(b, &db.status, 2 * Bs))) return fail(rc);
  db.info = db.status + Bs;
  if ((rc = dalloc(b, &db.lauum_order, 2 * gprx::LU * (size_t)db.nlj))) return fail(rc);
  if ((rc = dalloc(b, &b->opt_active, Bs))) return fail(rc);
  {
    std::vector<int> ord(2 * gprx::LU * (size_t)db.nlj);
    int nu, ni;
    gprx::lauum_plan(db.nt, d, &nu, &ni, ord.data());
    if (hipMemcpy(db.lauum_order, ord.data(), ord.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess)
      return fail(GPRX_DEVICE_ERROR);
  }
  if ((rc = alloc_test(b, M_max))) return fail(rc);
  if (hipHostMalloc((void**)&b->h_params, Bs * db.pst * sizeof(double)) != hipSuccess ||
      hipHostMalloc((void**)&b->h_out, Bs * (d + 3) * sizeof(double)) != hipSuccess ||
      hipHostMalloc((void**)&b->h_status, 2 * Bs * sizeof(int)) != hipSuccess) {
    (void)hipGetLastError();
    return fail(set_err(c, GPRX_OUT_OF_MEMORY, "hipHostMalloc failed"));
  }
  // zero padding of X / Y (pad columns never enter a result; kept finite)
  if (hipMemset(db.X, 0, Bs * db.Npad * d * sizeof(double)) != hipSuccess ||
      hipMemset(db.Y, 0, Bs * db.Npad * sizeof(double)) != hipSuccess ||
      hipMemset(db.Lw, 0, Bs * db.mat * sizeof(double)) != hipSuccess ||
      hipMemset(db.Linv, 0, Bs * db.mat * sizeof(double)) != hipSuccess ||
      hipMemset(db.Mt, 0, Bs * db.mat * sizeof(double)) != hipSuccess ||
      hipMemset(db.S, 0, Bs * db.mat * sizeof(double)) != hipSuccess)
    return fail(GPRX_DEVICE_ERROR);
  *out = b;
  return GPRX_OK;
}

// Frees a batch that is no longer in its context's set (the caller holds no lock, or the creating
// call's own lock: gprx_batch_create's failure path).
static void batch_free(gprx_batch* b) {
  if (b->ctx) (void)hipSetDevice(b->ctx->device);
  if (b->ctx) (void)hipStreamSynchronize(b->ctx->stream);
  for (int i = 0; i < 4; ++i)
    if (b->gvalid[i]) (void)hipGraphExecDestroy(b->gexec[i]);
  for (void* p : b->allocs) (void)hipFree(p);
  if (b->h_params) (void)hipHostFree(b->h_params);
  if (b->h_out) (void)hipHostFree(b->h_out);
  if (b->h_mu) (void)hipHostFree(b->h_mu);
  if (b->h_var) (void)hipHostFree(b->h_var);
  if (b->h_status) (void)hipHostFree(b->h_status);
  delete b;
}

void gprx_batch_destroy(gprx_batch* b) {
  if (!b) return;
  if (b->ctx) {
    std::lock_guard<std::mutex> g(b->ctx->mu);
    b->ctx->batches.erase(b);
  }
  batch_free(b);
}

int gprx_batch_dims(const gprx_batch* b, int* B, int* d, int* N, int* M_max) {
  if (!b) return GPRX_INVALID_ARGUMENT;
  if (B) *B = b->db.B;
  if (d) *d = b->db.d;
  if (N) *N = b->db.N;
  if (M_max) *M_max = b->db.Mpad;
  return GPRX_OK;
}

int gprx_batch_bytes(int B, int d, int N, int M_max, uint64_t* bytes) {
  if (bytes) *bytes = 0;
  if (!bytes || B < 1 || d < 1 || d > gprx::DMAX || N < 1 || M_max < 0) return GPRX_INVALID_ARGUMENT;
  const size_t Npad = pad64(N), Mpad = std::max<size_t>(pad64(M_max), TS);
  if (!sizes_addressable(Npad, Mpad)) return GPRX_INVALID_ARGUMENT;
  *bytes = batch_bytes((size_t)B, d, Npad, Mpad);
  return GPRX_OK;
}

int gprx_ctx_mem_info(gprx_ctx* c, uint64_t* free_bytes, uint64_t* total_bytes) {
  if (!c) return GPRX_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return GPRX_DEVICE_ERROR;
  size_t f = 0, t = 0;
  HIPCHK(c, hipMemGetInfo(&f, &t));
  if (free_bytes) *free_bytes = f;
  if (total_bytes) *total_bytes = t;
  return GPRX_OK;
}

int gprx_batch_set_train(gprx_batch* b, const double* X, int64_t xs, const double* Y, int64_t ys, int mem) {
  if (!b || !X || !Y || xs < 0 || ys < 0) return GPRX_INVALID_ARGUMENT;
  gprx_ctx* c = b->ctx;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return GPRX_DEVICE_ERROR;
  DevBatch& db = b->db;
  int rc;
  for (int s = 0; s < db.B; ++s) {
    // X slot: d x N contiguous (column t = CState t) -> d x Npad (tail zero)
    if ((rc = copy_in(c, db.X + (size_t)s * db.Npad * db.d, X + (size_t)s * xs, (size_t)db.N * db.d * sizeof(double), mem)))
      return rc;
    if ((rc = copy_in(c, db.Y + (size_t)s * db.Npad, Y + (size_t)s * ys, (size_t)db.N * sizeof(double), mem))) return rc;
  }
  gprx::launch_center(db, c->stream);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  b->have_train = true;
  b->factored = false;
  return GPRX_OK;
}

int gprx_batch_set_test(gprx_batch* b, const double* Xs, int M, int64_t xss, int mem) {
  if (!b || (!Xs && M > 0) || M < 0 || xss < 0) return GPRX_INVALID_ARGUMENT;
  gprx_ctx* c = b->ctx;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return GPRX_DEVICE_ERROR;
  DevBatch& db = b->db;
  if (M > db.Mpad) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    free_test(b);
    int rc = alloc_test(b, M);
    if (rc) return rc;
  }
  HIPCHK(c, hipMemsetAsync(db.Xs, 0, (size_t)db.B * db.Mpad * db.d * sizeof(double), c->stream));
  int rc;
  for (int s = 0; s < db.B && M > 0; ++s)
    if ((rc = copy_in(c, db.Xs + (size_t)s * db.Mpad * db.d, Xs + (size_t)s * xss, (size_t)M * db.d * sizeof(double), mem)))
      return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  db.M = M;
  b->have_test = M > 0;
  return GPRX_OK;
}

// Page-locked host memory (hipHostMalloc / registered, e.g. torch's pinned tensors): the device
// writes it by DMA, so the predictive outputs can go straight into the caller's buffer (one
// pitched copy) instead of through the batch's staging buffer and a host copy per slot.
static bool pinned_host(const void* p) {
  if (!p) return false;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory: not known to the runtime
    return false;
  }
  return a.type == hipMemoryTypeHost;
}
// queue the copy of a [B][Mpad] device output to the caller's [B][M] buffer when it is pinned;
// returns whether it did (else the caller stages it)
static bool out_direct(gprx_ctx* c, double* dst, const double* src, const DevBatch& db) {
  if (!pinned_host(dst)) return false;
  return hipMemcpy2DAsync(dst, (size_t)db.M * sizeof(double), src, (size_t)db.Mpad * sizeof(double), (size_t)db.M * sizeof(double),
                          db.B, hipMemcpyDeviceToHost, c->stream) == hipSuccess;
}

static int batch_predict_locked(gprx_batch* b, double* mu, double* var) {
  gprx_ctx* c = b->ctx;
  DevBatch& db = b->db;
  if (!b->factored) return set_err(c, GPRX_NOT_READY, "predict before a successful factorisation");
  if (!b->have_test || db.M == 0) return GPRX_OK;
  db.want_var = var != nullptr;
  int rc = run_eval(b, false, true, false);
  if (rc) return rc;
  const bool dmu = mu && out_direct(c, mu, db.out_mu, db), dvar = var && out_direct(c, var, db.out_var, db);
  if (mu && !dmu)
    HIPCHK(c, hipMemcpyAsync(b->h_mu, db.out_mu, (size_t)db.B * db.Mpad * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  if (var && !dvar)
    HIPCHK(c, hipMemcpyAsync(b->h_var, db.out_var, (size_t)db.B * db.Mpad * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  collect(c);
  for (int s = 0; s < db.B; ++s) {
    if (mu && !dmu) memcpy(mu + (size_t)s * db.M, b->h_mu + (size_t)s * db.Mpad, db.M * sizeof(double));
    if (var && !dvar) memcpy(var + (size_t)s * db.M, b->h_var + (size_t)s * db.Mpad, db.M * sizeof(double));
  }
  return GPRX_OK;
}

int gprx_batch_run(gprx_batch* b, const double* theta, unsigned flags, double* mll, double* grad, double* mu,
                   double* var, int* status, int* info) {
  if (!b || !theta) return GPRX_INVALID_ARGUMENT;
  gprx_ctx* c = b->ctx;
  std::lock_guard<std::mutex> g(c->mu);
  if (!b->have_train) return set_err(c, GPRX_INVALID_ARGUMENT, "gprx_batch_run before gprx_batch_set_train");
  if (hipSetDevice(c->device) != hipSuccess) return GPRX_DEVICE_ERROR;
  DevBatch& db = b->db;
  db.dist_mode = c->dist_mode;
  db.want_var = var != nullptr;
  set_geometry(c, db);
  const int d = db.d, B = db.B, np = d + 2;
  // hyper-parameters -> kernel parameters on the device (derive_params: SEArd / GPE's
  // il2 = exp(-2 log ell), sf2 = exp(2 log sf), noise = exp(2 logNoise) + eps()); h_params is the
  // pinned staging buffer (pst >= d + 2 doubles per slot)
  memcpy(b->h_params, theta, (size_t)B * np * sizeof(double));
  HIPCHK(c, hipMemcpyAsync(db.theta, b->h_params, (size_t)B * np * sizeof(double), hipMemcpyHostToDevice, c->stream));
  gprx::launch_params(db, c->stream);
  HIPCHK(c, hipGetLastError());
  const bool want_grad = (flags & GPRX_WANT_GRAD) != 0;
  const bool want_pred = (flags & GPRX_WANT_PREDICT) != 0 && b->have_test && db.M > 0;
  {
    int rc = run_eval(b, want_grad, want_pred, true);
    if (rc) return rc;
  }
  HIPCHK(c, hipMemcpyAsync(b->h_out, db.out, (size_t)B * (d + 3) * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(b->h_status, db.status, 2 * (size_t)B * sizeof(int), hipMemcpyDeviceToHost, c->stream));
  bool dmu = false, dvar = false;  // predictive outputs copied straight into pinned caller buffers
  if (want_pred) {
    dmu = mu && out_direct(c, mu, db.out_mu, db);
    dvar = var && out_direct(c, var, db.out_var, db);
    if (mu && !dmu)
      HIPCHK(c, hipMemcpyAsync(b->h_mu, db.out_mu, (size_t)B * db.Mpad * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    if (var && !dvar)
      HIPCHK(c, hipMemcpyAsync(b->h_var, db.out_var, (size_t)B * db.Mpad * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  collect(c);
  int first = GPRX_OK;
  for (int s = 0; s < B; ++s) {
    const int st = b->h_status[s];
    if (status) status[s] = st;
    if (info) info[s] = b->h_status[B + s];
    if (st != GPRX_OK && first == GPRX_OK) first = st;
    const double* o = b->h_out + (size_t)s * (d + 3);
    if (mll) mll[s] = o[0];
    if (grad && want_grad) memcpy(grad + (size_t)s * np, o + 1, np * sizeof(double));
    if (want_pred) {
      if (mu && !dmu) memcpy(mu + (size_t)s * db.M, b->h_mu + (size_t)s * db.Mpad, db.M * sizeof(double));
      if (var && !dvar) memcpy(var + (size_t)s * db.M, b->h_var + (size_t)s * db.Mpad, db.M * sizeof(double));
    }
  }
  b->factored = true;
  if (first != GPRX_OK) set_err(c, first, std::string("gprx_batch_run: ") + gprx_status_string(first));
  return first;
}

int gprx_batch_alpha(gprx_batch* b, double* alpha) {
  if (!b || !alpha) return GPRX_INVALID_ARGUMENT;
  gprx_ctx* c = b->ctx;
  std::lock_guard<std::mutex> g(c->mu);
  if (!b->factored) return set_err(c, GPRX_NOT_READY, "alpha before a successful factorisation");
  if (hipSetDevice(c->device) != hipSuccess) return GPRX_DEVICE_ERROR;
  const DevBatch& db = b->db;
  HIPCHK(c, hipMemcpy2DAsync(alpha, (size_t)db.N * sizeof(double), db.alpha, (size_t)db.Npad * sizeof(double),
                             (size_t)db.N * sizeof(double), db.B, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  // h_status holds the per-slot status of the evaluation that factorised the batch (gprx_batch_run
  // or the optimiser's refit): a slot that failed there has no alpha
  for (int s = 0; s < db.B; ++s)
    if (b->h_status[s] != GPRX_OK)
      for (int t = 0; t < db.N; ++t) alpha[(size_t)s * db.N + t] = NAN;
  return GPRX_OK;
}

int gprx_batch_predict(gprx_batch* b, double* mu, double* var) {
  if (!b) return GPRX_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> g(b->ctx->mu);
  if (hipSetDevice(b->ctx->device) != hipSuccess) return GPRX_DEVICE_ERROR;
  return batch_predict_locked(b, mu, var);
}

// ---- device hyper-parameter optimisation (gprx_lbfgs.hip) ---------------------------------------
static_assert(GPRX_STOP_ITERATIONS == gprx::LB_STOP_ITERATIONS && GPRX_STOP_G_TOL == gprx::LB_STOP_G_TOL &&
                  GPRX_STOP_X_TOL == gprx::LB_STOP_X_TOL && GPRX_STOP_F_TOL == gprx::LB_STOP_F_TOL &&
                  GPRX_STOP_LINESEARCH == gprx::LB_STOP_LINESEARCH && GPRX_STOP_MAX_EVALS == gprx::LB_STOP_MAX_EVALS &&
                  GPRX_STOP_TIME_LIMIT == gprx::LB_STOP_TIME_LIMIT &&
                  GPRX_STOP_NAN_GRADIENT == gprx::LB_STOP_NAN_GRADIENT,
              "stop codes");

void gprx_opt_defaults(gprx_opt_options* o) {
  if (!o) return;
  o->m = 10;
  o->iterations = 1000;
  o->max_evals = -1;
  o->ls_iterations = 1000;
  o->scaleinvH0 = 1;
  o->refit = 1;
  o->successive_f_tol = 1;
  o->g_abstol = 1e-8;
  o->time_limit = NAN;  // Optim: no limit
  o->alphaguess = 1.0;
  o->c_1 = 1e-4;
  o->rho_hi = 0.5;
  o->rho_lo = 0.1;
}

int gprx_batch_optimize(gprx_batch* b, const double* theta0, const gprx_opt_options* opt, double* theta_out,
                        double* minimum, int* iterations, int* f_calls, int* g_calls, int* stopped, int* rounds) {
  if (!b || !theta0) return GPRX_INVALID_ARGUMENT;
  gprx_ctx* c = b->ctx;
  std::lock_guard<std::mutex> g(c->mu);
  if (!b->have_train) return set_err(c, GPRX_INVALID_ARGUMENT, "gprx_batch_optimize before gprx_batch_set_train");
  gprx_opt_options o;
  gprx_opt_defaults(&o);
  if (opt) o = *opt;
  if (o.m < 1 || o.m > 64 || o.iterations < 0 || o.ls_iterations < 0 || o.successive_f_tol < 0 || !(o.c_1 > 0.0) || !(o.rho_lo > 0.0) ||
      !(o.rho_hi > 0.0) || !std::isfinite(o.alphaguess) || std::isnan(o.g_abstol))
    return set_err(c, GPRX_INVALID_ARGUMENT, "gprx_batch_optimize: bad options");
  if (hipSetDevice(c->device) != hipSuccess) return GPRX_DEVICE_ERROR;
  DevBatch& db = b->db;
  db.dist_mode = c->dist_mode;
  db.want_var = 0;
  set_geometry(c, db);
  const int B = db.B, n = db.d + 2;
  gprx::LbArgs a{};
  a.n = n;
  a.m = o.m;
  a.max_evals = o.max_evals;
  a.iterations = o.iterations;
  a.ls_iterations = o.ls_iterations;
  a.scaleinvH0 = o.scaleinvH0 ? 1 : 0;
  a.successive_f_tol = o.successive_f_tol;
  a.g_abstol = o.g_abstol;
  a.alphaguess = o.alphaguess;
  a.c_1 = o.c_1;
  a.rho_hi = o.rho_hi;
  a.rho_lo = o.rho_lo;
  // one device block: state, start points, flags, results; one pinned host mirror of the flags
  // and results
  const size_t wsd = (size_t)B * gprx::lb_ws_doubles(n, o.m), rd = (size_t)B * (n + 1);
  const size_t nd = wsd + (size_t)B * n + rd, ni = (size_t)B * (gprx::LB_NI + 1 + 4);
  char* dbuf = nullptr;
  char* hbuf = nullptr;
  if (hipMalloc((void**)&dbuf, nd * sizeof(double) + ni * sizeof(int)) != hipSuccess) {
    (void)hipGetLastError();
    return set_err(c, GPRX_OUT_OF_MEMORY, "gprx_batch_optimize: workspace");
  }
  if (hipHostMalloc((void**)&hbuf, rd * sizeof(double) + (size_t)B * 5 * sizeof(int)) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipFree(dbuf);
    return set_err(c, GPRX_OUT_OF_MEMORY, "gprx_batch_optimize: host buffer");
  }
  struct Free {
    char *d, *h;
    ~Free() {
      (void)hipFree(d);
      (void)hipHostFree(h);
    }
  } fr{dbuf, hbuf};
  a.ws = (double*)dbuf;
  double* th0d = a.ws + wsd;
  a.theta0 = th0d;
  a.result = th0d + (size_t)B * n;
  a.iws = (int*)(a.result + rd);
  // the optimisers' activity flags double as the evaluation mask of the rounds (finished slots are
  // skipped by every kernel); a per-batch buffer, so the captured round graph is reused across calls
  a.active = b->opt_active;
  a.result_i = a.iws + (size_t)B * gprx::LB_NI + B;
  double* h_res = (double*)hbuf;
  int* h_act = (int*)(h_res + rd);
  int* h_ri = h_act + B;
  // theta, L and the factorisation flags are overwritten from here on: the batch holds no valid
  // factorisation until the refit below has succeeded for every slot
  b->factored = false;
  struct Unmask {  // every exit path evaluates all slots again
    DevBatch& db;
    ~Unmask() { db.active = nullptr; }
  } um{db};
  // evaluation trace (gprx_batch_set_opt_trace): per round the evaluated theta and the answer of
  // every slot, staged in pinned memory (copied under the round's own synchronisation)
  const int trr = b->opt_trace ? b->opt_trace_rounds : 0;
  const size_t trs = (size_t)B * (2 * n + 1);  // staged doubles per round: theta(n), out(n + 1)
  std::vector<int> tr_act((size_t)trr * B, 0);
  double* h_tr = nullptr;
  if (trr > 0 && hipHostMalloc((void**)&h_tr, (size_t)trr * trs * sizeof(double)) != hipSuccess) {
    (void)hipGetLastError();
    return set_err(c, GPRX_OUT_OF_MEMORY, "gprx_batch_optimize: trace buffer");
  }
  struct FreeTr {
    double* h;
    ~FreeTr() {
      if (h) (void)hipHostFree(h);
    }
  } ftr{h_tr};
  HIPCHK(c, hipMemcpyAsync(th0d, theta0, (size_t)B * n * sizeof(double), hipMemcpyHostToDevice, c->stream));
  gprx::launch_lbfgs(a, db, 1, c->stream);
  db.active = a.active;
  const auto t0 = std::chrono::steady_clock::now();
  int nr = 0;
  for (;;) {
    HIPCHK(c, hipMemcpyAsync(h_act, a.active, (size_t)B * sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    int act = 0;
    for (int s = 0; s < B; ++s) act += h_act[s] != 0;
    if (!act) break;
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    a.time_up = (o.time_limit >= 0.0 && el > o.time_limit) ? 1 : 0;  // false for NaN
    int rc = run_eval(b, true, false, true);
    if (rc) return rc;
    collect(c);
    if (nr < trr) {
      double* h = h_tr + (size_t)nr * trs;
      memcpy(&tr_act[(size_t)nr * B], h_act, (size_t)B * sizeof(int));
      HIPCHK(c, hipMemcpyAsync(h, db.theta, (size_t)B * n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipMemcpyAsync(h + (size_t)B * n, db.out, (size_t)B * (n + 1) * sizeof(double), hipMemcpyDeviceToHost,
                               c->stream));
    }
    gprx::launch_lbfgs(a, db, 0, c->stream);
    HIPCHK(c, hipGetLastError());
    ++nr;
  }
  HIPCHK(c, hipMemcpyAsync(h_res, a.result, rd * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(h_ri, a.result_i, (size_t)B * 4 * sizeof(int), hipMemcpyDeviceToHost, c->stream));
  db.active = nullptr;
  if (o.refit) {  // optimize!: set_params!(gp, minimizer); update_target!(gp)
    gprx::launch_lbfgs_final(a, db, c->stream);
    int rc = run_eval(b, true, false, true);
    if (rc) return rc;
    HIPCHK(c, hipMemcpyAsync(b->h_out, db.out, (size_t)B * (db.d + 3) * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(b->h_status, db.status, 2 * (size_t)B * sizeof(int), hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  collect(c);
  if (trr > 0) {  // [active, theta(n), mll, dmll(n)] per slot and round; NaN beyond the last round
    const size_t w = 2 * (size_t)n + 2;
    for (int r = 0; r < trr; ++r)
      for (int s = 0; s < B; ++s) {
        double* t = b->opt_trace + ((size_t)r * B + s) * w;
        if (r >= nr) {
          for (size_t q = 0; q < w; ++q) t[q] = NAN;
          continue;
        }
        const double* h = h_tr + (size_t)r * trs;
        t[0] = tr_act[(size_t)r * B + s] ? 1.0 : 0.0;
        memcpy(t + 1, h + (size_t)s * n, n * sizeof(double));
        memcpy(t + 1 + n, h + (size_t)B * n + (size_t)s * (n + 1), (n + 1) * sizeof(double));
      }
  }
  for (int s = 0; s < B; ++s) {
    const double* r = h_res + (size_t)s * (n + 1);
    if (theta_out) memcpy(theta_out + (size_t)s * n, r, n * sizeof(double));
    if (minimum) minimum[s] = r[n];
    const int* ri = h_ri + (size_t)s * 4;
    if (iterations) iterations[s] = ri[0];
    if (f_calls) f_calls[s] = ri[1];
    if (g_calls) g_calls[s] = ri[2];
    if (stopped) stopped[s] = ri[3];
  }
  if (rounds) *rounds = nr;
  if (!o.refit) return GPRX_OK;
  // the refit's per-slot status, as gprx_batch_run reports it: a minimiser that is not finite
  // (status 2) or not positive definite (status 1) is an error of update_target!, and the batch is
  // then not left factorised
  int first = GPRX_OK, bad = -1;
  for (int s = 0; s < B && first == GPRX_OK; ++s)
    if (b->h_status[s] != GPRX_OK) first = b->h_status[s], bad = s;
  if (first != GPRX_OK)
    return set_err(c, first, "gprx_batch_optimize: refit at the minimiser of slot " + std::to_string(bad) + ": " +
                                 gprx_status_string(first));
  b->factored = true;
  return GPRX_OK;
}

int gprx_batch_set_opt_trace(gprx_batch* b, double* trace, int max_rounds, int64_t capacity) {
  if (!b || max_rounds < 0 || (max_rounds > 0 && !trace)) return GPRX_INVALID_ARGUMENT;
  const int64_t need = (int64_t)max_rounds * b->db.B * (2 * (int64_t)(b->db.d + 2) + 2);
  if (max_rounds > 0 && capacity < need)
    return set_err(b->ctx, GPRX_INVALID_ARGUMENT,
                   "gprx_batch_set_opt_trace: capacity " + std::to_string(capacity) + " < max_rounds * B * (2(d+2)+2) = " +
                       std::to_string(need) + " doubles");
  std::lock_guard<std::mutex> g(b->ctx->mu);
  b->opt_trace = max_rounds > 0 ? trace : nullptr;
  b->opt_trace_rounds = max_rounds;
  return GPRX_OK;
}

// ---- single GP ---------------------------------------------------------------------------------
int gprx_gp_create(gprx_ctx* c, const double* X, int d, int N, const double* y, gprx_gp** out) {
  if (!c || !X || !y || !out) return GPRX_INVALID_ARGUMENT;
  *out = nullptr;
  gprx_batch* b = nullptr;
  int rc = gprx_batch_create(c, 1, d, N, 0, &b);
  if (rc) return rc;
  rc = gprx_batch_set_train(b, X, 0, y, 0, GPRX_MEM_HOST);
  if (rc) {
    gprx_batch_destroy(b);
    return rc;
  }
  gprx_gp* gp = new gprx_gp();
  gp->batch = b;
  *out = gp;
  return GPRX_OK;
}

void gprx_gp_destroy(gprx_gp* gp) {
  if (!gp) return;
  gprx_batch_destroy(gp->batch);
  delete gp;
}

int gprx_gp_lml(gprx_gp* gp, const double* theta, double* mll) {
  if (!gp) return GPRX_INVALID_ARGUMENT;
  return gprx_batch_run(gp->batch, theta, 0u, mll, nullptr, nullptr, nullptr, nullptr, nullptr);
}

int gprx_gp_lml_grad(gprx_gp* gp, const double* theta, double* mll, double* grad) {
  if (!gp) return GPRX_INVALID_ARGUMENT;
  return gprx_batch_run(gp->batch, theta, GPRX_WANT_GRAD, mll, grad, nullptr, nullptr, nullptr, nullptr);
}

int gprx_gp_predict(gprx_gp* gp, const double* Xs, int M, double* mu, double* var) {
  if (!gp || M < 0) return GPRX_INVALID_ARGUMENT;
  if (M == 0) return GPRX_OK;
  int rc = gprx_batch_set_test(gp->batch, Xs, M, 0, GPRX_MEM_HOST);
  if (rc) return rc;
  return gprx_batch_predict(gp->batch, mu, var);
}

// ---- rollout in minimal coordinates ------------------------------------------------------------
int gprx_rollout_min(gprx_ctx* c, int mech, int usesin, double dt, int steps, int ngroups,
                     gprx_batch* const* batches, const int* slots, int T, const int* traj_group,
                     const double* start, double* final_state) {
  if (!c) return GPRX_INVALID_ARGUMENT;
  if (mech < GPRX_MECH_P1 || mech > GPRX_MECH_FB || steps < 0 || ngroups < 1 || T < 0 || !std::isfinite(dt))
    return set_err(c, GPRX_INVALID_ARGUMENT, "gprx_rollout_min: bad mechanism / steps / groups / dt");
  if (T == 0) return GPRX_OK;
  if (!batches || !slots || !traj_group || !start || !final_state)
    return set_err(c, GPRX_INVALID_ARGUMENT, "gprx_rollout_min: null argument");
  // coordinates (q, qdot) per mechanism: P1 theta; P2 theta1, theta2 (relative); CP x, theta;
  // FB theta1, theta3 -- the angle coordinates get (sin, cos) features when usesin
  const int nc = mech == GPRX_MECH_P1 ? 1 : 2;
  const int ang0 = mech == GPRX_MECH_CP ? 0 : 1, ang1 = nc > 1 ? 1 : 0;
  const int dobs = (usesin && ang0 ? 3 : 2) + (nc > 1 ? (usesin && ang1 ? 3 : 2) : 0);
  std::lock_guard<std::mutex> g(c->mu);
  std::vector<gprx::RolloutGP> gps((size_t)ngroups * nc);
  for (size_t k = 0; k < gps.size(); ++k) {
    gprx_batch* b = batches[k];
    const int s = slots[k];
    if (!b || b->ctx != c || s < 0 || s >= b->db.B)
      return set_err(c, GPRX_INVALID_ARGUMENT, "gprx_rollout_min: GP " + std::to_string(k) + " is not a slot of a batch of this context");
    if (b->db.d != dobs)
      return set_err(c, GPRX_INVALID_ARGUMENT, "gprx_rollout_min: input dimension " + std::to_string(b->db.d) + " != " + std::to_string(dobs) + " for this mechanism / usesin");
    if (!b->factored) return set_err(c, GPRX_NOT_READY, "gprx_rollout_min: batch not factorised (run it first)");
    if (b->h_status[s] != 0) return set_err(c, b->h_status[s], "gprx_rollout_min: slot " + std::to_string(s) + " failed its last evaluation");
    const DevBatch& db = b->db;
    gps[k] = gprx::RolloutGP{db.X + (size_t)s * db.Npad * db.d, db.alpha + (size_t)s * db.Npad, db.params + (size_t)s * db.pst, db.N, 0};
  }
  for (int t = 0; t < T; ++t)
    if (traj_group[t] < 0 || traj_group[t] >= ngroups) return set_err(c, GPRX_INVALID_ARGUMENT, "gprx_rollout_min: trajectory group out of range");
  if (hipSetDevice(c->device) != hipSuccess) return GPRX_DEVICE_ERROR;
  // one device buffer: [gps | group | start | out]
  const size_t o_grp = gps.size() * sizeof(gprx::RolloutGP);
  const size_t o_st = (o_grp + (size_t)T * sizeof(int) + 15) / 16 * 16;
  const size_t o_out = o_st + (size_t)T * 2 * nc * sizeof(double);
  const size_t need = o_out + (size_t)T * 2 * nc * sizeof(double);
  if (need > c->rcap) {
    if (c->rbuf) HIPCHK(c, hipFree(c->rbuf));
    c->rbuf = nullptr;
    c->rcap = 0;
    HIPCHK(c, hipMalloc(&c->rbuf, need));
    c->rcap = need;
  }
  char* base = (char*)c->rbuf;
  HIPCHK(c, hipMemcpyAsync(base, gps.data(), o_grp, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(base + o_grp, traj_group, (size_t)T * sizeof(int), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(base + o_st, start, (size_t)T * 2 * nc * sizeof(double), hipMemcpyHostToDevice, c->stream));
  gprx::RolloutArgs a{};
  a.gps = (const gprx::RolloutGP*)base;
  a.group = (const int*)(base + o_grp);
  a.start = (const double*)(base + o_st);
  a.out = (double*)(base + o_out);
  a.T = T;
  a.nc = nc;
  a.d = dobs;
  a.steps = steps;
  a.usesin = usesin ? 1 : 0;
  a.ang0 = ang0;
  a.ang1 = ang1;
  a.dt = dt;
  double np = 0.0;
  for (int t = 0; t < T; ++t)
    for (int q = 0; q < nc; ++q) np += gps[(size_t)traj_group[t] * nc + q].N;
  timed(c, c->stream, "rollout", np * steps * (3.0 * dobs + 24.0), np * steps * (dobs + 1) * 8.0,
        [&] { gprx::launch_rollout(a, c->dist_mode, c->stream); });
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(final_state, base + o_out, (size_t)T * 2 * nc * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  collect(c);
  return GPRX_OK;
}

// ---- maximal-coordinate physics -----------------------------------------------------------------
// The experiment mechanisms' joints (examples/utils/data/simulations.jl; oracle/projection_oracle.py
// mechanism()): sub-joints in the order of the equality constraints and their rows.
static bool build_mech(int mech, gprx::MechDev& M) {
  M = gprx::MechDev{};
  struct Sj {
    int kind, rows, a, b;
    double pa[3], pb[3], axis[3];
  };
  std::vector<Sj> js;
  const double O[3] = {0, 0, 0}, EX[3] = {1, 0, 0}, EY[3] = {0, 1, 0};
  auto add = [&](int kind, int rows, int a, int b, const double* pa, const double* pb, const double* ax) {
    Sj j{kind, rows, a, b, {pa[0], pa[1], pa[2]}, {pb[0], pb[1], pb[2]}, {ax[0], ax[1], ax[2]}};
    js.push_back(j);
  };
  auto rev = [&](int a, int b, const double* ax, const double* pa, const double* pb) {
    add(0, 3, a, b, pa, pb, ax);  // Translational3
    add(1, 2, a, b, pa, pb, ax);  // Rotational2 (free about the axis)
  };
  const double h1[3] = {0, 0, 0.5}, h1m[3] = {0, 0, -0.5}, hcp[3] = {0, 0, 0.25};
  switch (mech) {
    case GPRX_MECH_P1: M.nb = 1; rev(0, 1, EX, O, h1); break;
    case GPRX_MECH_P2: M.nb = 2; rev(0, 1, EX, O, h1); rev(1, 2, EX, h1m, h1); break;
    case GPRX_MECH_CP:
      M.nb = 2;
      add(0, 2, 0, 1, O, O, EY);  // Prismatic: Translational2 (free along y) + Rotational3
      add(1, 3, 0, 1, O, O, EY);
      rev(1, 2, EX, O, hcp);
      break;
    case GPRX_MECH_FB:
      M.nb = 4;
      rev(0, 1, EX, O, h1);
      rev(1, 2, EX, h1m, h1);
      add(0, 2, 1, 3, h1, h1, EX);  // Cylindrical: Translational2 + Rotational2
      add(1, 2, 1, 3, h1, h1, EX);
      rev(3, 4, EX, h1m, h1);
      rev(2, 4, EX, h1m, h1m);
      break;
    default: return false;
  }
  // bodies as examples/utils/data/simulations.jl builds them (gprx/vi.py MECHANISMS): m = 1, J = I m
  // l^2 / 12 for the unit links, the cart-pole's pole l = 0.5 (I / 48) and its cart a 0.2 x 0.3 x 0.1
  // box, diag(y^2 + z^2, x^2 + z^2, x^2 + y^2) m / 12
  for (int b = 0; b < M.nb; ++b) {
    M.m[b] = 1.0;
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) M.J[b][r][c] = r == c ? 1.0 / 12.0 : 0.0;
  }
  if (mech == GPRX_MECH_CP) {
    const double x = 0.2, y = 0.3, z = 0.1;
    M.J[0][0][0] = (y * y + z * z) * 1.0 / 12.0;
    M.J[0][1][1] = (x * x + z * z) * 1.0 / 12.0;
    M.J[0][2][2] = (x * x + y * y) * 1.0 / 12.0;
    for (int r = 0; r < 3; ++r) M.J[1][r][r] = 1.0 / 48.0;
  }
  int row = 0;
  M.nsub = (int)js.size();
  for (int k = 0; k < M.nsub; ++k) {
    gprx::SubJoint& S = M.sub[k];
    const Sj& j = js[k];
    S.kind = j.kind;
    S.a = j.a;
    S.b = j.b;
    S.rows = j.rows;
    S.row0 = row;
    row += j.rows;
    for (int i = 0; i < 3; ++i) {
      S.pa[i] = j.pa[i];
      S.pb[i] = j.pb[i];
    }
    if (j.rows == 3) {
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) S.C[r][c] = r == c ? 1.0 : 0.0;
    } else {  // two orthonormal rows normal to the axis (oracle normal_rows)
      const double* a = j.axis;
      const double na = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
      const double u[3] = {a[0] / na, a[1] / na, a[2] / na};
      const double t[3] = {std::fabs(u[2]) < 0.9 ? 0.0 : 1.0, 0.0, std::fabs(u[2]) < 0.9 ? 1.0 : 0.0};
      double v1[3] = {u[1] * t[2] - u[2] * t[1], u[2] * t[0] - u[0] * t[2], u[0] * t[1] - u[1] * t[0]};
      const double n1 = std::sqrt(v1[0] * v1[0] + v1[1] * v1[1] + v1[2] * v1[2]);
      for (double& x : v1) x /= n1;
      const double v2[3] = {u[1] * v1[2] - u[2] * v1[1], u[2] * v1[0] - u[0] * v1[2], u[0] * v1[1] - u[1] * v1[0]};
      for (int c = 0; c < 3; ++c) {
        S.C[0][c] = v1[c];
        S.C[1][c] = v2[c];
        S.C[2][c] = 0.0;
      }
    }
  }
  M.nd = row;
  return 6 * M.nb + M.nd <= gprx::PJ_MAXN;
}

// device scratch of a context for the physics calls: [args | in | out], grown on demand
static int ctx_scratch(gprx_ctx* c, size_t need, char** base) {
  if (need > c->rcap) {
    if (c->rbuf) HIPCHK(c, hipFree(c->rbuf));
    c->rbuf = nullptr;
    c->rcap = 0;
    HIPCHK(c, hipMalloc(&c->rbuf, need));
    c->rcap = need;
  }
  *base = (char*)c->rbuf;
  return GPRX_OK;
}
static size_t al16(size_t x) { return (x + 15) / 16 * 16; }

int gprx_projectv(gprx_ctx* c, int mech, double dt, int T, const double* cstates, const double* vw_pred,
                  double regularizer, int newton_iter, double eps, double* vw_out, int* iterations, int* status) {
  if (!c) return GPRX_INVALID_ARGUMENT;
  gprx::MechDev M;
  if (!build_mech(mech, M) || T < 0 || newton_iter < 0 || !(dt > 0.0) || !std::isfinite(regularizer) || !(eps >= 0.0))
    return set_err(c, GPRX_INVALID_ARGUMENT, "gprx_projectv: bad mechanism / T / newton_iter / dt / regularizer / eps");
  if (T == 0) return GPRX_OK;
  if (!cstates || !vw_pred || !vw_out) return set_err(c, GPRX_INVALID_ARGUMENT, "gprx_projectv: null argument");
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return GPRX_DEVICE_ERROR;
  const int nb = M.nb;
  const size_t o_cs = 0, o_vw = al16(o_cs + (size_t)T * 13 * nb * 8), o_out = al16(o_vw + (size_t)T * 6 * nb * 8),
               o_it = al16(o_out + (size_t)T * 6 * nb * 8), o_st = al16(o_it + (size_t)T * 4), need = al16(o_st + (size_t)T * 4);
  char* base;
  int rc = ctx_scratch(c, need, &base);
  if (rc) return rc;
  HIPCHK(c, hipMemcpyAsync(base + o_cs, cstates, (size_t)T * 13 * nb * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(base + o_vw, vw_pred, (size_t)T * 6 * nb * 8, hipMemcpyHostToDevice, c->stream));
  gprx::ProjArgs a{};
  a.mech = M;
  a.dt = dt;
  a.reg = regularizer;
  a.eps = eps;
  a.iters = newton_iter;
  a.T = T;
  a.cs = (const double*)(base + o_cs);
  a.vw = (const double*)(base + o_vw);
  a.out = (double*)(base + o_out);
  a.iters_out = (int*)(base + o_it);
  a.status = (int*)(base + o_st);
  timed(c, c->stream, "projectv", 0.0, (double)T * 8.0 * (13 + 12) * nb, [&] { gprx::launch_project(a, c->stream); });
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(vw_out, base + o_out, (size_t)T * 6 * nb * 8, hipMemcpyDeviceToHost, c->stream));
  std::vector<int> it(T), st(T);
  HIPCHK(c, hipMemcpyAsync(it.data(), base + o_it, (size_t)T * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(st.data(), base + o_st, (size_t)T * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  collect(c);
  if (iterations) memcpy(iterations, it.data(), (size_t)T * 4);
  if (status) memcpy(status, st.data(), (size_t)T * 4);
  return GPRX_OK;
}

int gprx_vi_step(gprx_ctx* c, int mech, double dt, int T, const double* cstates, double regularizer, int newton_iter,
                 double eps, double* out, int* iterations, int* status) {
  if (!c) return GPRX_INVALID_ARGUMENT;
  gprx::MechDev M;
  if (!build_mech(mech, M) || T < 0 || newton_iter < 0 || !(dt > 0.0) || !std::isfinite(regularizer) || !(eps >= 0.0))
    return set_err(c, GPRX_INVALID_ARGUMENT, "gprx_vi_step: bad mechanism / T / newton_iter / dt / regularizer / eps");
  if (T == 0) return GPRX_OK;
  if (!cstates || !out) return set_err(c, GPRX_INVALID_ARGUMENT, "gprx_vi_step: null argument");
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return GPRX_DEVICE_ERROR;
  const int nb = M.nb;
  const size_t o_cs = 0, o_out = al16(o_cs + (size_t)T * 13 * nb * 8), o_it = al16(o_out + (size_t)T * 13 * nb * 8),
               o_st = al16(o_it + (size_t)T * 4), need = al16(o_st + (size_t)T * 4);
  char* base;
  int rc = ctx_scratch(c, need, &base);
  if (rc) return rc;
  HIPCHK(c, hipMemcpyAsync(base + o_cs, cstates, (size_t)T * 13 * nb * 8, hipMemcpyHostToDevice, c->stream));
  gprx::ViArgs a{};
  a.mech = M;
  a.dt = dt;
  a.reg = regularizer;
  a.eps = eps;
  a.grav = 9.81;  // |mechanism.g| (simulations.jl; gprx/vi.py GRAV)
  a.iters = newton_iter;
  a.T = T;
  a.cs = (const double*)(base + o_cs);
  a.out = (double*)(base + o_out);
  a.iters_out = (int*)(base + o_it);
  a.status = (int*)(base + o_st);
  timed(c, c->stream, "vi_step", 0.0, (double)T * 8.0 * 26 * nb, [&] { gprx::launch_vi_step(a, c->stream); });
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(out, base + o_out, (size_t)T * 13 * nb * 8, hipMemcpyDeviceToHost, c->stream));
  std::vector<int> it(T), st(T);
  HIPCHK(c, hipMemcpyAsync(it.data(), base + o_it, (size_t)T * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(st.data(), base + o_st, (size_t)T * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  collect(c);
  if (iterations) memcpy(iterations, it.data(), (size_t)T * 4);
  if (status) memcpy(status, st.data(), (size_t)T * 4);
  return GPRX_OK;
}

int gprx_rollout_max(gprx_ctx* c, int mech, double dt, int steps, double regularizer, int ngroups,
                     gprx_batch* const* batches, const int* slots, int G, const int* vw_idx1, int T,
                     const int* traj_group, const double* start, double* final_state, double* proj_err, int* status) {
  if (!c) return GPRX_INVALID_ARGUMENT;
  gprx::MechDev M;
  if (!build_mech(mech, M) || steps < 0 || ngroups < 1 || T < 0 || G < 1 || G > gprx::PJ_MAXG || !(dt > 0.0) ||
      !std::isfinite(regularizer))
    return set_err(c, GPRX_INVALID_ARGUMENT, "gprx_rollout_max: bad mechanism / steps / groups / G / dt / regularizer");
  if (T == 0) return GPRX_OK;
  if (!batches || !slots || !vw_idx1 || !traj_group || !start || !final_state)
    return set_err(c, GPRX_INVALID_ARGUMENT, "gprx_rollout_max: null argument");
  const int d = 13 * M.nb;
  gprx::RolloutMaxArgs a{};
  for (int g = 0; g < G; ++g) {
    const int k = (vw_idx1[g] - 1) % 13;
    if (vw_idx1[g] < 1 || vw_idx1[g] > d || k < 7)
      return set_err(c, GPRX_INVALID_ARGUMENT, "gprx_rollout_max: vw index " + std::to_string(vw_idx1[g]) +
                                                   " is not a velocity / angular-velocity slot of the CState");
    a.vw[g] = vw_idx1[g] - 1;
  }
  std::lock_guard<std::mutex> lk(c->mu);
  std::vector<gprx::RolloutGP> gps((size_t)ngroups * G);
  for (size_t k = 0; k < gps.size(); ++k) {
    gprx_batch* b = batches[k];
    const int s = slots[k];
    if (!b || b->ctx != c || s < 0 || s >= b->db.B)
      return set_err(c, GPRX_INVALID_ARGUMENT, "gprx_rollout_max: GP " + std::to_string(k) + " is not a slot of a batch of this context");
    if (b->db.d != d)
      return set_err(c, GPRX_INVALID_ARGUMENT, "gprx_rollout_max: input dimension " + std::to_string(b->db.d) + " != 13 nbodies");
    if (!b->factored) return set_err(c, GPRX_NOT_READY, "gprx_rollout_max: batch not factorised (run it first)");
    if (b->h_status[s] != 0) return set_err(c, b->h_status[s], "gprx_rollout_max: slot " + std::to_string(s) + " failed its last evaluation");
    const DevBatch& db = b->db;
    gps[k] = gprx::RolloutGP{db.X + (size_t)s * db.Npad * db.d, db.alpha + (size_t)s * db.Npad, db.params + (size_t)s * db.pst, db.N, 0};
  }
  for (int t = 0; t < T; ++t)
    if (traj_group[t] < 0 || traj_group[t] >= ngroups) return set_err(c, GPRX_INVALID_ARGUMENT, "gprx_rollout_max: trajectory group out of range");
  if (hipSetDevice(c->device) != hipSuccess) return GPRX_DEVICE_ERROR;
  const size_t o_grp = al16(gps.size() * sizeof(gprx::RolloutGP)), o_st = al16(o_grp + (size_t)T * 4),
               o_out = al16(o_st + (size_t)T * d * 8), o_pe = al16(o_out + (size_t)T * d * 8),
               o_ss = al16(o_pe + (size_t)T * 8), need = al16(o_ss + (size_t)T * 4);
  char* base;
  int rc = ctx_scratch(c, need, &base);
  if (rc) return rc;
  HIPCHK(c, hipMemcpyAsync(base, gps.data(), gps.size() * sizeof(gprx::RolloutGP), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(base + o_grp, traj_group, (size_t)T * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(base + o_st, start, (size_t)T * d * 8, hipMemcpyHostToDevice, c->stream));
  a.mech = M;
  a.dt = dt;
  a.reg = regularizer;
  a.eps = 1e-10;  // projectv! defaults (implicitProjection.jl:80)
  a.iters = 100;
  a.steps = steps;
  a.T = T;
  a.G = G;
  a.d = d;
  a.gps = (const gprx::RolloutGP*)base;
  a.group = (const int*)(base + o_grp);
  a.start = (const double*)(base + o_st);
  a.out = (double*)(base + o_out);
  a.perr = (double*)(base + o_pe);
  a.status = (int*)(base + o_ss);
  double np = 0.0;
  for (int t = 0; t < T; ++t)
    for (int g = 0; g < G; ++g) np += gps[(size_t)traj_group[t] * G + g].N;
  timed(c, c->stream, "rollout_max", np * steps * (3.0 * d + 24.0), np * steps * (d + 1) * 8.0,
        [&] { gprx::launch_rollout_max(a, c->dist_mode, c->stream); });
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(final_state, base + o_out, (size_t)T * d * 8, hipMemcpyDeviceToHost, c->stream));
  std::vector<double> pe(T);
  std::vector<int> ss(T);
  HIPCHK(c, hipMemcpyAsync(pe.data(), base + o_pe, (size_t)T * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(ss.data(), base + o_ss, (size_t)T * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  collect(c);
  if (proj_err) memcpy(proj_err, pe.data(), (size_t)T * 8);
  if (status) memcpy(status, ss.data(), (size_t)T * 4);
  return GPRX_OK;
}

gprx_batch* gprx_gp_batch(gprx_gp* gp) { return gp ? gp->batch : nullptr; }

// ---- host CState helpers -----------------------------------------------------------------------
int gprx_cstate_pack(int nb, const double* xc, const double* q, const double* vc, const double* wc, double* out) {
  if (nb < 1 || !xc || !q || !vc || !wc || !out) return GPRX_INVALID_ARGUMENT;
  for (int b = 0; b < nb; ++b) {
    double* o = out + 13 * b;
    for (int k = 0; k < 3; ++k) o[k] = xc[3 * b + k];
    for (int k = 0; k < 4; ++k) o[3 + k] = q[4 * b + k];
    for (int k = 0; k < 3; ++k) o[7 + k] = vc[3 * b + k];
    for (int k = 0; k < 3; ++k) o[10 + k] = wc[3 * b + k];
  }
  return GPRX_OK;
}

int gprx_select_outputs(const double* Xc, int d, int N, const int* idx1, int G, double* Y) {
  if (!Xc || !idx1 || !Y || d < 1 || N < 0 || G < 0) return GPRX_INVALID_ARGUMENT;
  for (int k = 0; k < G; ++k)
    if (idx1[k] < 1 || idx1[k] > d) return GPRX_INVALID_ARGUMENT;
  for (int k = 0; k < G; ++k)
    for (int t = 0; t < N; ++t) Y[(size_t)k * N + t] = Xc[(size_t)t * d + (idx1[k] - 1)];
  return GPRX_OK;
}

}  // extern "C"
