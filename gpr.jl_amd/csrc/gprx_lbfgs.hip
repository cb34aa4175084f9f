// gprx_lbfgs.hip -- device-side hyper-parameter optimiser.
//
// GaussianProcesses.optimize!(gp, LBFGS(linesearch=BackTracking(order=2)), Options(...)) as called
// by every experiment (examples/maximal_coordinates/CPnoise.jl:41), restated from Optim 1.4.1
// (LBFGS: m = 10, alphaguess InitialStatic(alpha = 1), scaleinvH0, twoloop!, update_h!,
// assess_convergence with g_abstol = 1e-8, x_abstol = f_abstol = 0, successive_f_tol = 1 and
// the non-finite-gradient break) and LineSearches 7.1.1
// (BackTracking order 2: c_1 = 1e-4, rho_hi = 0.5, rho_lo = 0.1, iterfinite from 0) -- [ext, not in
// the reference tree; Manifest.toml pins the versions].  The host restatement of the same
// algorithm is gpr.jl_amd/gprx/optim.py (lbfgs_steps / BackTracking.search); this kernel is its
// state machine, one thread per slot, so a whole batch's optimisers advance in lock-step between
// two evaluations of the batch without a host round trip for the parameters.
//
// Per round (host loop in gprx_api.hip, gprx_batch_optimize):
//   k_lbfgs(init=1)                          first requests -> params / status of every slot
//   repeat: evaluation graph (gram .. finalize, with gradient) ; k_lbfgs(init=0)
// k_lbfgs(init=0) reads each pending slot's answer (f = -mll, g = -grad; +Inf / NaN when the
// slot failed or its point is not finite), runs the slot's optimiser until it requests a point
// that is not its cached last evaluation (the accepted line-search point is always cached, since
// every evaluation carries the gradient), writes that point's kernel parameters exactly as
// gprx_batch_run derives them, and flags the slot active.  Finished slots keep their parameters.
#include <cfloat>

#include "gprx_internal.h"

namespace gprx {

enum LbPhase : int {
  PH_START = 0,
  PH_INIT_ANS,
  PH_ITER,
  PH_LS_FIRST,
  PH_LS_FIN,
  PH_LS_FIN_ANS,
  PH_LS_ARM,
  PH_LS_BT_ANS,
  PH_STEP,
  PH_STEP_ANS,
  PH_DONE
};
enum LbInt : int {  // per-slot int state (LB_NI entries)
  I_PH = 0, I_RESUME, I_PENDING, I_IT, I_PSEUDO, I_ITFIN, I_ITLS, I_FCALLS, I_GCALLS, I_STOP, I_CONV,
  I_LSOK, I_CVALID, I_FCNT
};
enum LbDbl : int {  // per-slot scalar state (LB_NS entries)
  D_FX = 0, D_FPREV, D_DPHI0, D_PHI0, D_A1, D_A2, D_PHIX0, D_PHIX1, D_ALPHA, D_LSPHI, D_CF
};

__device__ __forceinline__ double nanmin_(double a, double b) { return a != a ? b : (b != b ? a : fmin(a, b)); }
__device__ __forceinline__ double nanmax_(double a, double b) { return a != a ? b : (b != b ? a : fmax(a, b)); }
// numpy max(abs(v)): NaN if any element is NaN
__device__ __forceinline__ double maxabs_(const double* v, int n) {
  double m = 0.0;
  for (int i = 0; i < n; ++i) {
    const double a = fabs(v[i]);
    if (a != a) return a;
    m = a > m ? a : m;
  }
  return m;
}
__device__ __forceinline__ double dot_(const double* a, const double* b, int n) {
  double s = 0.0;
  for (int i = 0; i < n; ++i) s += a[i] * b[i];
  return s;
}

// Per-slot double workspace layout (n = d + 2 parameters, m history pairs)
struct LbView {
  double *x, *g, *s, *gp, *xr, *xp, *dx, *cx, *cg, *th0, *dxh, *dgh, *rho, *al, *sc;
  int* iv;
};
__device__ __forceinline__ LbView lb_view_at(int n, int m, double* w, int* iv) {
  LbView v;
  v.x = w; v.g = w + n; v.s = w + 2 * n; v.gp = w + 3 * n; v.xr = w + 4 * n; v.xp = w + 5 * n;
  v.dx = w + 6 * n; v.cx = w + 7 * n; v.cg = w + 8 * n; v.th0 = w + 9 * n;
  v.dxh = w + 10 * n; v.dgh = v.dxh + m * n; v.rho = v.dgh + m * n; v.al = v.rho + m; v.sc = v.al + m;
  v.iv = iv;
  return v;
}
__device__ __forceinline__ LbView lb_view(const LbArgs& a, int slot) {
  const int n = a.n, m = a.m;
  double* w = a.ws + (size_t)slot * lb_ws_doubles(n, m);
  LbView v;
  v.x = w; v.g = w + n; v.s = w + 2 * n; v.gp = w + 3 * n; v.xr = w + 4 * n; v.xp = w + 5 * n;
  v.dx = w + 6 * n; v.cx = w + 7 * n; v.cg = w + 8 * n; v.th0 = w + 9 * n;
  v.dxh = w + 10 * n; v.dgh = v.dxh + m * n; v.rho = v.dgh + m * n; v.al = v.rho + m; v.sc = v.al + m;
  v.iv = a.iws + (size_t)slot * LB_NI;
  return v;
}

// Optim's twoloop!: s = -H g from the history pairs of pseudo-iterations [pseudo - m, pseudo - 1]
__device__ void lb_twoloop(const LbView& v, int n, int m, int pseudo, int scaleinvH0) {
  double* q = v.s;
  for (int j = 0; j < n; ++j) q[j] = v.g[j];
  const int upper = pseudo - 1, lower = pseudo - m;
  for (int index = upper; index >= lower; --index) {
    if (index < 1) continue;
    const int i = (index - 1) % m;
    const double* dxi = v.dxh + (size_t)i * n;
    const double* dgi = v.dgh + (size_t)i * n;
    v.al[i] = v.rho[i] * dot_(dxi, q, n);
    for (int j = 0; j < n; ++j) q[j] -= v.al[i] * dgi[j];
  }
  if (scaleinvH0 && pseudo > 1) {
    const int i = (upper - 1) % m;
    const double* dxi = v.dxh + (size_t)i * n;
    const double* dgi = v.dgh + (size_t)i * n;
    const double sc = dot_(dxi, dgi, n) / dot_(dgi, dgi, n);
    for (int j = 0; j < n; ++j) q[j] = sc * q[j];
  }
  for (int index = lower; index <= upper; ++index) {
    if (index < 1) continue;
    const int i = (index - 1) % m;
    const double* dxi = v.dxh + (size_t)i * n;
    const double* dgi = v.dgh + (size_t)i * n;
    const double beta = v.rho[i] * dot_(dgi, q, n);
    for (int j = 0; j < n; ++j) q[j] += dxi[j] * (v.al[i] - beta);
  }
  for (int j = 0; j < n; ++j) q[j] = -q[j];
}

// the requested point becomes the slot's theta (a non-finite point evaluates the start point
// instead, as optimize_batch does: its answer is +Inf whatever the evaluation gives) and its
// kernel parameters follow by the same derive_params every evaluation uses
__device__ void lb_write_params(const LbArgs& a, const DevBatch& db, int slot, const double* th, const double* th0) {
  const int n = a.n;
  bool finite = true;
  for (int q = 0; q < n; ++q) finite = finite && isfinite(th[q]);
  double* T = db.theta + (size_t)slot * n;
  for (int q = 0; q < n; ++q) T[q] = finite ? th[q] : th0[q];
  derive_params(db, slot);
}

// One slot's optimiser between two evaluations (one thread; v: its state, in LDS or in HBM)
__device__ void lbfgs_slot(const LbArgs& a, const DevBatch& db, int slot, int init, const LbView& v) {
  const int n = a.n, m = a.m;
  int* I = v.iv;
  double* S = v.sc;
  if (init) {
    for (int j = 0; j < n; ++j) {
      v.x[j] = a.theta0[(size_t)slot * n + j];
      v.th0[j] = v.x[j];
    }
    for (int k = 0; k < LB_NI; ++k) I[k] = 0;
    for (int k = 0; k < LB_NS; ++k) S[k] = 0.0;
    S[D_FX] = __builtin_nan("");
    I[I_PH] = PH_START;
  } else if (I[I_PENDING]) {
    // answer of the slot's request from this round's evaluation (optimize_batch's cache entry)
    bool fin = true;
    for (int j = 0; j < n; ++j) fin = fin && isfinite(v.xr[j]);
    const double* o = db.out + (size_t)slot * (db.d + 3);
    const bool ok = fin && db.status[slot] == 0;
    for (int j = 0; j < n; ++j) {
      v.cx[j] = v.xr[j];
      v.cg[j] = ok ? -o[1 + j] : __builtin_nan("");
    }
    S[D_CF] = ok ? -o[0] : __builtin_inf();
    I[I_CVALID] = 1;
    I[I_PENDING] = 0;
    I[I_PH] = I[I_RESUME];
  }
  const double iterfinitemax = 52.0;  // -log2(eps(Float64))
  const bool capped = a.max_evals > 0;  // Optim: f_calls_limit > 0 && f_calls >= f_calls_limit
  // run until the slot needs an evaluation that is not its cached one, or finishes
  for (int guard = 0; guard < 4096; ++guard) {
    int ph = I[I_PH];
    if (ph == PH_DONE) break;
    bool want = false, want_g = false;  // request issued by this step: point in v.xr
    int resume = PH_DONE;
    switch (ph) {
      case PH_START:  // value_gradient!!: one f and one g call
        I[I_FCALLS] += 1;
        I[I_GCALLS] += 1;
        want = want_g = true;
        for (int j = 0; j < n; ++j) v.xr[j] = v.x[j];
        resume = PH_INIT_ANS;
        break;
      case PH_INIT_ANS: {
        S[D_FX] = S[D_CF];
        for (int j = 0; j < n; ++j) v.g[j] = v.cg[j];
        I[I_PSEUDO] = 0;
        I[I_CONV] = maxabs_(v.g, n) <= a.g_abstol;
        if (I[I_CONV]) {
          I[I_STOP] = LB_STOP_G_TOL;
          I[I_PH] = PH_DONE;
        } else {
          I[I_PH] = PH_ITER;
        }
        break;
      }
      case PH_ITER: {
        if (I[I_IT] >= a.iterations) {
          I[I_STOP] = LB_STOP_ITERATIONS;
          I[I_PH] = PH_DONE;
          break;
        }
        I[I_IT] += 1;
        I[I_PSEUDO] += 1;
        lb_twoloop(v, n, m, I[I_PSEUDO], a.scaleinvH0);
        for (int j = 0; j < n; ++j) v.gp[j] = v.g[j];
        double dphi0 = dot_(v.g, v.s, n);
        if (dphi0 >= 0.0) {  // reset_search_direction!
          I[I_PSEUDO] = 1;
          for (int j = 0; j < n; ++j) v.s[j] = -v.g[j];
          dphi0 = dot_(v.g, v.s, n);
        }
        S[D_DPHI0] = dphi0;
        S[D_A1] = S[D_A2] = a.alphaguess;
        S[D_PHI0] = S[D_FX];
        I[I_FCALLS] += 1;
        want = true;
        for (int j = 0; j < n; ++j) v.xr[j] = v.x[j] + S[D_A2] * v.s[j];
        resume = PH_LS_FIRST;
        break;
      }
      case PH_LS_FIRST:
        S[D_PHIX0] = S[D_PHI0];
        S[D_PHIX1] = S[D_CF];
        I[I_ITFIN] = 0;
        I[I_PH] = PH_LS_FIN;
        break;
      case PH_LS_FIN:
        if (!isfinite(S[D_PHIX1]) && I[I_ITFIN] < iterfinitemax) {
          I[I_ITFIN] += 1;
          S[D_A1] = S[D_A2];
          S[D_A2] = S[D_A1] / 2.0;
          I[I_FCALLS] += 1;
          want = true;
          for (int j = 0; j < n; ++j) v.xr[j] = v.x[j] + S[D_A2] * v.s[j];
          resume = PH_LS_FIN_ANS;
        } else {
          I[I_ITLS] = 0;
          I[I_PH] = PH_LS_ARM;
        }
        break;
      case PH_LS_FIN_ANS:
        S[D_PHIX1] = S[D_CF];
        I[I_PH] = PH_LS_FIN;
        break;
      case PH_LS_ARM: {
        const double a2 = S[D_A2], phi0 = S[D_PHI0], dphi0 = S[D_DPHI0], phix1 = S[D_PHIX1];
        if (phix1 > phi0 + a.c_1 * a2 * dphi0) {
          I[I_ITLS] += 1;
          if (I[I_ITLS] > a.ls_iterations) {  // LineSearchException(alpha_2)
            S[D_ALPHA] = a2;
            S[D_LSPHI] = phix1;
            I[I_LSOK] = 0;
            I[I_PH] = PH_STEP;
            break;
          }
          double atmp = -(dphi0 * (a2 * a2)) / (2.0 * (phix1 - phi0 - dphi0 * a2));  // dphi_0 * a2^2
          atmp = nanmin_(atmp, a2 * a.rho_hi);
          S[D_A1] = a2;
          S[D_A2] = nanmax_(atmp, a2 * a.rho_lo);
          I[I_FCALLS] += 1;
          want = true;
          for (int j = 0; j < n; ++j) v.xr[j] = v.x[j] + S[D_A2] * v.s[j];
          resume = PH_LS_BT_ANS;
        } else {
          S[D_ALPHA] = a2;
          I[I_LSOK] = 1;
          I[I_PH] = PH_STEP;
        }
        break;
      }
      case PH_LS_BT_ANS:
        S[D_PHIX0] = S[D_PHIX1];
        S[D_PHIX1] = S[D_CF];
        I[I_PH] = PH_LS_ARM;
        break;
      case PH_STEP: {
        const double alpha = S[D_ALPHA];
        for (int j = 0; j < n; ++j) {
          v.dx[j] = alpha * v.s[j];
          v.xp[j] = v.x[j];
          v.x[j] = v.x[j] + v.dx[j];
        }
        S[D_FPREV] = S[D_FX];
        if (!I[I_LSOK]) {  // update_state! reports the failed search: break before update_g!
          S[D_FX] = S[D_LSPHI];
          I[I_STOP] = LB_STOP_LINESEARCH;
          I[I_PH] = PH_DONE;
          break;
        }
        I[I_GCALLS] += 1;
        want = want_g = true;
        for (int j = 0; j < n; ++j) v.xr[j] = v.x[j];
        resume = PH_STEP_ANS;
        break;
      }
      case PH_STEP_ANS: {
        S[D_FX] = S[D_CF];
        for (int j = 0; j < n; ++j) v.g[j] = v.cg[j];
        // update_h!: dg = g - g_previous; rho = 1 / (dx . dg), pair stored unless rho is infinite
        double den = 0.0;
        for (int j = 0; j < n; ++j) den += v.dx[j] * (v.g[j] - v.gp[j]);
        const double r = 1.0 / den;
        if (!isinf(r)) {
          const int i = (I[I_PSEUDO] - 1) % m;
          for (int j = 0; j < n; ++j) {
            v.dxh[(size_t)i * n + j] = v.dx[j];
            v.dgh[(size_t)i * n + j] = v.g[j] - v.gp[j];
          }
          v.rho[i] = r;
        }
        double xch = 0.0;
        bool xnan = false;
        for (int j = 0; j < n; ++j) {
          const double e = fabs(v.x[j] - v.xp[j]);
          xnan = xnan || e != e;
          xch = e > xch ? e : xch;
        }
        // assess_convergence; an exact f repeat converges on successive_f_tol + 1 successive
        // iterations; then the time limit; then Optim's non-finite-gradient break
        const bool fconv = fabs(S[D_FX] - S[D_FPREV]) <= 0.0;
        I[I_FCNT] = fconv ? I[I_FCNT] + 1 : 0;
        bool gfin = true;
        for (int j = 0; j < n; ++j) gfin = gfin && isfinite(v.g[j]);
        if (maxabs_(v.g, n) <= a.g_abstol) I[I_STOP] = LB_STOP_G_TOL, I[I_CONV] = 1;
        else if (!xnan && xch <= 0.0) I[I_STOP] = LB_STOP_X_TOL, I[I_CONV] = 1;
        else if (I[I_FCNT] > a.successive_f_tol) I[I_STOP] = LB_STOP_F_TOL, I[I_CONV] = 1;
        if (I[I_CONV]) I[I_PH] = PH_DONE;
        else if (a.time_up) I[I_STOP] = LB_STOP_TIME_LIMIT, I[I_PH] = PH_DONE;
        else if (capped && I[I_FCALLS] >= a.max_evals) I[I_STOP] = LB_STOP_MAX_EVALS, I[I_PH] = PH_DONE;  // f_calls_limit
        else if (!gfin) I[I_STOP] = LB_STOP_NAN_GRADIENT, I[I_PH] = PH_DONE;
        else I[I_PH] = PH_ITER;
        break;
      }
      default:
        I[I_PH] = PH_DONE;
        break;
    }
    if (!want) continue;
    I[I_RESUME] = resume;
    bool hit = I[I_CVALID] != 0;
    for (int j = 0; j < n && hit; ++j) hit = v.cx[j] == v.xr[j];
    (void)want_g;  // every evaluation carries the gradient, so any cached point answers both kinds
    if (hit) {
      I[I_PH] = resume;
      continue;
    }
    I[I_PENDING] = 1;
    I[I_PH] = resume;
    lb_write_params(a, db, slot, v.xr, v.th0);
    break;
  }
  a.active[slot] = I[I_PENDING] || I[I_PH] != PH_DONE;  // (the guard can end a round unfinished)
  // results (read by the host once every slot is done)
  double* r = a.result + (size_t)slot * (n + 1);
  for (int j = 0; j < n; ++j) r[j] = v.x[j];
  r[n] = S[D_FX];
  int* ri = a.result_i + (size_t)slot * 4;
  ri[0] = I[I_IT];
  ri[1] = I[I_FCALLS];
  ri[2] = I[I_GCALLS];
  ri[3] = I[I_STOP] | (I[I_CONV] ? 0x100 : 0);
}

// One workgroup per slot: the slot's state (at most 74 KB: m = 64, d = DMAX) is copied into LDS
// by the whole wave, the state machine runs on lane 0 against LDS (its dependent loads no longer
// wait on L2), and the state is written back.
static_assert((size_t)(10 + 2 * 64) * (DMAX + 2) * 8 + (2 * 64 + LB_NS) * 8 + LB_NI * 4 <= (size_t)LB_LDS_MAX,
              "the largest optimiser state fits in LDS");
__global__ __launch_bounds__(64) void k_lbfgs(LbArgs a, DevBatch db, int init) {
  extern __shared__ __attribute__((aligned(16))) double lws[];
  const int slot = blockIdx.x, l = threadIdx.x;
  if (slot >= db.B) return;
  const size_t nws = lb_ws_doubles(a.n, a.m);
  double* gw = a.ws + (size_t)slot * nws;
  int* gi = a.iws + (size_t)slot * LB_NI;
  int* liv = (int*)(lws + nws);
  for (size_t i = l; i < nws; i += 64) lws[i] = gw[i];
  if (l < LB_NI) liv[l] = gi[l];
  __syncthreads();
  if (l == 0) lbfgs_slot(a, db, slot, init, lb_view_at(a.n, a.m, lws, liv));
  __syncthreads();
  for (size_t i = l; i < nws; i += 64) gw[i] = lws[i];
  if (l < LB_NI) gi[l] = liv[l];
}

// the minimiser's kernel parameters (Optim's result -> set_params!; update_target! follows).  The
// minimiser is written as it is: a non-finite one (the NaN-gradient stop of a non-PD start) makes
// derive_params mark the slot GPRX_INVALID_ARGUMENT, so the refit reports it instead of quietly
// factorising the start point.
__global__ __launch_bounds__(64) void k_lbfgs_final(LbArgs a, DevBatch db) {
  const int slot = blockIdx.x * 64 + threadIdx.x;
  if (slot >= db.B) return;
  LbView v = lb_view(a, slot);
  double* T = db.theta + (size_t)slot * a.n;
  for (int q = 0; q < a.n; ++q) T[q] = v.x[q];
  derive_params(db, slot);
}

size_t lbfgs_lds_bytes(int n, int m) { return lb_ws_doubles(n, m) * sizeof(double) + LB_NI * sizeof(int); }
// up to the CU's 160 KB (the default cap is 64 KB); once per device, from set_kernel_attributes
void set_lbfgs_attributes() {
  (void)hipFuncSetAttribute((const void*)k_lbfgs, hipFuncAttributeMaxDynamicSharedMemorySize, LB_LDS_MAX);
}
void launch_lbfgs(const LbArgs& a, const DevBatch& db, int init, hipStream_t s) {
  hipLaunchKernelGGL(k_lbfgs, dim3(db.B), dim3(64), lbfgs_lds_bytes(a.n, a.m), s, a, db, init);
}
void launch_lbfgs_final(const LbArgs& a, const DevBatch& db, hipStream_t s) {
  hipLaunchKernelGGL(k_lbfgs_final, dim3((db.B + 63) / 64), dim3(64), 0, s, a, db);
}

}  // namespace gprx
