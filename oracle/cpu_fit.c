/* ORACLE -- test infrastructure only (loaded by tests/ and by bench.py's cpu_baseline leg; never
 * by the product path).
 *
 * The CPU baseline BASELINE.md section 2 plans: the reference algorithm in C on the host's LAPACK,
 * one "fit"  = Gram + Cholesky + alpha + LML, the full gradient, and the
 * predictive mean and variance.  It follows oracle/gp_oracle.py statement for statement (direct
 * distances, the GaussianProcesses.jl v0.12.4 path restated there [ext]):
 *   KernelData's per-dimension distance stack D_p = (x_p,i - x_p,j)^2 (d x N x N, as the reference
 *   holds it), r = sum_p il2_p D_p in order p = 1..d, Kf = sf2 exp(-r/2), K = Kf + (sn2 + eps) I;
 *   cholesky!(Symmetric(K, :U)) -> dpotrf('U'); alpha = K \ y -> dpotrs; logdet = 2 sum log U_ii;
 *   K^-1 = ldiv!(chol, I) -> dpotrs on the identity (2N^3, as the reference);
 *   W = alpha alpha' - K^-1; dmll = [sn2 tr W, 1/2 sum W.Kf.D_p il2_p, 1/2 sum W.Kf 2];
 *   predict_f: k* = sf2 exp(-r(X, x*)/2), mu = k*' alpha, v = U' \ k*, var = max(sf2 - v'v, 0).
 * LAPACK/BLAS come from the host's OpenBLAS at run time (the scipy wheel's libscipy_openblas,
 * symbols scipy_*; path passed to cpufit_init), the library family Julia's cholesky! uses.
 * Parity against gp_oracle.py: tests/test_cpu_fit.py.
 * Build: oracle/Makefile (gcc -O3 -fopenmp, no -ffast-math: IEEE arithmetic as numpy's). */
#include <dlfcn.h>
#include <math.h>
#include <omp.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef void (*potrf_t)(const char*, const int*, double*, const int*, int*, size_t);
typedef void (*potrs_t)(const char*, const int*, const int*, const double*, const int*, double*, const int*, int*,
                        size_t);
typedef void (*trsm_t)(const char*, const char*, const char*, const char*, const int*, const int*, const double*,
                       const double*, const int*, double*, const int*, size_t, size_t, size_t, size_t);
typedef void (*nthreads_t)(int);
typedef int (*getthreads_t)(void);

static potrf_t dpotrf_;
static potrs_t dpotrs_;
static trsm_t dtrsm_;
static nthreads_t set_threads_;
static getthreads_t get_threads_;

#define LOG2PI 1.8378770664093453
#define EPS 2.220446049250313e-16

/* 0 on success */
int cpufit_init(const char* openblas_path) {
  void* h = dlopen(openblas_path, RTLD_NOW | RTLD_LOCAL);
  if (!h) return 1;
  dpotrf_ = (potrf_t)dlsym(h, "scipy_dpotrf_");
  dpotrs_ = (potrs_t)dlsym(h, "scipy_dpotrs_");
  dtrsm_ = (trsm_t)dlsym(h, "scipy_dtrsm_");
  set_threads_ = (nthreads_t)dlsym(h, "scipy_openblas_set_num_threads");
  get_threads_ = (getthreads_t)dlsym(h, "scipy_openblas_get_num_threads");
  return (dpotrf_ && dpotrs_ && dtrsm_ && set_threads_ && get_threads_) ? 0 : 2;
}

/* The library is the one scipy itself loaded: every call that changes its thread count restores
 * it, so numpy/scipy results elsewhere in the process are not perturbed. */
void cpufit_blas_threads(int n) { set_threads_(n); }
int cpufit_get_blas_threads(void) { return get_threads_(); }

/* per-fit workspace: the distance stack and four N x N matrices, reused across fits */
typedef struct {
  size_t cap;
  double* buf;
} Work;
static double* work_get(Work* w, size_t need) {
  if (need > w->cap) {
    free(w->buf);
    w->buf = malloc(sizeof(double) * need);
    w->cap = w->buf ? need : 0;
  }
  return w->buf;
}
static size_t work_need(int d, int N, int M) {
  const size_t NN = (size_t)N * N;
  return (size_t)d * NN + 3 * NN + (size_t)N + (size_t)d + (size_t)N * M;
}
static int fit_ws(int d, int N, int M, const double* X, const double* y, const double* theta, const double* Xs,
                  double* mll, double* grad, double* mu, double* var, double* ws);

/* One fit.  X: d x N (x_p of point j at X[p N + j]), y: N, theta: d + 2 ([log sn, log ell_1..d,
 * log sf]), Xs: d x M (may be NULL when M = 0).  Outputs: *mll, grad[d+2], mu[M], var[M].
 * Returns 0, or the dpotrf info (> 0: not positive definite), or -1 (allocation). */
int cpufit_fit(int d, int N, int M, const double* X, const double* y, const double* theta, const double* Xs,
               double* mll, double* grad, double* mu, double* var) {
  Work w = {0, NULL};
  double* ws = work_get(&w, work_need(d, N, M));
  const int rc = ws ? fit_ws(d, N, M, X, y, theta, Xs, mll, grad, mu, var, ws) : -1;
  free(w.buf);
  return rc;
}

static int fit_ws(int d, int N, int M, const double* X, const double* y, const double* theta, const double* Xs,
                  double* mll, double* grad, double* mu, double* var, double* ws) {
  const size_t NN = (size_t)N * N;
  double* D = ws;
  double* Kf = D + (size_t)d * NN;
  double* K = Kf + NN;
  double* Ki = K + NN;
  double* al = Ki + NN;
  double* il2 = al + N;
  double* Ks = M > 0 ? il2 + d : NULL;
  int rc = 0;
  for (int p = 0; p < d; ++p) il2[p] = exp(-2.0 * theta[1 + p]);
  const double sf2 = exp(2.0 * theta[d + 1]), sn2 = exp(2.0 * theta[0]), noise = sn2 + EPS;
  /* distance stack (the KernelData pairwise per dimension), then r in order p = 1..d */
  for (int p = 0; p < d; ++p) {
    const double* xp = X + (size_t)p * N;
    double* Dp = D + (size_t)p * NN;
    for (int i = 0; i < N; ++i)
      for (int j = 0; j < N; ++j) {
        const double t = xp[i] - xp[j];
        Dp[(size_t)i * N + j] = t * t;
      }
  }
  for (size_t e = 0; e < NN; ++e) {
    double r = 0.0;
    for (int p = 0; p < d; ++p) r = r + D[(size_t)p * NN + e] * il2[p];
    Kf[e] = sf2 * exp(-r * 0.5);
    K[e] = Kf[e];
  }
  for (int i = 0; i < N; ++i) K[(size_t)i * N + i] = K[(size_t)i * N + i] + noise;
  int info = 0, one = 1;
  dpotrf_("U", &N, K, &N, &info, 1);
  if (info != 0) {
    rc = info;
    goto done;
  }
  for (int i = 0; i < N; ++i)
    if (!isfinite(K[(size_t)i * N + i])) {
      rc = i + 1;
      goto done;
    }
  memcpy(al, y, sizeof(double) * N);
  dpotrs_("U", &N, &one, K, &N, al, &N, &info, 1);
  double ld = 0.0, ya = 0.0;
  for (int i = 0; i < N; ++i) ld += log(K[(size_t)i * N + i]);
  for (int i = 0; i < N; ++i) ya += y[i] * al[i];
  *mll = -(ya + 2.0 * ld + LOG2PI * N) / 2.0;
  /* K^-1 = ldiv!(chol, I) */
  memset(Ki, 0, sizeof(double) * NN);
  for (int i = 0; i < N; ++i) Ki[(size_t)i * N + i] = 1.0;
  dpotrs_("U", &N, &N, K, &N, Ki, &N, &info, 1);
  /* W o Kf in place of Ki (symmetric: row / column order agree), then the gradient sums */
  double trw = 0.0;
  for (int i = 0; i < N; ++i) trw += al[i] * al[i] - Ki[(size_t)i * N + i];
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < N; ++i) {
      const size_t e = (size_t)j * N + i;
      Ki[e] = (al[i] * al[j] - Ki[e]) * Kf[e];
    }
  grad[0] = sn2 * trw;
  for (int p = 0; p < d; ++p) {
    const double* Dp = D + (size_t)p * NN;
    double s = 0.0;
    for (size_t e = 0; e < NN; ++e) s += Ki[e] * Dp[e];
    grad[1 + p] = 0.5 * s * il2[p];
  }
  {
    double s = 0.0;
    for (size_t e = 0; e < NN; ++e) s += Ki[e];
    grad[d + 1] = 0.5 * s * 2.0;
  }
  if (M > 0) {  /* predict_f */
    for (int m = 0; m < M; ++m)
      for (int i = 0; i < N; ++i) {
        double r = 0.0;
        for (int p = 0; p < d; ++p) {
          const double t = X[(size_t)p * N + i] - Xs[(size_t)p * M + m];
          r = r + (t * t) * il2[p];
        }
        Ks[(size_t)m * N + i] = sf2 * exp(-r * 0.5);
      }
    for (int m = 0; m < M; ++m) {
      double s = 0.0;
      for (int i = 0; i < N; ++i) s += Ks[(size_t)m * N + i] * al[i];
      mu[m] = s;
    }
    const double a1 = 1.0;
    dtrsm_("L", "U", "T", "N", &N, &M, &a1, K, &N, Ks, &N, 1, 1, 1, 1);
    for (int m = 0; m < M; ++m) {
      double s = 0.0;
      for (int i = 0; i < N; ++i) s += Ks[(size_t)m * N + i] * Ks[(size_t)m * N + i];
      const double v = sf2 - s;
      var[m] = v > 0.0 ? v : 0.0;
    }
  }
done:
  return rc;
}

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

/* Timed sample: fits s = 0, 1, ... (slot s of the arrays, round robin over nslots) until
 * max_seconds, with `threads` OpenMP threads each running whole fits (BLAS single-threaded: the
 * trial-parallel mode) or, threads = 1, one fit at a time with BLAS on blas_threads cores (the
 * single-fit mode).  Returns the fits completed; *seconds the elapsed wall time. */
int cpufit_timed(int nslots, int d, int N, int M, const double* X, const double* Y, const double* T, const double* XS,
                 int threads, int blas_threads, double max_seconds, int max_fits, double* seconds) {
  const int saved = get_threads_();
  set_threads_(threads > 1 ? 1 : blas_threads);
  const double t0 = now_s();
  int done = 0;
  double* scratch = malloc(sizeof(double) * (size_t)(threads > 0 ? threads : 1) * (3 + d + 2 * M));
#pragma omp parallel num_threads(threads > 0 ? threads : 1)
  {
    double* o = scratch + (size_t)omp_get_thread_num() * (3 + d + 2 * M);
    Work w = {0, NULL};  /* this thread's workspace, allocated (and first touched) once */
    double* ws = work_get(&w, work_need(d, N, M));
    for (; ws;) {
      int k;
#pragma omp atomic capture
      k = done++;
      if (k >= max_fits || now_s() - t0 > max_seconds) break;
      const int s = k % nslots;
      fit_ws(d, N, M, X + (size_t)s * d * N, Y + (size_t)s * N, T + (size_t)s * (d + 2), XS ? XS + (size_t)s * d * M : NULL,
             o, o + 1, o + 3 + d, o + 3 + d + M, ws);
    }
    free(w.buf);
  }
  free(scratch);
  *seconds = now_s() - t0;
  set_threads_(saved);
  /* every thread's last claim past the deadline or budget was not a fit */
  const int claimed = done, nthr = threads > 0 ? threads : 1;
  return claimed - nthr < 0 ? 0 : (claimed - nthr > max_fits ? max_fits : claimed - nthr);
}
