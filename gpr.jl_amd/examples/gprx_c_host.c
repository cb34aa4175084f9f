/* gprx_c_host.c -- a plain C host over the C ABI (include/gprx.h), no Python and no HIP types:
 * what a Julia `ccall` shim or any other FFI does, written out in C.
 *
 *   gprx_c_host <trial.cst> <theta.f64> <xs.f64> <M>
 *
 * trial.cst: a GPRXCST1 file (gprx/dataset.py: X d x N column-major, Y rows); theta.f64: d+2
 * doubles [log sn, log ell_1..d, log sf]; xs.f64: d x M column-major test states.  Prints, as
 * "key v1 v2 ..." lines with %.17g:
 *   single GP on Y row 0 (GP / update_target_and_dtarget! / predict_f):  mll, grad, mu, var
 *   the G outputs of the trial as one batch (one gprx_batch_run):        batch_mll
 *   optimize! of every output on the device, f_calls_limit 15:             opt_min, opt_evals,
 *                                                                        opt_theta0 (slot 0)
 * Exit status 0 on success; on failure the gprx status string goes to stderr.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/gprx.h"

static double* read_f64(const char* path, size_t count) {
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  double* p = (double*)malloc(count * sizeof(double));
  size_t n = p ? fread(p, sizeof(double), count, f) : 0;
  fclose(f);
  if (n != count) {
    free(p);
    return NULL;
  }
  return p;
}

static void print_row(const char* key, const double* v, int n) {
  printf("%s", key);
  for (int i = 0; i < n; ++i) printf(" %.17g", v[i]);
  printf("\n");
}

static int fail(const char* what, int rc, gprx_ctx* ctx) {
  fprintf(stderr, "%s: %s (%s)\n", what, gprx_status_string(rc), ctx ? gprx_ctx_last_error(ctx) : "");
  return 1;
}

int main(int argc, char** argv) {
  if (argc != 5) {
    fprintf(stderr, "usage: %s trial.cst theta.f64 xs.f64 M\n", argv[0]);
    return 2;
  }
  if (gprx_abi_version() != GPRX_ABI_VERSION) {
    fprintf(stderr, "libgprx implements ABI version %d, this host was built against %d\n", gprx_abi_version(),
            GPRX_ABI_VERSION);
    return 2;
  }
  /* GPRXCST1 header: magic[8], u32 d, u32 G, u64 N, u64 reserved */
  FILE* f = fopen(argv[1], "rb");
  if (!f) return fail("open trial", GPRX_INVALID_ARGUMENT, NULL);
  char magic[8];
  uint32_t d32, G32;
  uint64_t N64, res;
  if (fread(magic, 1, 8, f) != 8 || memcmp(magic, "GPRXCST1", 8) != 0 || fread(&d32, 4, 1, f) != 1 ||
      fread(&G32, 4, 1, f) != 1 || fread(&N64, 8, 1, f) != 1 || fread(&res, 8, 1, f) != 1 || G32 < 1) {
    fclose(f);
    return fail("trial header", GPRX_INVALID_ARGUMENT, NULL);
  }
  const int d = (int)d32, G = (int)G32, N = (int)N64, M = atoi(argv[4]);
  double* X = (double*)malloc((size_t)d * N * sizeof(double));
  double* Y = (double*)malloc((size_t)G * N * sizeof(double));
  const int ok = X && Y && fread(X, sizeof(double), (size_t)d * N, f) == (size_t)d * N &&
                 fread(Y, sizeof(double), (size_t)G * N, f) == (size_t)G * N;
  fclose(f);
  double* theta = read_f64(argv[2], (size_t)d + 2);
  double* Xs = read_f64(argv[3], (size_t)d * M);
  if (!ok || !theta || !Xs || M < 1) return fail("inputs", GPRX_INVALID_ARGUMENT, NULL);

  gprx_ctx* ctx = NULL;
  int rc = gprx_ctx_create(0, &ctx);
  if (rc) return fail("gprx_ctx_create", rc, NULL);

  /* the GPE surface: GP(x, y, MeanZero(), SEArd(...)); optimize!'s evaluation; predict_f */
  gprx_gp* gp = NULL;
  rc = gprx_gp_create(ctx, X, d, N, Y, &gp);
  if (rc) return fail("gprx_gp_create", rc, ctx);
  double mll = 0.0;
  double* grad = (double*)malloc((size_t)(d + 2) * sizeof(double));
  double* mu = (double*)malloc((size_t)M * sizeof(double));
  double* var = (double*)malloc((size_t)M * sizeof(double));
  rc = gprx_gp_lml_grad(gp, theta, &mll, grad);
  if (rc) return fail("gprx_gp_lml_grad", rc, ctx);
  rc = gprx_gp_predict(gp, Xs, M, mu, var);
  if (rc) return fail("gprx_gp_predict", rc, ctx);
  print_row("mll", &mll, 1);
  print_row("grad", grad, d + 2);
  print_row("mu", mu, M);
  print_row("var", var, M);
  gprx_gp_destroy(gp);

  /* the trial's G outputs as one batch sharing X (CPnoise.jl:37-43 in one launch sequence) */
  gprx_batch* b = NULL;
  rc = gprx_batch_create(ctx, G, d, N, 0, &b);
  if (rc) return fail("gprx_batch_create", rc, ctx);
  rc = gprx_batch_set_train(b, X, 0, Y, N, GPRX_MEM_HOST);
  if (rc) return fail("gprx_batch_set_train", rc, ctx);
  double* th = (double*)malloc((size_t)G * (d + 2) * sizeof(double));
  double* bm = (double*)malloc((size_t)G * sizeof(double));
  for (int g = 0; g < G; ++g) memcpy(th + (size_t)g * (d + 2), theta, (size_t)(d + 2) * sizeof(double));
  rc = gprx_batch_run(b, th, 0u, bm, NULL, NULL, NULL, NULL, NULL);
  if (rc) return fail("gprx_batch_run", rc, ctx);
  print_row("batch_mll", bm, G);
  /* GaussianProcesses.optimize! (CPnoise.jl:41) for all G outputs in lock-step on the device */
  gprx_opt_options opt;
  gprx_opt_defaults(&opt);
  opt.max_evals = 15;
  double* thx = (double*)malloc((size_t)G * (d + 2) * sizeof(double));
  double* fmin = (double*)malloc((size_t)G * sizeof(double));
  int* fc = (int*)malloc((size_t)G * sizeof(int));
  int* gc = (int*)malloc((size_t)G * sizeof(int));
  double* ev = (double*)malloc((size_t)G * sizeof(double));
  int rounds = 0;
  rc = gprx_batch_optimize(b, th, &opt, thx, fmin, NULL, fc, gc, NULL, &rounds);
  if (rc) return fail("gprx_batch_optimize", rc, ctx);
  for (int g = 0; g < G; ++g) ev[g] = fc[g];  /* f calls = device evaluations (Optim f_calls_limit) */
  print_row("opt_min", fmin, G);
  print_row("opt_evals", ev, G);
  print_row("opt_theta0", thx, d + 2);
  free(thx);
  free(fmin);
  free(fc);
  free(gc);
  free(ev);
  gprx_batch_destroy(b);
  gprx_ctx_destroy(ctx);
  free(X);
  free(Y);
  free(theta);
  free(Xs);
  free(grad);
  free(mu);
  free(var);
  free(th);
  free(bm);
  return 0;
}
