/*
 * gprx.h -- C ABI of the MI355X-native exact-GP (SE-ARD, fp64) hot path for GPR.jl.
 *
 * Plain C: pointers, sizes, status codes.  No torch / HIP types cross this boundary.
 *
 * What each entry point replaces in the reference (amacati/GPR.jl, whose GP arithmetic is
 * delegated to GaussianProcesses.jl v0.12.4, pinned in /root/reference/Manifest.toml):
 *
 *   gprx_gp_create / gprx_batch_set_train
 *       GP(xtrain_old, yi, mean, kernel)            examples/maximal_coordinates/CPnoise.jl:40
 *       (X = reduce(hcat, CState.(traindf.sold)),   CPnoise.jl:26; y = yi - mean(X),
 *        mean from MeanZero or MeanDynamics         src/mDynamics.jl:41-55, theta-independent :29)
 *   gprx_gp_lml        update_mll! inside GP()/optimize! value evaluations   [ext] CPnoise.jl:40-41
 *   gprx_gp_lml_grad   update_mll! + update_dmll! (one LBFGS evaluation)     [ext] CPnoise.jl:41
 *   gprx_gp_predict    predict_f / predict_y(gp, x*)  examples/utils/predictdynamics.jl:13
 *   gprx_rollout_min   predictdynamicsmin             examples/utils/predictdynamics.jl:30-102
 *   gprx_batch_*       the G per-output GPs of a trial (CPnoise.jl:37-43) and the trial loop
 *                      (examples/parallel/core.jl:28) evaluated as one device batch
 *   gprx_cstate_pack   CState(::Vector{State})      src/CState.jl:25-28
 *   gprx_select_outputs  ytrain = [[s[i] for s in X_curr] for i in vwindices]   CPnoise.jl:28-29
 *
 * Hyper-parameter vector convention (GaussianProcesses get_params(gp) order, d+2 entries):
 *     theta = [ log sigma_n, log ell_1 ... log ell_d, log sigma_f ]
 * built by the callers as SEArd(log.(p[2:end]), log(p[1])) with default logNoise = -2.0
 * (CPnoise.jl:38-40).  Gradients are returned in the same order, with the same sign as
 * GaussianProcesses' gp.dmll (derivative of the log marginal likelihood, not of -mll).
 *
 * Memory: the caller owns every buffer it passes; the library copies on entry.  A batch owns
 * its device workspace (X, y, K/L, L^-1, L^-T, alpha, test points) until destroyed.
 * Threading: a context owns one HIP stream and a mutex; calls on one context serialise, calls on
 * different contexts (e.g. one per Julia thread / per GPU) run concurrently.  All calls block
 * until results are in host memory.
 */
#ifndef GPRX_H
#define GPRX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI versions:
 *   1  first release.
 *   2  gprx_opt_options.max_evals <= 0 means "no limit" (Optim's f_calls_limit = 0); under
 *      version 1, 0 was a real cap of zero evaluations.  No signature changed.
 *   3  gprx_batch_set_opt_trace takes the trace buffer's capacity; new gprx_batch_bytes and
 *      gprx_ctx_mem_info (device-batch chunking); gprx_batch_create / gprx_batch_set_test refuse
 *      sizes beyond the kernels' 32-bit buffer addressing (Npad * max(Npad, Mpad) * 8 >= 2^31 - 16). */
#define GPRX_ABI_VERSION 3

/* status codes (mirrors the reference's failure modes) */
#define GPRX_OK 0
#define GPRX_NOT_POSITIVE_DEFINITE 1 /* cholesky! -> PosDefException; Optim then sees +Inf   */
#define GPRX_INVALID_ARGUMENT 2      /* bad sizes, non-finite theta (ArgumentError)          */
#define GPRX_DEVICE_ERROR 3
#define GPRX_OUT_OF_MEMORY 4
#define GPRX_NOT_READY 5 /* predict before any successful factorisation */

/* gprx_batch_run flags */
#define GPRX_WANT_GRAD 1u    /* d mll / d theta (update_dmll!)                          */
#define GPRX_WANT_PREDICT 2u /* predictive mean + variance at the batch's test points    */

/* squared-distance formulation of the SE-ARD kernel (see DESIGN.md "distance modes") */
/* Per-dimension squared distance in the Gram / cross-covariance:
 *   DIRECT   (default): sum_d w_d (a_d - b_d)^2, as GaussianProcesses' cov_ij for StationaryARD
 *            kernels (distij over WeightedSqEuclidean) [ext]
 *   EXPANDED: a^2 + b^2 - 2ab clamped at 0 per dimension, the rounding of the Distances.jl 0.10.5
 *            pairwise(SqEuclidean()) stack that GaussianProcesses keeps for gradients [ext]       */
#define GPRX_DIST_EXPANDED 0
#define GPRX_DIST_DIRECT 1

/* memory kind of pointer arguments */
#define GPRX_MEM_HOST 0
#define GPRX_MEM_DEVICE 1

typedef struct gprx_ctx gprx_ctx;
typedef struct gprx_batch gprx_batch;
typedef struct gprx_gp gprx_gp;

int gprx_abi_version(void);
const char* gprx_status_string(int status);
/* first 16 hex digits of the SHA-256 of the sources the library was built from (the host checks
 * it against the sources it ships with, so a stale prebuilt library is refused)                 */
const char* gprx_build_id(void);
/* number of visible devices (hipGetDeviceCount; 0 when none or on error): hosts map their worker
 * threads / ranks onto devices with it (core.jl:28's threads, jobid mod ndevices)               */
int gprx_device_count(void);

/* ---- context: one device, one stream ------------------------------------------------------ */
int gprx_ctx_create(int device, gprx_ctx** out);
/* also destroys the context's remaining batches / GPs: their handles become invalid */
void gprx_ctx_destroy(gprx_ctx* ctx);
const char* gprx_ctx_last_error(const gprx_ctx* ctx);
int gprx_ctx_set_dist_mode(gprx_ctx* ctx, int mode);
int gprx_ctx_device(const gprx_ctx* ctx);
/* per-kernel timing (HIP events around every launch on the context stream); off by default */
int gprx_ctx_set_profiling(gprx_ctx* ctx, int enable);
/* launch-geometry options (results are identical under every setting; tests cover each path):
 *   GPRX_OPT_LEAF_TILES  recursion nodes of <= value tiles (64 x 64) run fused in one leaf
 *                        kernel; 1: every 64 x 64 diagonal tile on its own; 0 (default) = auto
 *   GPRX_OPT_SMALL_N     recursion nodes of <= value tiles use the 64 x 32 pair-unit GEMM; 0 = auto
 *   GPRX_OPT_GRAPHS      1: replay each evaluation's launch sequence as a hipGraph (default 0)
 *   GPRX_OPT_NODE_WAVES  the whole-8-tile-node kernel (batches >= 32 slots): 8 = one 8-wave
 *                        workgroup per slot (0, the default, is 8); 4 = a 4-wave workgroup per
 *                        slot, two slots per CU (measured slower on MI355X)          */
#define GPRX_OPT_LEAF_TILES 1
#define GPRX_OPT_SMALL_N 2
#define GPRX_OPT_GRAPHS 3
#define GPRX_OPT_NODE_WAVES 4
int gprx_ctx_set_option(gprx_ctx* ctx, int option, int value);
int gprx_ctx_kernel_stats(gprx_ctx* ctx, const char* kernel, double* total_ms, int64_t* launches,
                          double* algo_flops, double* algo_bytes);
int gprx_ctx_reset_stats(gprx_ctx* ctx);
/* free and total device memory of the context's device (hipMemGetInfo), for sizing batches      */
int gprx_ctx_mem_info(gprx_ctx* ctx, uint64_t* free_bytes, uint64_t* total_bytes);

/* ---- batch: B GP slots with equal (d, N); slot b has its own X_b, y_b, theta_b ------------ */
/* M_max: maximum number of test points per slot (0 = no prediction).  d <= 64, N >= 1, and
 * Npad * max(Npad, Mpad) * 8 < 2^31 - 16 (Npad, Mpad: N, M_max rounded up to 64; N <= 16320):
 * the kernels address a matrix panel with 32-bit byte offsets.  Larger sizes: GPRX_INVALID_ARGUMENT. */
int gprx_batch_create(gprx_ctx* ctx, int B, int d, int N, int M_max, gprx_batch** out);
/* Device bytes gprx_batch_create(B, d, N, M_max) allocates (host arithmetic only, no device call;
 * the optimiser's workspace, B * ((10 + 2m)(d+2) + 2m + 16) doubles, comes on top during
 * gprx_batch_optimize).  GPRX_INVALID_ARGUMENT for sizes gprx_batch_create refuses.  Hosts split
 * a rank's trials into device batches that fit the free memory with it (the reference's
 * parallelrun holds no such limit: core.jl:27-67 runs every trial in host RAM).                 */
int gprx_batch_bytes(int B, int d, int N, int M_max, uint64_t* bytes);
void gprx_batch_destroy(gprx_batch* batch);
/* X: d x N column-major per slot (column t = one CState), slot b at X + b*x_slot_stride
 *    (x_slot_stride = 0: all slots share one X, as the G outputs of one trial do);
 * Y: N targets per slot (y - mean(X)), slot b at Y + b*y_slot_stride.                          */
int gprx_batch_set_train(gprx_batch* batch, const double* X, int64_t x_slot_stride, const double* Y,
                         int64_t y_slot_stride, int mem);
/* Xs: d x M column-major per slot, slot b at Xs + b*xs_slot_stride (0 = shared), M <= M_max.   */
int gprx_batch_set_test(gprx_batch* batch, const double* Xs, int M, int64_t xs_slot_stride, int mem);
/* Evaluate every slot at theta[b*(d+2) ...]: Gram build, Cholesky, alpha, log marginal
 * likelihood; optionally its gradient and the predictive mean/variance (f-space: no noise, no
 * prior mean) at the test points.  var == NULL skips the O(N^2 M) variance computation (the
 * rollout pattern of predictdynamics.jl:13, which uses the mean only).  Outputs (host pointers,
 * any may be NULL):
 *   mll[B], grad[B*(d+2)], mu[B*M], var[B*M], status[B], info[B] (1-based failing pivot).
 * Returns GPRX_OK when every slot succeeded, otherwise the first failing slot's status.          */
int gprx_batch_run(gprx_batch* batch, const double* theta, unsigned flags, double* mll, double* grad,
                   double* mu, double* var, int* status, int* info);
/* Predictive mean/variance from the factorisation of the last gprx_batch_run (f-space);
 * var == NULL: mean only.                                                                      */
int gprx_batch_predict(gprx_batch* batch, double* mu, double* var);
int gprx_batch_dims(const gprx_batch* batch, int* B, int* d, int* N, int* M_max);
/* alpha = K^-1 (y - mean) of the last factorisation, alpha[b*N + t] (GPE's gp.alpha; N doubles
 * per slot), for hosts that keep GaussianProcesses' own fields current.  A slot whose status in
 * that evaluation was not GPRX_OK has no alpha: its N entries are NaN.                          */
int gprx_batch_alpha(gprx_batch* batch, double* alpha);

/* ---- hyper-parameter optimisation on the device ------------------------------------------- */
/* GaussianProcesses.optimize!(gp, LBFGS(linesearch=BackTracking(order=2)), Optim.Options(...))
 * (examples/maximal_coordinates/CPnoise.jl:41 and its 15 siblings) for every slot of a batch:
 * Optim 1.4.1 LBFGS + LineSearches 7.1.1 BackTracking restated as a device state machine, one
 * per slot, advanced in lock-step between evaluations of the whole batch (every evaluation
 * carries the gradient).  Minimises -mll over theta = [log sn, log ell_1..d, log sf]; a failed
 * evaluation (not positive definite, non-finite theta) counts as +Inf, as get_optim_target.   */
#define GPRX_STOP_ITERATIONS 0
#define GPRX_STOP_G_TOL 1
#define GPRX_STOP_X_TOL 2
#define GPRX_STOP_F_TOL 3
#define GPRX_STOP_LINESEARCH 4
#define GPRX_STOP_MAX_EVALS 5
#define GPRX_STOP_TIME_LIMIT 6
#define GPRX_STOP_NAN_GRADIENT 7 /* Optim: "Terminated early due to NaN in gradient"             */
#define GPRX_STOP_CONVERGED 0x100 /* or-ed into stopped[] when assess_convergence succeeded */
typedef struct gprx_opt_options {
  int m;              /* LBFGS history length (Optim: 10)                                        */
  int iterations;     /* Options.iterations (1000)                                               */
  int max_evals;      /* Options.f_calls_limit, the deterministic budget: a soft limit on f calls
                         (the initial evaluation + every line-search trial = the device evaluations),
                         checked after each iteration; <= 0: none (default;
                         Optim's f_calls_limit = 0)                        */
  int ls_iterations;  /* BackTracking.iterations (1000)                                          */
  int scaleinvH0;     /* LBFGS scaleinvH0 (true)                                                 */
  int refit;          /* 1: end with one evaluation of every slot at its minimiser, as optimize!
                         does (set_params! + update_target!); mll/predict then use it (default 1) */
  int successive_f_tol; /* Options.successive_f_tol (1): an exact f repeat converges only after
                           successive_f_tol + 1 successive iterations                          */
  double g_abstol;    /* Options.g_abstol (1e-8); x_abstol = f_abstol = 0 as Optim's defaults     */
  double time_limit;  /* seconds (the experiments use 10); NaN (default) or < 0: none.  Checked
                         between rounds: a slot stops after the iteration that sees it expired  */
  double alphaguess;  /* InitialStatic alpha (1.0)                                               */
  double c_1, rho_hi, rho_lo; /* BackTracking (1e-4, 0.5, 0.1)                                   */
} gprx_opt_options;
void gprx_opt_defaults(gprx_opt_options* opt);
/* theta0[B*(d+2)] start points; outputs (host, any may be NULL): theta_out[B*(d+2)] minimisers,
 * minimum[B] = -mll at the minimiser as Optim reports it, iterations/f_calls/g_calls[B],
 * stopped[B] = GPRX_STOP_* | GPRX_STOP_CONVERGED, rounds = batch evaluations performed
 * (excluding the refit; a round evaluates only the slots whose optimisers are still running, so a
 * ragged batch costs less per round as slots finish).  Returns GPRX_OK, or an error of the evaluations themselves
 * (device / memory); per-slot failures during the search are +Inf answers, not errors.  With
 * refit, a minimiser whose refit fails (not finite: GPRX_INVALID_ARGUMENT; not positive definite:
 * GPRX_NOT_POSITIVE_DEFINITE) is returned as that status (first failing slot), the outputs are
 * still filled, and the batch is left unfactorised (predict answers GPRX_NOT_READY).
 * time_limit is one wall clock for the whole call (all slots), not per GP as Optim's per-call
 * Options(time_limit=10.) at CPnoise.jl:41.  The context's mutex is held for the whole call:
 * other threads sharing the context wait until the optimisation ends.                         */
/* Outputs are written when the call returns GPRX_OK or a refit status after the search.  A call
 * rejected before the search (no training data, options out of range: GPRX_INVALID_ARGUMENT)
 * and a device / memory error write none of them.                                               */
int gprx_batch_optimize(gprx_batch* batch, const double* theta0, const gprx_opt_options* opt, double* theta_out,
                        double* minimum, int* iterations, int* f_calls, int* g_calls, int* stopped, int* rounds);
/* Diagnostics: record the optimiser's evaluations.  With a host buffer of max_rounds * B * (2(d+2)+2)
 * doubles registered, every later gprx_batch_optimize on this batch writes, for round r < max_rounds
 * and slot b, at trace[(r*B + b) * (2(d+2)+2)]: [active (1/0: evaluated in this round), theta(d+2)
 * as evaluated, mll, dmll(d+2) as answered]; rounds past the last are NaN.  capacity: the buffer's
 * size in doubles; smaller than max_rounds * B * (2(d+2)+2) is GPRX_INVALID_ARGUMENT (nothing is
 * registered).  The buffer must stay valid while registered; max_rounds = 0 unregisters it.  (No
 * reference counterpart: it makes the device optimiser's evaluation sequence comparable with a
 * host restatement's, gprx/optim.py.)                                                           */
int gprx_batch_set_opt_trace(gprx_batch* batch, double* trace, int max_rounds, int64_t capacity);

/* ---- single GP: the GPE surface, a batch of one ------------------------------------------- */
int gprx_gp_create(gprx_ctx* ctx, const double* X, int d, int N, const double* y_minus_mean,
                   gprx_gp** out);
void gprx_gp_destroy(gprx_gp* gp);
int gprx_gp_lml(gprx_gp* gp, const double* theta, double* mll);
int gprx_gp_lml_grad(gprx_gp* gp, const double* theta, double* mll, double* grad);
/* f-space predictive mean (k*^T alpha) and variance (max(k** - |L^-1 k*|^2, 0)) at the
 * factorisation of the last lml call; var may be NULL.                                          */
int gprx_gp_predict(gprx_gp* gp, const double* Xs, int M, double* mu_f, double* var_f);

/* the single GP's underlying batch of one (slot 0), e.g. for gprx_rollout_min              */
gprx_batch* gprx_gp_batch(gprx_gp* gp);

/* ---- rollout in minimal coordinates (examples/utils/predictdynamics.jl:30-102) ------------ */
#define GPRX_MECH_P1 1 /* pendulum:           q = theta                                  */
#define GPRX_MECH_P2 2 /* double pendulum:    q = (theta1, theta2 relative)              */
#define GPRX_MECH_CP 3 /* cart-pole:          q = (x, theta)                             */
#define GPRX_MECH_FB 4 /* four-bar:           q = (theta1, theta3)                       */
/* predictdynamicsmin for T trajectories in one launch.  A rollout group is the nc GPs of one
 * trial (nc = 1 for P1, else 2; GP g predicts the rate of coordinate g), given as
 * (batches[k], slots[k]) for k = group*nc + g, each factorised by its last gprx_batch_run with
 * MeanZero targets.  Trajectory t uses group traj_group[t] and starts at
 * start[t*2nc ...] = (q_1, qdot_1, ..., q_nc, qdot_nc); the GP input per step is
 * (q, qdot) per coordinate, or (sin q, cos q, qdot) for angles when usesin (input dimension
 * must match).  Each of the `steps` steps predicts the rates at the previous state and advances
 * q by rate*dt, exactly as the reference loop.  final_state[t*2nc ...] = (q_cur, qdot_last);
 * the reference's returned CState is built from q_cur with zero velocities (host side).        */
int gprx_rollout_min(gprx_ctx* ctx, int mech, int usesin, double dt, int steps, int ngroups,
                     gprx_batch* const* batches, const int* slots, int T, const int* traj_group,
                     const double* start, double* final_state);

/* ---- maximal-coordinate physics: projectv! and predictdynamics ----------------------------- */
/* projectv!(vu, wu, mechanism; newtonIter, eps, regularizer)  src/projections/implicitProjection.jl:80-107
 * for T independent mechanism states in one launch: state t is the mechanism's CState
 * cstates[t*13nb ...] (setstates!: positions, quaternions, velocities; the discrete pose follows as
 * x2 = x + v dt, q2 = q * wbar(w) dt/2), the prediction vw_pred[t*6nb ...] = (v_1, w_1, ..., v_nb,
 * w_nb).  Outputs vw_out (the projected twists; NaN for a failed state), iterations[t], status[t]
 * (0 ok, 1 singular KKT matrix: Julia's F \ f throws SingularException).  mech: GPRX_MECH_*, the
 * experiment mechanisms of examples/utils/data/simulations.jl (P1 pendulum, P2 double pendulum,
 * CP cart-pole, FB four-bar).  dt: mechanism.dt (0.01 in the experiments).                       */
int gprx_projectv(gprx_ctx* ctx, int mech, double dt, int T, const double* cstates, const double* vw_pred,
                  double regularizer, int newton_iter, double eps, double* vw_out, int* iterations, int* status);
/* One variational-integrator step, ConstrainedDynamics 0.7.4 newton!(mechanism) after
 * setstates!(mechanism, CState(x)) -- the prior mean of GPR's MeanDynamics (src/mDynamics.jl:41-60,
 * getmu = CState(mechanism, usesolution=true)) -- for T independent states in one launch, one wave
 * each.  cstates[t*13nb ...]: the current CState; out[t*13nb ...]: the solution CState [x2, q2, v2,
 * w2] per body (NaN row for a failed state).  status[t]: 0 converged (|f| < eps and |ds| < eps), 1
 * not converged within newton_iter iterations, 2 failed (a non-finite system, |w| beyond 2/dt: the
 * reference's DomainError; or a singular one: SingularException).  regularizer: the impulses'
 * regularisation (1e-10 for the four-bar's redundant loop constraints, 0 otherwise).  The host
 * restatement and its documentation: gpr.jl_amd/gprx/vi.py (vi_step).                          */
int gprx_vi_step(gprx_ctx* ctx, int mech, double dt, int T, const double* cstates, double regularizer,
                 int newton_iter, double eps, double* out, int* iterations, int* status);
/* predictdynamics(mechanism, gps, startobservation, steps, getvw; regularizer)
 * examples/utils/predictdynamics.jl:7-22 for T trajectories in one launch: per step the G GPs'
 * mean predictions at the current CState (predict_y(gp, obs)[1][1], MeanZero), getvw (output g
 * placed at 1-based CState position vw_idx1[g], a velocity or angular-velocity slot), projectv!
 * and updatestate!; one closing updatestate!.  GPs as for gprx_rollout_min: (batches[k],
 * slots[k]) for k = group*G + g, factorised, input dimension 13 nb.  Outputs final_state[t*13nb]
 * (the predicted CState), proj_err[t] (mean projection error per step), status[t] (0 ok, 1
 * singular projection).                                                                          */
int gprx_rollout_max(gprx_ctx* ctx, int mech, double dt, int steps, double regularizer, int ngroups,
                     gprx_batch* const* batches, const int* slots, int G, const int* vw_idx1, int T,
                     const int* traj_group, const double* start, double* final_state, double* proj_err,
                     int* status);

/* ---- host-side CState helpers (bit-exact copies) ------------------------------------------ */
/* out[13*b + 0..12] = [xc(3), qc.w, qc.x, qc.y, qc.z, vc(3), wc(3)] for body b (CState.jl:20,26) */
int gprx_cstate_pack(int nbodies, const double* xc, const double* qc_wxyz, const double* vc,
                     const double* wc, double* out);
/* Y[k*N + t] = Xcurr[t*d + (idx1[k]-1)]  (1-based indices, as vwindices in the experiments)     */
int gprx_select_outputs(const double* Xcurr, int d, int N, const int* idx1, int G, double* Y);

#ifdef __cplusplus
}
#endif
#endif /* GPRX_H */
