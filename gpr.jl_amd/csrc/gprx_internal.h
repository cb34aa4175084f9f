// Internal declarations shared by the HIP kernels (gprx_kernels.hip) and the C-ABI host code
// (gprx_api.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <cfloat>
#include <stddef.h>
#include <stdint.h>

namespace gprx {

constexpr int TS = 64;     // tile edge (rows/cols) of every matrix block
constexpr int NTHR = 256;  // threads per workgroup (4 waves)
constexpr int DMAX = 64;   // largest input dimension d supported (FB: 52)

// Device-resident state of one batch of B GP slots with equal (d, N).  Passed to every kernel by
// value.  Matrices are column-major with leading dimension ld = Npad (Npad = ceil(N/64)*64).
//   K    : Gram matrix (lower tiles), reduced in place by the recursive Cholesky's SYRK updates.
//   Lw   : recursion workspace: L21 blocks (strictly lower tiles) and T^T = L11^-1 L21^T blocks
//          (strictly upper tiles).
//   Linv : L^{-1} (lower).      Mt : L^{-T} (upper) = Linv^T, so that every GEMM streams operands
//                                    along contiguous columns.
struct DevBatch {
  int B, d, N, Npad, nt, ntl;  // nt = Npad/64 tiles per edge, ntl = nt(nt+1)/2 lower tiles
  int M, Mpad, mt;             // test points (per slot), padded to 64, mt = Mpad/64
  int dist_mode;               // GPRX_DIST_EXPANDED / GPRX_DIST_DIRECT
  int want_var;                // predictive variance requested (var output non-NULL); 0 skips the
                               // O(N^2 M) variance GEMM (predictdynamics.jl uses the mean only)
  int small_n;                 // recursion nodes of <= small_n tiles use the 64 x 32 pair-unit GEMM
                               // (default, set_geometry in gprx_api.hip: 4 for B >= 32, all nodes
                               // below that, where the 64 x 64 units leave most of the chip idle);
                               // larger: 64 x 64 core
  int xs;                      // row stride of Xc: d | 1 (odd: spreads LDS banks)
  int pst;                     // stride of params per slot
  int gps;                     // stride of per-unit gradient partials (d + 2)
  int ngu;                     // gradient partial units per slot (lauum 4-tile units)
  int nlj;                     // lauum jobs per slot (units folded in pairs)
  int nimg;                    // largest number of point-tile images of a lauum unit (LDS size)
  size_t ld, mat;              // ld = Npad, mat = Npad*Npad
  double* X;                   // B x [Npad][d]   (column t = one CState, contiguous d values)
  double* Xc;                  // B x [Npad][xs]  X minus its per-dimension mean over the N points,
                               //                 dimensions d..xs-1 zero (theta-independent; the
                               //                 gradient's distance sums)
  double* Y;                   // B x Npad        (y - mean(X), zero padded)
  double* K;                   // B x mat: lower tiles of K as the Gram wrote them (kept: the gradient
                               //   reads its off-diagonal entries as Kf)
  double* S;                   // B x mat: lower tiles of the trailing matrices the SYRKs update
  double* Lw;                  // B x mat
  double* Linv;                // B x mat
  double* Mt;                  // B x mat
  double* z;                   // B x Npad        z = L^{-1} y
  double* zp;                  // B x 2nt x Npad  per-tile partials of z (see zp_acc4)
  double* alpha;               // B x Npad        alpha = K^{-1} y
  double* params;              // B x pst: [0,d) il2 = exp(-2 log ell), d: sf2, d+1: noise diag
                               //          (sn2 + eps), d+2: sn2
  double* theta;               // B x (d+2) hyper-parameters [log sn, log ell_1..d, log sf] of the
                               //          evaluation; params derive from it on the device
  double* logdet_part;         // B x nt          sum_r log L_rr per diagonal tile
  double* grad_part;           // B x ngu x gps   per lauum unit: S_p (d), S_f, trace(W)
  double* Xs;                  // B x [Mpad][d]   test points
  double* KsT;                 // B x [Npad][Mpad] K*^T (column-major M x N, ld = Mpad)
  double* mu_part;             // B x nt x Mpad
  double* var_part;            // B x nt x Mpad
  double* out;                 // B x (d+3): mll, grad[d+2]
  double* out_mu;              // B x Mpad
  double* out_var;             // B x Mpad
  int* status;                 // B
  int* info;                   // B
  int* lauum_order;            // nlj x 2 x LU: two units per job, long + short (lauum_plan)
  const int* active;           // B or null: evaluate only the slots with active[s] != 0 (the device
                               //   optimiser's rounds; null = every slot)
};

// GEMM operations of the recursive factorisation / inverse / prediction (tile units, see
// gprx_kernels.hip k_gemm):
enum GemmOp : int {
  OP_TRSM = 0,    // Lw[b2,b1]  = K[b2,b1] Linv[b1,b1]^T
  OP_SYRK = 1,    // K[b2,b2]  -= Lw[b2,b1] Lw[b2,b1]^T   (lower tiles)
  OP_TT = 2,      // Lw[b1,b2]  = Mt[b1,b1] Lw[b2,b1]^T   (= T^T, T = L21 L11^-1)
  OP_LINV21 = 3,  // Linv[b2,b1] = -Linv[b2,b2] T ; Mt[b1,b2] = Linv[b2,b1]^T
  OP_PREDVAR = 4  // var_part   = colsum((Linv K*)^2)
};
constexpr int OP_NONE = -1;
struct GemmGeom {
  int op;
  int o, h, n;  // node: offset o, split h, size n (tile units); block1 = [o, o+h), block2 = [o+h, o+n)
  int upd = 0;  // the node lies in an ancestor's trailing block: its tiles are read from S, not K
};
// Output rectangle of an op in tiles: origin (r0, c0), R x C, lower triangle only when tri.
__host__ __device__ inline void op_rect(const GemmGeom& g, int nt, int mt, int& r0, int& c0, int& R, int& C, bool& tri) {
  tri = false;
  switch (g.op) {
    case OP_TRSM:
    case OP_LINV21: r0 = g.o + g.h; c0 = g.o; R = g.n - g.h; C = g.h; break;
    case OP_SYRK: r0 = c0 = g.o + g.h; R = C = g.n - g.h; tri = true; break;
    case OP_TT: r0 = g.o; c0 = g.o + g.h; R = g.h; C = g.n - g.h; break;
    case OP_PREDVAR: r0 = 0; c0 = 0; R = nt; C = mt; break;
    default: r0 = c0 = R = C = 0; break;
  }
}

// Minimal-coordinate rollout (k_rollout): one GP of a rollout group, read from a batch slot after
// its factorisation (X: [Npad][d], alpha: Npad, params: il2[d], sf2, ...).
struct RolloutGP {
  const double* X;
  const double* alpha;
  const double* params;
  int N;
  int pad;
};
struct RolloutArgs {
  const RolloutGP* gps;  // ngroups x nc, GP g of a group predicts the rate of coordinate g
  const int* group;      // T: rollout group of each trajectory
  const double* start;   // T x 2nc: (q, qdot) per coordinate (predictdynamicsmin's startobservation)
  double* out;           // T x 2nc: (q_cur, qdot_last) per coordinate
  int T, nc, d, steps;
  int usesin, ang0, ang1;  // obs (sin q, cos q, qdot) for angle coordinates when usesin
  double dt;
};
constexpr int ROLLOUT_DMAX = 6;

// Maximal-coordinate physics of the rollout (gprx_projection.hip): the joint constraints of a
// mechanism as sub-joints (Revolute = T3 + R2, Prismatic = T2 + R3, Cylindrical = T2 + R2), rows of
// each written in the order of the reference's equality constraints.
constexpr int PJ_MAXB = 4;    // bodies (FB)
constexpr int PJ_MAXSUB = 12; // sub-joints
constexpr int PJ_MAXN = 56;   // 6 nb + constraint rows (FB: 24 + 24 = 48)
constexpr int PJ_MAXG = 16;   // GP outputs of one rollout group
struct SubJoint {
  int kind;       // 0 translational, 1 rotational
  int a, b;       // parent (0 = origin) and child body, 1-based
  int rows, row0; // constraint rows (2 or 3) and the first row among all constraint rows
  double pa[3], pb[3];
  double C[3][3]; // rows of the constraint matrix (I3, or the 2 rows normal to the axis)
};
struct MechDev {
  int nb, nd, nsub;  // bodies, constraint rows, sub-joints
  SubJoint sub[PJ_MAXSUB];
  double m[PJ_MAXB];        // body masses and inertia tensors (body frame; the variational
  double J[PJ_MAXB][3][3];  // integrator's dynamics, k_vi_step)
};
struct ProjArgs {
  MechDev mech;
  double dt, reg, eps;
  int iters;          // newtonIter
  int T;              // trajectories
  const double* cs;   // T x 13 nb CStates (the mechanism state: xc, qc, vc, wc per body)
  const double* vw;   // T x 6 nb predicted (v, w) per body (projectv!'s vu, wu)
  double* out;        // T x 6 nb projected (v, w)
  int* iters_out;     // T Newton iterations
  int* status;        // T: 0 ok, 1 singular KKT matrix (Julia's F \ f throws)
};
struct RolloutMaxArgs {
  MechDev mech;
  double dt, reg, eps;
  int iters, steps, T, G, d;
  int vw[PJ_MAXG];      // 0-based CState position of output g (getvw)
  const RolloutGP* gps; // ngroups x G
  const int* group;     // T
  const double* start;  // T x d
  double* out;          // T x d final CStates
  double* perr;         // T mean projection error per step
  int* status;          // T
};
// One variational-integrator step (ConstrainedDynamics 0.7.4 newton!, restated in gprx/vi.py) for T
// independent states: the MeanDynamics prior mean (src/mDynamics.jl:41-60).
struct ViArgs {
  MechDev mech;
  double dt, reg, eps, grav;
  int iters;          // newtonIter
  int T;
  const double* cs;   // T x 13 nb current CStates
  double* out;        // T x 13 nb solution CStates [x2, q2, v2, w2] per body (NaN row: failed)
  int* iters_out;     // T Newton iterations
  int* status;        // T: 0 converged, 1 not converged, 2 failed (non-finite / singular system)
};
void launch_project(const ProjArgs& a, hipStream_t s);
void launch_vi_step(const ViArgs& a, hipStream_t s);
void launch_rollout_max(const RolloutMaxArgs& a, int dist_mode, hipStream_t s);

// hyper-parameters -> kernel parameters for one slot, exactly as SEArd / GPE derive them:
//   il2 = exp(-2 log ell), sf2 = exp(2 log sf), noise = exp(2 logNoise) + eps();
// a non-finite theta is an ArgumentError (status GPRX_INVALID_ARGUMENT = 2, parameters 1).
// The one derivation every evaluation uses (k_params for gprx_batch_run, k_lbfgs for the device
// optimiser), so both see the same device exp().
__device__ inline void derive_params(const DevBatch& b, int slot) {
  const int d = b.d, np = d + 2;
  const double* th = b.theta + (size_t)slot * np;
  double* P = b.params + (size_t)slot * b.pst;
  bool finite = true;
  for (int q = 0; q < np; ++q) finite = finite && isfinite(th[q]);
  for (int p = 0; p < d; ++p) P[p] = finite ? exp(-2.0 * th[1 + p]) : 1.0;
  P[d] = finite ? exp(2.0 * th[d + 1]) : 1.0;
  const double sn2 = finite ? exp(2.0 * th[0]) : 1.0;
  P[d + 1] = sn2 + DBL_EPSILON;
  P[d + 2] = sn2;
  P[d + 3] = 0.0;
  b.status[slot] = finite ? 0 : 2;
  b.info[slot] = 0;
}

// Device LBFGS (gprx_lbfgs.hip): one optimiser state machine per slot, advanced between two
// evaluations of the batch.  n = d + 2 parameters in GaussianProcesses order, m history pairs.
constexpr int LB_NI = 16;  // ints of state per slot
constexpr int LB_NS = 16;  // scalar doubles of state per slot
__host__ __device__ inline size_t lb_ws_doubles(int n, int m) { return (size_t)(10 + 2 * m) * n + 2 * m + LB_NS; }
// stop reasons (GPRX_STOP_* in gprx.h); result_i[3] = reason | 0x100 when converged
enum LbStop : int {
  LB_STOP_ITERATIONS = 0, LB_STOP_G_TOL = 1, LB_STOP_X_TOL = 2, LB_STOP_F_TOL = 3, LB_STOP_LINESEARCH = 4,
  LB_STOP_MAX_EVALS = 5, LB_STOP_TIME_LIMIT = 6, LB_STOP_NAN_GRADIENT = 7
};
struct LbArgs {
  double* ws;            // B x lb_ws_doubles(n, m)
  int* iws;              // B x LB_NI
  const double* theta0;  // B x n
  int* active;           // B: slot requested an evaluation / is not finished
  double* result;        // B x (n + 1): x, f(x) = -mll
  int* result_i;         // B x 4: iterations, f calls, g calls, stop | converged
  int n, m, max_evals, iterations, ls_iterations, scaleinvH0, successive_f_tol, time_up;
  double g_abstol, alphaguess, c_1, rho_hi, rho_lo;
};
constexpr int LB_LDS_MAX = 160 * 1024;
size_t lbfgs_lds_bytes(int n, int m);

// kernel launchers (gprx_kernels.hip); every launcher is asynchronous on `s`
void set_kernel_attributes();  // once per device (gprx_ctx_create), before any launch
void set_lbfgs_attributes();   // gprx_lbfgs.hip, called by set_kernel_attributes
void launch_params(const DevBatch& b, hipStream_t s);
void launch_gram(const DevBatch& b, hipStream_t s);
void launch_center(const DevBatch& b, hipStream_t s);
void launch_diag(const DevBatch& b, int jt, int upd, hipStream_t s);
void launch_leaf(const DevBatch& b, int o, int n, int upd, hipStream_t s);
// the first half of an 8-tile node (top leaf, TRSM, SYRK + TT) in one launch (k_node8; B >= 32)
// four: the 4-wave form (k_node8h, two slots per CU; bit-identical results)
void launch_node8(const DevBatch& b, int o, int upd, hipStream_t s, bool four = false);  // a whole 8-tile node (k_node8)
// one launch; with g2.op != OP_NONE the units of g2 are appended to g's (independent ops)
void launch_gemm(const DevBatch& b, const GemmGeom& g, hipStream_t s, const GemmGeom& g2 = GemmGeom{OP_NONE, 0, 0, 0});
void launch_alpha(const DevBatch& b, hipStream_t s, int phase);
void launch_lauum_grad(const DevBatch& b, hipStream_t s);
// k_lauum_grad's job table: units of 4 output tiles, folded in pairs; LU ints per unit (see
// lauum_plan in gprx_kernels.hip).  Returns the jobs per slot; *nunits the units, *nimg the
// largest image count; out (nullable) receives jobs x 2 x LU ints.
constexpr int LU = 24;
int lauum_plan(int nt, int d, int* nunits, int* nimg, int* out);
void launch_finalize(const DevBatch& b, int want_grad, hipStream_t s);
void launch_pred_cross(const DevBatch& b, hipStream_t s);
void launch_pred_final(const DevBatch& b, hipStream_t s);
void launch_rollout(const RolloutArgs& a, int dist_mode, hipStream_t s);
void launch_lbfgs(const LbArgs& a, const DevBatch& db, int init, hipStream_t s);  // gprx_lbfgs.hip
void launch_lbfgs_final(const LbArgs& a, const DevBatch& db, hipStream_t s);

}  // namespace gprx
