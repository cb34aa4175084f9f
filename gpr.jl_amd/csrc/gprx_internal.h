// Internal declarations shared by the HIP kernels (gprx_kernels.hip) and the C-ABI host code
// (gprx_api.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace gprx {

constexpr int TS = 64;     // tile edge (rows/cols) of every matrix block
constexpr int NTHR = 256;  // threads per workgroup (4 waves)
constexpr int DMAX = 64;   // largest input dimension d supported (FB: 52)

// Device-resident state of one batch of B GP slots with equal (d, N).  Passed to every kernel by
// value.  Matrices are column-major with leading dimension ld = Npad (Npad = ceil(N/64)*64).
//   K    : Gram matrix, overwritten in place by its lower Cholesky factor L (K = L L^T).
//   Linv : L^{-1} (lower).          Mt : L^{-T} (upper) = Linv^T, kept so that every GEMM reads
//                                        operands along contiguous columns.
struct DevBatch {
  int B, d, N, Npad, nt, ntl;  // nt = Npad/64 tiles per edge, ntl = nt(nt+1)/2 lower tiles
  int M, Mpad, mt;             // test points (per slot), padded to 64, mt = Mpad/64
  int dist_mode;               // GPRX_DIST_EXPANDED / GPRX_DIST_DIRECT
  int pst;                     // stride of params per slot
  int gps;                     // stride of per-tile gradient partials (d + 2)
  size_t ld, mat;              // ld = Npad, mat = Npad*Npad
  double* X;                   // B x [Npad][d]   (column t = one CState, contiguous d values)
  double* Y;                   // B x Npad        (y - mean(X), zero padded)
  double* K;                   // B x mat
  double* Linv;                // B x mat
  double* Mt;                  // B x mat
  double* z;                   // B x Npad        z = L^{-1} y
  double* alpha;               // B x Npad        alpha = K^{-1} y
  double* params;              // B x pst: [0,d) il2 = exp(-2 log ell), d: sf2, d+1: noise diag
                               //          (sn2 + eps), d+2: sn2
  double* logdet_part;         // B x nt          sum_r log L_rr per diagonal tile
  double* grad_part;           // B x ntl x gps   per lower tile: S_p (d), S_f, trace(W)
  double* Xs;                  // B x [Mpad][d]   test points
  double* KsT;                 // B x [Npad][Mpad] K*^T (column-major M x N, ld = Mpad)
  double* mu_part;             // B x nt x Mpad
  double* var_part;            // B x nt x Mpad
  double* out;                 // B x (d+3): mll, grad[d+2]
  double* out_mu;              // B x Mpad
  double* out_var;             // B x Mpad
  int* status;                 // B
  int* info;                   // B
};

// kernel launchers (gprx_kernels.hip); every launcher is asynchronous on `s`
void launch_gram(const DevBatch& b, hipStream_t s);
void launch_potrf_update(const DevBatch& b, int j, hipStream_t s);
void launch_potrf_diag(const DevBatch& b, int j, hipStream_t s);
void launch_trsm(const DevBatch& b, int j, hipStream_t s);
void launch_trtri(const DevBatch& b, int sdiag, hipStream_t s);
void launch_alpha(const DevBatch& b, hipStream_t s, int phase);
void launch_lauum_grad(const DevBatch& b, hipStream_t s);
void launch_finalize(const DevBatch& b, int want_grad, hipStream_t s);
void launch_pred_cross(const DevBatch& b, hipStream_t s);
void launch_pred_var(const DevBatch& b, hipStream_t s);
void launch_pred_final(const DevBatch& b, hipStream_t s);

}  // namespace gprx
