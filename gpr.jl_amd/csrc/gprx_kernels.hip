// gprx_kernels.hip -- CDNA4 (gfx950) kernels of the exact SE-ARD GP hot path, fp64.
//
// Algorithm (restating GaussianProcesses.jl v0.12.4 update_cK!/update_mll!/update_dmll!/predict_f
// as used by examples/maximal_coordinates/*noise.jl; see DESIGN.md for the kernel map):
//   K     = sf2 * exp(-r/2) + (sn2 + eps) I,  r_ij = sum_p il2_p * dist_p(x_i, x_j)     (gram)
//   K     = L L^T      left-looking tile Cholesky (update -> diag -> trsm per tile column)
//   L^-1  tile by tile, one sub-diagonal per launch                                  (trtri)
//   alpha = L^-T (L^-1 y)                                                            (alpha)
//   K^-1  = L^-T L^-1 tile by tile, fused with the gradient reduction of
//           W = alpha alpha^T - K^-1 against dK/dtheta (never written to HBM)        (lauum_grad)
//   mll, dmll                                                                        (finalize)
//   mu* = k*^T alpha,  var* = max(sf2 - |L^-1 k*|^2, 0)                             (pred_*)
//
// Every dense product is a 64x64 output tile per 256-thread workgroup, 4 waves of 32x32, built
// from v_mfma_f64_16x16x4_f64 with operands streamed straight from L2 (fp64 MFMA is 64 cycles per
// instruction per SIMD, so a 2x2 register tile per wave already keeps the pipe fed).
// Workgroup -> (slot, tile) mapping keeps every slot's tiles on one XCD (blocks b, b+8, ... share
// an XCD), so the panels all tiles of a slot re-read stay in that XCD's L2.
#include "gprx_internal.h"

namespace gprx {

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ d4 mfma(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// blockIdx -> (slot, tile); slots' tiles on one XCD when B % 8 == 0 (speed only, never correctness)
__device__ __forceinline__ void map_block(int bid, int B, int T, int& slot, int& tile) {
  if ((B & 7) == 0) {
    const int x = bid & 7, q = bid >> 3;
    slot = (q / T) * 8 + x;
    tile = q % T;
  } else {
    slot = bid / T;
    tile = bid % T;
  }
}

// t-th lower tile in column-major order -> (i, j), i >= j
__device__ __forceinline__ void lower_tile(int t, int nt, int& i, int& j) {
  int c = 0;
  while (t >= nt - c) {
    t -= nt - c;
    ++c;
  }
  j = c;
  i = c + t;
}

// Squared distance along one input dimension.
//  EXPANDED: Distances.jl 0.10.5 _pairwise!(r, SqEuclidean(), a, b) on the 1-row views that
//            GaussianProcesses' StationaryARD KernelData builds: max(a^2 + b^2 - 2(ab), 0).
//  DIRECT  : (a - b)^2.
// The file is compiled with -ffp-contract=off so these round exactly as written.
__device__ __forceinline__ double sqd(double a, double b, int mode) {
  if (mode == 0) {
    const double s = a * a + b * b;
    const double v = s - 2.0 * (a * b);
    return v > 0.0 ? v : 0.0;
  }
  const double t = a - b;
  return t * t;
}

__device__ __forceinline__ double readlane_d(double v, int lane) {
  const long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(u & 0xffffffffll), lane);
  const int hi = __builtin_amdgcn_readlane((int)(u >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Deterministic sum over the 256 threads of a workgroup; every thread gets the result.
__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  const double r = ((red[0] + red[1]) + red[2]) + red[3];
  __syncthreads();
  return r;
}

// ---------------------------------------------------------------------------------------------
// 32x32 wave tile:  acc[a][b] += A(32 x K) * B(32 x K)^T
//   A rows a0..a0+31 with element (r, k) at A[r + k*lda] (column-major; rows contiguous),
//   same for B.  The MFMA is issued with the operands swapped (A-op <- B rows, B-op <- A rows) so
//   that lane&15 indexes the output ROW: acc[a][b] lane l, reg q holds
//       C[16a + (l&15)][16b + (l>>4) + 4q]
//   (f64 16x16x4 C/D map: row = (lane>>4) + 4 reg, col = lane & 15; verified on gfx950), which
//   makes stores into column-major C contiguous over 16 lanes.
//   K must be a multiple of 16; operands are prefetched one 16-deep stage ahead into registers.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void mma_abt(d4 (&acc)[2][2], const double* __restrict__ A, size_t lda,
                                        const double* __restrict__ B, size_t ldb, int K) {
  if (K <= 0) return;
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const double* pa = A + lr + (size_t)lk * lda;
  const double* pb = B + lr + (size_t)lk * ldb;
  const size_t sa = 4 * lda, sb = 4 * ldb;
  double a0[4], a1[4], b0[4], b1[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    a0[s] = pa[s * sa];
    a1[s] = pa[s * sa + 16];
    b0[s] = pb[s * sb];
    b1[s] = pb[s * sb + 16];
  }
  const int nst = K >> 4;
  for (int it = 1; it < nst; ++it) {
    pa += 4 * sa;
    pb += 4 * sb;
    double na0[4], na1[4], nb0[4], nb1[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      na0[s] = pa[s * sa];
      na1[s] = pa[s * sa + 16];
      nb0[s] = pb[s * sb];
      nb1[s] = pb[s * sb + 16];
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      acc[0][0] = mfma(b0[s], a0[s], acc[0][0]);
      acc[0][1] = mfma(b1[s], a0[s], acc[0][1]);
      acc[1][0] = mfma(b0[s], a1[s], acc[1][0]);
      acc[1][1] = mfma(b1[s], a1[s], acc[1][1]);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      a0[s] = na0[s];
      a1[s] = na1[s];
      b0[s] = nb0[s];
      b1[s] = nb1[s];
    }
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    acc[0][0] = mfma(b0[s], a0[s], acc[0][0]);
    acc[0][1] = mfma(b1[s], a0[s], acc[0][1]);
    acc[1][0] = mfma(b0[s], a1[s], acc[1][0]);
    acc[1][1] = mfma(b1[s], a1[s], acc[1][1]);
  }
}

__device__ __forceinline__ void acc_zero(d4 (&acc)[2][2]) {
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = (d4){0.0, 0.0, 0.0, 0.0};
}

// C (column-major, ld) block of this wave  <-  scale * acc
__device__ __forceinline__ void acc_store(const d4 (&acc)[2][2], double* C, size_t ld, double scale) {
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) C[(size_t)(16 * b + lk + 4 * q) * ld + 16 * a + lr] = scale * acc[a][b][q];
}

// ============================================================================================
// Gram: lower tiles of K.  grid = B * ntl, 256 threads.
// ============================================================================================
__global__ __launch_bounds__(NTHR) void k_gram(DevBatch db) {
  __shared__ double xi[DMAX * TS], xj[DMAX * TS], pw[DMAX + 4];
  int slot, t, i, j;
  map_block(blockIdx.x, db.B, db.ntl, slot, t);
  lower_tile(t, db.nt, i, j);
  const int d = db.d, tid = threadIdx.x;
  const double* X = db.X + (size_t)slot * db.Npad * d;
  for (int e = tid; e < TS * d; e += NTHR) {
    const int r = e / d, p = e - r * d;
    xi[p * TS + r] = X[(size_t)i * TS * d + e];
    xj[p * TS + r] = X[(size_t)j * TS * d + e];
  }
  const double* P = db.params + (size_t)slot * db.pst;
  for (int e = tid; e < d + 3; e += NTHR) pw[e] = P[e];
  __syncthreads();
  const double sf2 = pw[d], noise = pw[d + 1];
  const int r = tid & 63, gi = i * TS + r, mode = db.dist_mode;
  double* K = db.K + (size_t)slot * db.mat;
#pragma unroll 2
  for (int q = 0; q < 16; ++q) {
    const int c = (tid >> 6) + 4 * q, gj = j * TS + c;
    double v;
    if (gi >= db.N || gj >= db.N) {
      v = (gi == gj) ? 1.0 : 0.0;
    } else {
      double rr = 0.0;
      for (int p = 0; p < d; ++p) rr = rr + sqd(xi[p * TS + r], xj[p * TS + c], mode) * pw[p];
      v = sf2 * exp(-rr * 0.5);
      if (gi == gj) v = v + noise;
    }
    K[(size_t)gj * db.ld + gi] = v;
  }
}

// ============================================================================================
// Left-looking Cholesky, tile column j.
//   update: K_ij -= sum_{k<j} L_ik L_jk^T  for i >= j           grid = B * (nt - j)
//   diag  : K_jj = L_jj L_jj^T (in registers), Dinv_j = L_jj^-1  grid = B
//   trsm  : L_ij = K_ij Dinv_j^T  for i > j                       grid = B * (nt - j - 1)
// ============================================================================================
__global__ __launch_bounds__(NTHR) void k_potrf_update(DevBatch db, int j) {
  int slot, t;
  map_block(blockIdx.x, db.B, db.nt - j, slot, t);
  const int i = j + t, w = threadIdx.x >> 6, wr = w >> 1, wc = w & 1;
  double* K = db.K + (size_t)slot * db.mat;
  const size_t ld = db.ld;
  d4 acc[2][2];
  acc_zero(acc);
  mma_abt(acc, K + i * TS + 32 * wr, ld, K + j * TS + 32 * wc, ld, j * TS);
  double* C = K + (size_t)(j * TS + 32 * wc) * ld + i * TS + 32 * wr;
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        double* pc = C + (size_t)(16 * b + lk + 4 * q) * ld + 16 * a + lr;
        *pc = *pc - acc[a][b][q];
      }
}

// Unblocked Cholesky of the 64x64 diagonal tile plus its triangular inverse.  Wave w owns
// columns 16w..16w+15 of the tile, lane = row; pivot columns are broadcast through LDS (one
// barrier per column, double-buffered).  Failure (pivot <= 0 or NaN, as LAPACK dpotrf) records
// status 1 and the 1-based global pivot index, and continues with pivot 1.
__global__ __launch_bounds__(NTHR) void k_potrf_diag(DevBatch db, int j) {
  __shared__ double colbuf[2][TS];
  __shared__ double Ls[TS * (TS + 1)];
  __shared__ double rowbuf[4][16];
  __shared__ double invd[TS];
  __shared__ double red[4];
  const int slot = blockIdx.x, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  double* K = db.K + (size_t)slot * db.mat;
  const size_t ld = db.ld;
  double* T = K + (size_t)j * TS * ld + j * TS;
  double a[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) a[q] = T[(size_t)(16 * w + q) * ld + lane];
  double logacc = 0.0;
  int fail_at = -1;
#pragma unroll
  for (int k = 0; k < TS; ++k) {
    const int wk = k >> 4, qk = k & 15;
    if (w == wk) {
      double dkk = readlane_d(a[qk], k);
      if (!(dkk > 0.0)) {
        if (fail_at < 0) fail_at = k;
        dkk = 1.0;
      }
      const double s = sqrt(dkk), inv = 1.0 / s;
      const double lv = (lane > k) ? a[qk] * inv : (lane == k ? s : 0.0);
      a[qk] = lv;
      colbuf[k & 1][lane] = (lane > k) ? lv : 0.0;
      if (lane == k) {
        logacc += log(s);
        invd[k] = inv;
      }
    }
    __syncthreads();
    const double lrk = colbuf[k & 1][lane];
#pragma unroll
    for (int q = 0; q < 16; ++q) a[q] = fma(-lrk, colbuf[k & 1][16 * w + q], a[q]);
  }
  // L_jj (upper triangle zero) back to K, and into LDS for the inverse
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    T[(size_t)(16 * w + q) * ld + lane] = a[q];
    Ls[(16 * w + q) * (TS + 1) + lane] = a[q];
  }
  // status: fail_at is wave-uniform inside the owning wave; the first failure across waves wins
  {
    const double lsum = wave_sum(logacc);
    __shared__ int fails[4];
    if (lane == 0) {
      red[w] = lsum;
      fails[w] = fail_at;
    }
    __syncthreads();
    if (tid == 0) {
      db.logdet_part[(size_t)slot * db.nt + j] = ((red[0] + red[1]) + red[2]) + red[3];
      int f = -1;
      for (int q = 0; q < 4; ++q)
        if (fails[q] >= 0 && (f < 0 || fails[q] < f)) f = fails[q];
      if (f >= 0 && db.status[slot] == 0) {
        db.status[slot] = 1;
        db.info[slot] = j * TS + f + 1;
      }
    }
  }
  // Dinv = L_jj^{-1}: wave w solves L X = I for columns 16w..16w+15, lane = row.
  double x[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) x[q] = (lane == 16 * w + q) ? 1.0 : 0.0;
  const int own = w;
#pragma unroll
  for (int k = 0; k < TS; ++k) {
    // row k of X for this wave's columns: lane k finalises and publishes it
    if (lane == k) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        x[q] = x[q] * invd[k];
        rowbuf[own][q] = x[q];
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const double lrk = (lane > k) ? Ls[k * (TS + 1) + lane] : 0.0;
#pragma unroll
    for (int q = 0; q < 16; ++q) x[q] = fma(-lrk, rowbuf[own][q], x[q]);
    __builtin_amdgcn_wave_barrier();
  }
  double* Li = db.Linv + (size_t)slot * db.mat + (size_t)j * TS * ld + j * TS;
#pragma unroll
  for (int q = 0; q < 16; ++q) Li[(size_t)(16 * w + q) * ld + lane] = x[q];
  // Mt_jj = Dinv^T through LDS
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 16; ++q) Ls[(16 * w + q) * (TS + 1) + lane] = x[q];  // Ls[c][r] = Dinv[r][c]
  __syncthreads();
  double* Mj = db.Mt + (size_t)slot * db.mat + (size_t)j * TS * ld + j * TS;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int c = 16 * w + q;  // Mt[r][c] = Dinv[c][r] = Ls[r][c]
    Mj[(size_t)c * ld + lane] = Ls[lane * (TS + 1) + c];
  }
}

__global__ __launch_bounds__(NTHR) void k_trsm(DevBatch db, int j) {
  int slot, t;
  map_block(blockIdx.x, db.B, db.nt - j - 1, slot, t);
  const int i = j + 1 + t, w = threadIdx.x >> 6, wr = w >> 1, wc = w & 1;
  double* K = db.K + (size_t)slot * db.mat;
  const double* Li = db.Linv + (size_t)slot * db.mat;
  const size_t ld = db.ld;
  d4 acc[2][2];
  acc_zero(acc);
  mma_abt(acc, K + (size_t)j * TS * ld + i * TS + 32 * wr, ld, Li + (size_t)j * TS * ld + j * TS + 32 * wc, ld, TS);
  __syncthreads();  // every wave has read its rows of K_ij before any wave overwrites them
  acc_store(acc, K + (size_t)(j * TS + 32 * wc) * ld + i * TS + 32 * wr, ld, 1.0);
}

// ============================================================================================
// Triangular inverse, sub-diagonal s:  for j, i = j + s
//   X         = sum_{k=j}^{i-1} L_ik Linv_kj      (B-operand rows from Mt = Linv^T)
//   Linv_ij   = -Dinv_i X,   Mt_ji = Linv_ij^T
// grid = B * (nt - s)
// ============================================================================================
constexpr int XS = 80;  // LDS row stride (doubles) of the X / Y staging tile
__global__ __launch_bounds__(NTHR) void k_trtri(DevBatch db, int s) {
  __shared__ double Xs[TS * XS];
  int slot, j;
  map_block(blockIdx.x, db.B, db.nt - s, slot, j);
  const int i = j + s, w = threadIdx.x >> 6, wr = w >> 1, wc = w & 1;
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const double* L = db.K + (size_t)slot * db.mat;
  double* Li = db.Linv + (size_t)slot * db.mat;
  double* Mt = db.Mt + (size_t)slot * db.mat;
  const size_t ld = db.ld;
  d4 acc[2][2];
  acc_zero(acc);
  mma_abt(acc, L + (size_t)j * TS * ld + i * TS + 32 * wr, ld, Mt + (size_t)j * TS * ld + j * TS + 32 * wc, ld, s * TS);
  // X -> LDS, row-major Xs[r][c]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) Xs[(32 * wr + 16 * a + lr) * XS + 32 * wc + 16 * b + lk + 4 * q] = acc[a][b][q];
  __syncthreads();
  // Y = Dinv_i X : A rows = Dinv_i (global, Linv_ii), B rows = X^T: Bm[c][t] = X[t][c] = Xs[t*XS + c]
  d4 acc2[2][2];
  acc_zero(acc2);
  mma_abt(acc2, Li + (size_t)i * TS * ld + i * TS + 32 * wr, ld, Xs + 32 * wc, XS, TS);
  acc_store(acc2, Li + (size_t)(j * TS + 32 * wc) * ld + i * TS + 32 * wr, ld, -1.0);
  __syncthreads();
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) Xs[(32 * wr + 16 * a + lr) * XS + 32 * wc + 16 * b + lk + 4 * q] = -acc2[a][b][q];
  __syncthreads();
  // Mt_ji[r'][c'] = Y[c'][r'] = Xs[c'*XS + r']
  double* Mji = Mt + (size_t)i * TS * ld + j * TS;
  const int rr = threadIdx.x & 63;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int c = (threadIdx.x >> 6) + 4 * q;
    Mji[(size_t)c * ld + rr] = Xs[c * XS + rr];
  }
}

// ============================================================================================
// alpha = L^-T (L^-1 y).  phase 0: z = Linv y ; phase 1: alpha = Mt z.   grid = B * nt
// ============================================================================================
__global__ __launch_bounds__(NTHR) void k_alpha(DevBatch db, int phase) {
  __shared__ double part[4][TS];
  int slot, i;
  map_block(blockIdx.x, db.B, db.nt, slot, i);
  const int r = threadIdx.x & 63, pt = threadIdx.x >> 6;
  const size_t ld = db.ld;
  const double* A = (phase == 0 ? db.Linv : db.Mt) + (size_t)slot * db.mat + i * TS + r;
  const double* v = (phase == 0 ? db.Y : db.z) + (size_t)slot * db.Npad;
  const int k0 = (phase == 0) ? 0 : i * TS, k1 = (phase == 0) ? (i + 1) * TS : db.Npad;
  double acc = 0.0;
  for (int k = k0 + pt; k < k1; k += 4) acc = fma(A[(size_t)k * ld], v[k], acc);
  part[pt][r] = acc;
  __syncthreads();
  if (pt == 0) {
    const double s = ((part[0][r] + part[1][r]) + part[2][r]) + part[3][r];
    (phase == 0 ? db.z : db.alpha)[(size_t)slot * db.Npad + i * TS + r] = s;
  }
}

// ============================================================================================
// K^-1 lower tile (i,j) = sum_{k>=i} Mt_ik Mt_jk^T, fused with the gradient partial sums
//   G_ij = wt_ij * (alpha_i alpha_j - Kinv_ij) * Kf_ij     (wt = 1/2 on the diagonal, as
//                                                          dmll_kern! weights ααinvcKI[j,j]/2)
//   S_p  = sum G_ij dist_p(x_i, x_j),  S_f = sum G_ij,  T = sum_diag W_ii
// grid = B * ntl
// ============================================================================================
constexpr int GS = 65;
__global__ __launch_bounds__(NTHR) void k_lauum_grad(DevBatch db) {
  __shared__ double xi[DMAX * TS], xj[DMAX * TS];
  __shared__ double g[TS * GS];
  __shared__ double ai[TS], aj[TS], pw[DMAX + 4], sp[DMAX], red[4];
  int slot, t, i, j;
  map_block(blockIdx.x, db.B, db.ntl, slot, t);
  lower_tile(t, db.nt, i, j);
  const int tid = threadIdx.x, w = tid >> 6, wr = w >> 1, wc = w & 1;
  const int l = tid & 63, lr = l & 15, lk = l >> 4;
  const int d = db.d, mode = db.dist_mode;
  const double* Mt = db.Mt + (size_t)slot * db.mat;
  const size_t ld = db.ld;
  d4 acc[2][2];
  acc_zero(acc);
  mma_abt(acc, Mt + (size_t)i * TS * ld + i * TS + 32 * wr, ld, Mt + (size_t)i * TS * ld + j * TS + 32 * wc, ld,
          (db.nt - i) * TS);
  const double* X = db.X + (size_t)slot * db.Npad * d;
  for (int e = tid; e < TS * d; e += NTHR) {
    const int r = e / d, p = e - r * d;
    xi[p * TS + r] = X[(size_t)i * TS * d + e];
    xj[p * TS + r] = X[(size_t)j * TS * d + e];
  }
  const double* P = db.params + (size_t)slot * db.pst;
  for (int e = tid; e < d + 3; e += NTHR) pw[e] = P[e];
  if (tid < TS) ai[tid] = db.alpha[(size_t)slot * db.Npad + i * TS + tid];
  else if (tid < 2 * TS) aj[tid - TS] = db.alpha[(size_t)slot * db.Npad + j * TS + tid - TS];
  __syncthreads();
  const double sf2 = pw[d];
  double sf = 0.0, tr = 0.0;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = 32 * wr + 16 * a + lr, c = 32 * wc + 16 * b + lk + 4 * q;
        const int gi = i * TS + r, gj = j * TS + c;
        double G = 0.0;
        if (gi < db.N && gj < db.N && gi >= gj) {
          double rr = 0.0;
          for (int p = 0; p < d; ++p) rr = rr + sqd(xi[p * TS + r], xj[p * TS + c], mode) * pw[p];
          const double kf = sf2 * exp(-rr * 0.5);
          const double W = ai[r] * aj[c] - acc[a][b][q];
          if (gi == gj) {
            G = 0.5 * (W * kf);
            tr += W;
          } else {
            G = W * kf;
          }
          sf += G;
        }
        g[c * GS + r] = G;
      }
  __syncthreads();
  // S_p: work item (p, r) -> one wave per p per pass, reduced over rows by the wave
  for (int e = tid; e < d * TS; e += NTHR) {
    const int p = e >> 6, r = e & 63;
    const double x0 = xi[p * TS + r];
    double s = 0.0;
    for (int c = 0; c < TS; ++c) s = fma(g[c * GS + r], sqd(x0, xj[p * TS + c], mode), s);
    s = wave_sum(s);
    if (r == 0) sp[p] = s;
  }
  const double sfa = block_sum(sf, red);
  const double tra = block_sum(tr, red);
  double* out = db.grad_part + ((size_t)slot * db.ntl + t) * db.gps;
  for (int e = tid; e < d; e += NTHR) out[e] = sp[e];
  if (tid == 0) {
    out[d] = sfa;
    out[d + 1] = tra;
  }
}

// ============================================================================================
// Per slot: mll = -(y.alpha + logdet + N log 2pi)/2 ; gradient (d+2) in GaussianProcesses order
// [log sn, log ell_1..d, log sf].  grid = B
// ============================================================================================
__global__ __launch_bounds__(NTHR) void k_finalize(DevBatch db, int want_grad) {
  __shared__ double red[4];
  const int slot = blockIdx.x, tid = threadIdx.x, d = db.d;
  const double* y = db.Y + (size_t)slot * db.Npad;
  const double* al = db.alpha + (size_t)slot * db.Npad;
  double s = 0.0;
  for (int k = tid; k < db.N; k += NTHR) s = fma(y[k], al[k], s);
  const double ya = block_sum(s, red);
  double* out = db.out + (size_t)slot * (d + 3);
  if (tid == 0) {
    double ld = 0.0;
    for (int k = 0; k < db.nt; ++k) ld += db.logdet_part[(size_t)slot * db.nt + k];
    const double log2pi = 1.8378770664093453;  // log(2pi), Julia's log2π
    out[0] = -((ya + 2.0 * ld) + log2pi * db.N) / 2.0;
  }
  if (want_grad) {
    const double* P = db.params + (size_t)slot * db.pst;
    const double* gp = db.grad_part + (size_t)slot * db.ntl * db.gps;
    for (int q = tid; q < d + 2; q += NTHR) {
      double tot = 0.0;
      for (int t = 0; t < db.ntl; ++t) tot += gp[(size_t)t * db.gps + q];
      if (q < d) out[2 + q] = P[q] * tot;           // d mll / d log ell_q = il2_q * S_q
      else if (q == d) out[2 + d] = 2.0 * tot;      // d mll / d log sf     = 2 S_f
      else out[1] = P[d + 2] * tot;                 // d mll / d log sn     = sn2 tr(W)
    }
  }
}

// ============================================================================================
// Prediction.
//   pred_cross: K*^T tile (64 test x 64 train) + partial means over the train tile.
//               grid = B * nt * mt
//   pred_var  : V = Linv K* row tile i, column sums of V^2 -> var_part.  grid = B * nt * mt
//   pred_final: mu = sum mu_part, var = max(sf2 - sum var_part, 0).       grid = B
// ============================================================================================
__global__ __launch_bounds__(NTHR) void k_pred_cross(DevBatch db) {
  __shared__ double xt[DMAX * TS], xs[DMAX * TS], pw[DMAX + 4], at[TS];
  __shared__ double part[4][TS];
  int slot, t;
  map_block(blockIdx.x, db.B, db.nt * db.mt, slot, t);
  const int ch = t / db.mt, mtile = t - ch * db.mt;
  const int tid = threadIdx.x, d = db.d, mode = db.dist_mode;
  const double* X = db.X + (size_t)slot * db.Npad * d;
  const double* Xq = db.Xs + (size_t)slot * db.Mpad * d;
  for (int e = tid; e < TS * d; e += NTHR) {
    const int r = e / d, p = e - r * d;
    xt[p * TS + r] = X[(size_t)ch * TS * d + e];
    xs[p * TS + r] = Xq[(size_t)mtile * TS * d + e];
  }
  const double* P = db.params + (size_t)slot * db.pst;
  for (int e = tid; e < d + 3; e += NTHR) pw[e] = P[e];
  if (tid < TS) at[tid] = db.alpha[(size_t)slot * db.Npad + ch * TS + tid];
  __syncthreads();
  const double sf2 = pw[d];
  const int m = tid & 63, pt = tid >> 6, gm = mtile * TS + m;
  double* KsT = db.KsT + (size_t)slot * db.Npad * db.Mpad;
  double macc = 0.0;
  for (int r = pt; r < TS; r += 4) {
    const int gt = ch * TS + r;
    double kv = 0.0;
    if (gt < db.N && gm < db.M) {
      double rr = 0.0;
      for (int p = 0; p < d; ++p) rr = rr + sqd(xt[p * TS + r], xs[p * TS + m], mode) * pw[p];
      kv = sf2 * exp(-rr * 0.5);
    }
    KsT[(size_t)gt * db.Mpad + gm] = kv;
    macc = fma(kv, at[r], macc);
  }
  part[pt][m] = macc;
  __syncthreads();
  if (pt == 0)
    db.mu_part[((size_t)slot * db.nt + ch) * db.Mpad + gm] = ((part[0][m] + part[1][m]) + part[2][m]) + part[3][m];
}

__global__ __launch_bounds__(NTHR) void k_pred_var(DevBatch db) {
  __shared__ double cs[2][2][32];
  int slot, t;
  map_block(blockIdx.x, db.B, db.nt * db.mt, slot, t);
  const int i = t / db.mt, mtile = t - i * db.mt;
  const int w = threadIdx.x >> 6, wr = w >> 1, wc = w & 1;
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const double* Li = db.Linv + (size_t)slot * db.mat;
  const double* KsT = db.KsT + (size_t)slot * db.Npad * db.Mpad;
  d4 acc[2][2];
  acc_zero(acc);
  mma_abt(acc, Li + i * TS + 32 * wr, db.ld, KsT + mtile * TS + 32 * wc, db.Mpad, (i + 1) * TS);
  // column sums of squares: sum over rows = over a, lr (16 lanes), wr (2 waves)
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      double v = acc[0][b][q] * acc[0][b][q] + acc[1][b][q] * acc[1][b][q];
      v += __shfl_xor(v, 1);
      v += __shfl_xor(v, 2);
      v += __shfl_xor(v, 4);
      v += __shfl_xor(v, 8);
      if (lr == 0) cs[wr][wc][16 * b + lk + 4 * q] = v;
    }
  __syncthreads();
  if (threadIdx.x < TS) {
    const int c = threadIdx.x, cw = c >> 5, cc = c & 31;
    db.var_part[((size_t)slot * db.nt + i) * db.Mpad + mtile * TS + c] = cs[0][cw][cc] + cs[1][cw][cc];
  }
}

__global__ __launch_bounds__(NTHR) void k_pred_final(DevBatch db) {
  const int slot = blockIdx.x;
  const double sf2 = db.params[(size_t)slot * db.pst + db.d];
  for (int m = threadIdx.x; m < db.Mpad; m += NTHR) {
    double mu = 0.0, s = 0.0;
    for (int k = 0; k < db.nt; ++k) {
      mu += db.mu_part[((size_t)slot * db.nt + k) * db.Mpad + m];
      s += db.var_part[((size_t)slot * db.nt + k) * db.Mpad + m];
    }
    const double v = sf2 - s;
    db.out_mu[(size_t)slot * db.Mpad + m] = mu;
    db.out_var[(size_t)slot * db.Mpad + m] = v > 0.0 ? v : 0.0;
  }
}

// ---------------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------------
void launch_gram(const DevBatch& b, hipStream_t s) {
  hipLaunchKernelGGL(k_gram, dim3(b.B * b.ntl), dim3(NTHR), 0, s, b);
}
void launch_potrf_update(const DevBatch& b, int j, hipStream_t s) {
  hipLaunchKernelGGL(k_potrf_update, dim3(b.B * (b.nt - j)), dim3(NTHR), 0, s, b, j);
}
void launch_potrf_diag(const DevBatch& b, int j, hipStream_t s) {
  hipLaunchKernelGGL(k_potrf_diag, dim3(b.B), dim3(NTHR), 0, s, b, j);
}
void launch_trsm(const DevBatch& b, int j, hipStream_t s) {
  hipLaunchKernelGGL(k_trsm, dim3(b.B * (b.nt - j - 1)), dim3(NTHR), 0, s, b, j);
}
void launch_trtri(const DevBatch& b, int sd, hipStream_t s) {
  hipLaunchKernelGGL(k_trtri, dim3(b.B * (b.nt - sd)), dim3(NTHR), 0, s, b, sd);
}
void launch_alpha(const DevBatch& b, hipStream_t s, int phase) {
  hipLaunchKernelGGL(k_alpha, dim3(b.B * b.nt), dim3(NTHR), 0, s, b, phase);
}
void launch_lauum_grad(const DevBatch& b, hipStream_t s) {
  hipLaunchKernelGGL(k_lauum_grad, dim3(b.B * b.ntl), dim3(NTHR), 0, s, b);
}
void launch_finalize(const DevBatch& b, int want_grad, hipStream_t s) {
  hipLaunchKernelGGL(k_finalize, dim3(b.B), dim3(NTHR), 0, s, b, want_grad);
}
void launch_pred_cross(const DevBatch& b, hipStream_t s) {
  hipLaunchKernelGGL(k_pred_cross, dim3(b.B * b.nt * b.mt), dim3(NTHR), 0, s, b);
}
void launch_pred_var(const DevBatch& b, hipStream_t s) {
  hipLaunchKernelGGL(k_pred_var, dim3(b.B * b.nt * b.mt), dim3(NTHR), 0, s, b);
}
void launch_pred_final(const DevBatch& b, hipStream_t s) {
  hipLaunchKernelGGL(k_pred_final, dim3(b.B), dim3(NTHR), 0, s, b);
}

}  // namespace gprx
