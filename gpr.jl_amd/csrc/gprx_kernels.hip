// gprx_kernels.hip -- CDNA4 (gfx950) kernels of the exact SE-ARD GP hot path, fp64.
//
// Algorithm (restating GaussianProcesses.jl v0.12.4 update_cK!/update_mll!/update_dmll!/predict_f
// as used by examples/maximal_coordinates/*noise.jl; see DESIGN.md for the kernel map):
//   K = sf2 * exp(-r/2) + (sn2 + eps) I,  r_ij = sum_p il2_p * dist_p(x_i, x_j)          (gram)
//   recursive Cholesky + triangular inverse on 64x64 tiles (host recursion, gprx_api.hip):
//     [A11 .; A21 A22]: rec(A11) -> L11, L11^-1 ; L21 = A21 L11^-T (TRSM) ;
//     A22 -= L21 L21^T (SYRK) ; rec(A22) ; T^T = L11^-T L21^T (TT) ; L21^-1 = -L22^-1 T (LINV21)
//     leaves: 64x64 Cholesky + inverse in one workgroup (diag)
//   alpha = L^-T (L^-1 y)                                                            (alpha)
//   K^-1  = L^-T L^-1 tile by tile, fused with the gradient reduction of
//           W = alpha alpha^T - K^-1 against dK/dtheta (K^-1 never written to HBM)   (lauum_grad)
//   mll, dmll                                                                        (finalize)
//   mu* = k*^T alpha,  var* = max(sf2 - |L^-1 k*|^2, 0)                             (pred_*)
//
// Dense products: one wave computes a 64x32 block with v_mfma_f64_16x16x4_f64 (4x2 16x16
// accumulators), operands streamed straight from L2 one 16-deep stage ahead (fp64 MFMA is 64
// cycles per instruction per SIMD; a 4x2 register tile needs 0.75 fragment loads per MFMA).  A
// workgroup = 4 waves = two vertically adjacent 64x64 tiles sharing their B panel.  Each wave has
// its own K range, so triangular operands are skipped at tile granularity.
// Workgroup -> (slot, unit) mapping keeps every slot's units on one XCD (blocks b, b+8, ... share
// an XCD), so the panels of a slot stay in that XCD's L2.
#include "gprx_internal.h"
#include <algorithm>
#include <array>
#include <cstdlib>
#include <vector>

namespace gprx {

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ d4 mfma(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// blockIdx -> (slot, unit).  With B >= 8, slot s runs on the blocks b with b % 8 == s % 8, i.e.
// on one XCD under the dispatcher's round-robin placement (speed only, never correctness), so
// its panels stay in one L2; the grid is padded to 8 * ceil(B/8) * T blocks and surplus blocks
// return at once.  With B < 8 that would leave XCDs idle, so a slot's units are spread over
// all of them (linear mapping).
__host__ __device__ inline int grid_blocks(int B, int T) { return B < 8 ? B * T : 8 * ((B + 7) / 8) * T; }
__device__ __forceinline__ bool map_block(int bid, int B, int T, int& slot, int& unit) {
  if (B < 8) {
    slot = bid / T;
    unit = bid - slot * T;
    return slot < B;
  }
  const int x = bid & 7, q = bid >> 3;
  slot = (q / T) * 8 + x;
  unit = q % T;
  return slot < B;
}

// ... and the slot's evaluation mask: db.active (optional, device) lets the optimiser's rounds skip
// the slots whose optimisers have finished (every workgroup of such a slot returns at once)
__device__ __forceinline__ bool slot_active(const DevBatch& db, int slot) { return !db.active || db.active[slot] != 0; }
__device__ __forceinline__ bool map_slot(const DevBatch& db, int T, int& slot, int& unit) {
  return map_block(blockIdx.x, db.B, T, slot, unit) && slot_active(db, slot);
}

// Units of a tile-pair decomposition.  rect R x C: pairs of rows per column; lower triangle of
// R x R: column c holds rows c..R-1.
__host__ __device__ inline int pair_units(int R, int C, bool tri) {
  if (!tri) return ((R + 1) / 2) * C;
  int u = 0;
  for (int c = 0; c < R; ++c) u += (R - c + 1) / 2;
  return u;
}
__device__ __forceinline__ void pair_unit(int u, int R, int C, bool tri, int& r, int& c) {
  if (!tri) {
    const int P = (R + 1) / 2;
    c = u / P;
    r = 2 * (u - c * P);
    return;
  }
  int cc = 0;
  while (u >= (R - cc + 1) / 2) {
    u -= (R - cc + 1) / 2;
    ++cc;
  }
  c = cc;
  r = cc + 2 * u;
}

// Squared distance along one input dimension.
//  EXPANDED: Distances.jl 0.10.5 _pairwise!(r, SqEuclidean(), a, b) on the 1-row views that
//            GaussianProcesses' StationaryARD KernelData builds: max(a^2 + b^2 - 2(ab), 0).
//            (s - 2t with t = fl(ab) equals fma(-2, t, s): 2t is exact.)
//  DIRECT  : (a - b)^2.
// The file is compiled with -ffp-contract=off so everything else rounds exactly as written.
__device__ __forceinline__ double sqd(double a, double b, int mode) {
  if (mode == 0) {
    const double t = a * b;
    const double v = fma(-2.0, t, a * a + b * b);
    return v > 0.0 ? v : 0.0;
  }
  const double t = a - b;
  return t * t;
}
// same with the squares precomputed
// r + d(a, b) w.  Expanded mode keeps the Distances.jl stack's rounding (d, then w d, then +; 6 fp64
// ops per element and dimension).  Direct mode is distij's s += (a-b)^2 w with the accumulation
// fused (3 ops): a rounding-level reordering, like the reference's own @simd sum.  (k_gram and
// k_pred_cross go one step further in direct mode: coordinates pre-scaled by 1/ell, 2 ops.)
__device__ __forceinline__ double sqd2(double a, double a2, double b, double b2, int mode);
template <int MODE>
__device__ __forceinline__ double wacc(double r, double a, double a2, double b, double b2, double w) {
  if (MODE == 0) return r + sqd2(a, a2, b, b2, 0) * w;
  const double t = a - b;
  return __builtin_fma(t * t, w, r);
}
__device__ __forceinline__ double sqd2(double a, double a2, double b, double b2, int mode) {
  if (mode == 0) {
    const double v = fma(-2.0, a * b, a2 + b2);
    return v > 0.0 ? v : 0.0;
  }
  const double t = a - b;
  return t * t;
}

// sqrt(p) and 1/sqrt(p) for p > 0 (normal range) by v_rsq_f64 + Newton: two steps on r = p^-1/2,
// then one Heron step on s = p r (about 1 ulp; no library call on the pivot chain)
__device__ __forceinline__ void sqrt_rsqrt(double p, double& s, double& r) {
  r = __builtin_amdgcn_rsq(p);
  r = r * fma(-0.5 * p * r, r, 1.5);
  r = r * fma(-0.5 * p * r, r, 1.5);
  s = p * r;
  s = fma(0.5 * r, fma(-s, s, p), s);
}
// sf2 exp(x) for x <= 0 (the Gram's K and the test cross-covariance): x = (64 m + j) ln2/64 + r
// with |r| <= ln2/128 + 2^-50 (Cody-Waite, r exact by fma), e^r = 1 + q with q a degree-5 Taylor
// polynomial (truncation |r|^6/720 < 4e-17 relative), sf2 2^(j/64) = hi_j + lo_j from a 64-entry
// table the kernel stages in static LDS (sf2 folded in at staging, the product's error by fma;
// the static address makes the lookup two instructions), result hi + (hi q + lo) scaled by 2^m;
// 0 below -745, NaN propagates.  n = rint(x 64/ln2) by the 1.5 2^52 shift: one fma and one add
// for a multiply, a rint and a conversion (the fused product can pick the other neighbour when
// x 64/ln2 lies within an ulp of a half-integer: |r| grows by 2^-50, the accuracy does not
// change).  About 0.51 ulp; the guard is a select, not a branch around the evaluation.
// The coefficients live in a mutable device array that a kernel copies into registers once
// (uniform loads: SGPRs): with literal constants the compiler rematerialises every coefficient
// per exp as two v_mov_b32.
struct ExpK {
  double c[4];         // 1/5!, 1/4!, 1/3!, 1/2
  double k64, hi, lo;  // 64/ln2; ln2/64 split, hi with 32 significant bits (n hi exact, |n| < 2^21)
};
__device__ ExpK g_expk = {{8.333333333333333e-03, 4.1666666666666664e-02, 0.16666666666666666, 0.5},
                          92.33248261689366, 0.01083042469326756, 2.9815858269852933e-12};
__device__ const double g_exp2tab[128] = {  // (hi_j, lo_j): 2^(j/64) = hi_j + lo_j, j = 0..63
    1.0, 0.0, 1.0108892860517005, -1.5234778603368577e-17,
    1.0218971486541166, 5.109225028973444e-17, 1.0330248790212284, 7.600838874027088e-18,
    1.0442737824274138, 8.551889705537965e-17, 1.0556451783605572, 1.759325738772092e-18,
    1.0671404006768237, -7.899853966841582e-17, 1.0787607977571199, -6.656660436056593e-17,
    1.0905077326652577, -3.046782079812471e-17, 1.102382583307841, 5.2660368715706944e-17,
    1.1143867425958924, 1.0410278456845571e-16, 1.1265216186082418, 5.165856758795457e-17,
    1.1387886347566916, 8.912812676025408e-17, 1.1511892299529827, 3.250710218863827e-17,
    1.1637248587775775, 3.8292048369240935e-17, 1.1763969916502812, 5.554203254218079e-17,
    1.189207115002721, 3.982015231465646e-17, 1.202156731452703, 6.644981499252301e-17,
    1.215247359980469, -7.712630692681488e-17, 1.22848053610687, -1.89878163130253e-17,
    1.241857812073484, 4.658027591836937e-17, 1.255380757024691, -6.7113898212968784e-18,
    1.2690509571917332, 2.667932131342186e-18, 1.2828700160787783, 1.713594918243561e-17,
    1.2968395546510096, 2.5382502794888315e-17, 1.3109612115247644, -7.181536135519454e-17,
    1.3252366431597413, -2.8587312100388614e-17, 1.339667524053303, 8.927282594831732e-17,
    1.3542555469368927, 7.70094837980299e-17, 1.3690024229745905, 9.593797919118849e-17,
    1.383909881963832, -6.770511658794786e-17, 1.3989796725383112, -9.614213209051323e-17,
    1.4142135623730951, -9.667293313452913e-17, 1.42961333839197, -1.2031642489053655e-17,
    1.4451808069770467, -3.0237581349939873e-17, 1.460917794180647, -5.600377186075216e-17,
    1.4768261459394993, -3.483994556892796e-17, 1.4929077282912648, 1.4192920154284036e-17,
    1.5091644275934228, -1.016455327754295e-16, 1.5255981507445384, -1.1024941712342561e-16,
    1.5422108254079407, 7.949834809697621e-17, 1.559004400237837, 3.7812070533575275e-17,
    1.5759808451078865, -1.0136916471278304e-17, 1.593142151342267, -1.0094406542311964e-16,
    1.6104903319492543, 2.4707192569797888e-17, 1.6280274218573478, -6.712955084707084e-17,
    1.645755478153965, -1.0125679913674773e-16, 1.6636765803267364, 5.8909926967131e-17,
    1.681792830507429, 8.199010020581497e-17, 1.7001063537185235, -8.0237193703977e-18,
    1.718619298122478, -1.851380418263111e-17, 1.7373338352737062, 3.164389299292957e-17,
    1.7562521603732995, 2.960140695448873e-17, 1.7753764925265212, 6.429731796556572e-17,
    1.7947090750031072, 1.8227458427912087e-17, 1.8142521755003989, -9.969531538920349e-17,
    1.8340080864093424, 3.283107224245627e-17, 1.8539791250833855, 9.761887490727594e-17,
    1.8741676341103, -6.122763413004143e-17, 1.8945759815869656, 3.4034035352165297e-17,
    1.9152065613971474, -1.0619946056195963e-16, 1.9360617934922943, 1.0332385960676326e-16,
    1.9571441241754002, 8.960767791036668e-17, 1.978456026387951, 4.0388753109278167e-17
};
__device__ __forceinline__ double exp_sf(double x, const ExpK& k, const double* tab0) {
  constexpr double SH = 6755399441055744.0;  // 1.5 2^52
  const double t = fma(x, k.k64, SH);
  const double n = t - SH;
  const int ni = (int)__double_as_longlong(t);
  double r = fma(-n, k.hi, x);
  r = fma(-n, k.lo, r);
  double q = k.c[0];
#pragma unroll
  for (int i = 1; i < 4; ++i) q = fma(q, r, k.c[i]);
  q = fma(q, r, 1.0) * r;  // e^r - 1
  const double2 tt = *(const double2*)((const char*)tab0 + ((ni << 4) & 0x3f0));  // entry ni & 63
  const double v = ldexp(tt.x + fma(tt.x, q, tt.y), ni >> 6);
  return x < -745.0 ? 0.0 : v;
}
// 1/p by v_rcp_f64 + two Newton steps (|error| <= 1 ulp; the reference's dpotf2 scales by 1/ajj too)
__device__ __forceinline__ double recip(double p) {
  double r = __builtin_amdgcn_rcp(p);
  r = fma(r, fma(-p, r, 1.0), r);
  r = fma(r, fma(-p, r, 1.0), r);
  return r;
}

__device__ __forceinline__ double readlane_d(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
// v from another lane of the same 16-lane row by a DPP control (two 32-bit DPP moves, no LDS)
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
// sum over the 16 lanes of each row, the same value in every lane of the row: quad pairs (quad_perm
// [1,0,3,2], [2,3,0,1]), then quad with quad (row_half_mirror), half-row with half-row (row_mirror)
__device__ __forceinline__ double row_sum16(double v) {
  v += dpp_f64<0xB1>(v);
  v += dpp_f64<0x4E>(v);
  v += dpp_f64<0x141>(v);
  v += dpp_f64<0x140>(v);
  return v;
}
// v + v(lane ^ 16) and v + v(lane ^ 32) by gfx950's lane-swap instructions (VALU, no LDS round
// trip as with ds_bpermute).  A swap of v with itself leaves v and its partner's value in every
// lane, in one order or the other, so the sum of the two results is v + partner exactly (addition
// commutes): the same values as v += __shfl_xor(v, 16 / 32) (scratch/permlane_check.hip).
__device__ __forceinline__ double sum_xor16(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)b, (unsigned)b, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
  return __builtin_bit_cast(double, ((long long)hi[0] << 32) | lo[0]) + __builtin_bit_cast(double, ((long long)hi[1] << 32) | lo[1]);
}
__device__ __forceinline__ double sum_xor32(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)b, (unsigned)b, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
  return __builtin_bit_cast(double, ((long long)hi[0] << 32) | lo[0]) + __builtin_bit_cast(double, ((long long)hi[1] << 32) | lo[1]);
}

// lane m of each row of 16 lanes, broadcast to the row (DPP row_newbcast, gfx90a+; m folds to a
// constant once the caller's loop is unrolled)
__device__ __forceinline__ double row_bcast16(double v, int m) {
  switch (m & 15) {
    case 0: return dpp_f64<0x150>(v);
    case 1: return dpp_f64<0x151>(v);
    case 2: return dpp_f64<0x152>(v);
    case 3: return dpp_f64<0x153>(v);
    case 4: return dpp_f64<0x154>(v);
    case 5: return dpp_f64<0x155>(v);
    case 6: return dpp_f64<0x156>(v);
    case 7: return dpp_f64<0x157>(v);
    case 8: return dpp_f64<0x158>(v);
    case 9: return dpp_f64<0x159>(v);
    case 10: return dpp_f64<0x15A>(v);
    case 11: return dpp_f64<0x15B>(v);
    case 12: return dpp_f64<0x15C>(v);
    case 13: return dpp_f64<0x15D>(v);
    case 14: return dpp_f64<0x15E>(v);
    default: return dpp_f64<0x15F>(v);
  }
}

// per-tile partials of z = L^-1 y (see zp_acc4)
__device__ __forceinline__ double* zp_row(const DevBatch& db, int slot, int h) {
  return db.zp + ((size_t)slot * 2 * db.nt + h) * db.Npad;
}
// a diagonal tile from an LDS image: row r of X at img[r * rs + c * cs].  The 256-thread
// workgroup splits the 64 columns in 4 quarters through the [256]-double scratch (no serial
// chain); call from every thread of the workgroup (contains barriers).
__device__ __forceinline__ void zp_diag(const DevBatch& db, int slot, int jt, const double* img, int rs, int cs,
                                        double* scr) {
  const double* y = db.Y + (size_t)slot * db.Npad + jt * TS;
  const int r = threadIdx.x & 63, qc = threadIdx.x >> 6;
  double t = 0.0;
#pragma unroll
  for (int c = 16 * qc; c < 16 * qc + 16; ++c) t = fma(img[r * rs + c * cs], y[c], t);  // X upper = 0
  __syncthreads();
  scr[qc * TS + r] = t;
  __syncthreads();
  if (qc == 0) {
    zp_row(db, slot, 2 * jt)[jt * TS + r] = ((scr[r] + scr[TS + r]) + scr[2 * TS + r]) + scr[3 * TS + r];
    zp_row(db, slot, 2 * jt + 1)[jt * TS + r] = 0.0;
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------------------------
// Wave GEMM core:  acc[a][b] += A(64 x K) * B(32 x K)^T
//   A rows r0..r0+63 with element (r, k) at A[r + k*lda] (column-major; rows contiguous); B rows
//   c0..c0+31 likewise.  The MFMA is issued with the operands swapped (A-op <- B rows, B-op <- A
//   rows) so that lane&15 indexes the output ROW: acc[a][b] lane l, reg q holds
//       C[16a + (l&15)][16b + (l>>4) + 4q]
//   (f64 16x16x4 C/D map: row = (lane>>4) + 4 reg, col = lane & 15; verified on gfx950), which
//   makes stores into column-major C contiguous over 16 lanes.
//   K is a multiple of 16; operands are prefetched one 16-deep stage ahead into registers.
// ---------------------------------------------------------------------------------------------
constexpr int WM = 4, WN = 2;
struct Frag {
  double a[4][WM], b[4][WN];
};
__device__ __forceinline__ void frag_load(Frag& f, const double* pa, const double* pb, size_t sa, size_t sb) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
#pragma unroll
    for (int a = 0; a < WM; ++a) f.a[s][a] = pa[s * sa + 16 * a];
#pragma unroll
    for (int b = 0; b < WN; ++b) f.b[s][b] = pb[s * sb + 16 * b];
  }
}
__device__ __forceinline__ void frag_mma(d4 (&acc)[WM][WN], const Frag& f) {
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int a = 0; a < WM; ++a)
#pragma unroll
      for (int b = 0; b < WN; ++b) acc[a][b] = mfma(f.b[s][b], f.a[s][a], acc[a][b]);
}
__device__ __forceinline__ void mma_64x32(d4 (&acc)[WM][WN], const double* __restrict__ A, size_t lda,
                                          const double* __restrict__ B, size_t ldb, int K) {
  // K is wave-uniform but derived from threadIdx.x >> 6; make that provable, otherwise hipcc
  // builds a divergent loop and moves all accumulator registers VGPR<->AGPR every stage.
  const int nst = __builtin_amdgcn_readfirstlane(K >> 4);
  if (nst <= 0) return;
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const double* pa = A + lr + (size_t)lk * lda;
  const double* pb = B + lr + (size_t)lk * ldb;
  const size_t sa = 4 * lda, sb = 4 * ldb;
  // two register stages in ping-pong: stage it+1 is in flight while stage it is multiplied.
  // K is a multiple of 64 (whole tiles), so nst is even; the last prefetch re-reads the last
  // stage (clamped index) instead of branching around the loads.
  Frag f0, f1;
  frag_load(f0, pa, pb, sa, sb);
  for (int it = 0; it < nst; it += 2) {
    frag_load(f1, pa + (size_t)(it + 1) * 4 * sa, pb + (size_t)(it + 1) * 4 * sb, sa, sb);
    frag_mma(acc, f0);
    const int n2 = (it + 2 < nst) ? it + 2 : nst - 1;
    frag_load(f0, pa + (size_t)n2 * 4 * sa, pb + (size_t)n2 * 4 * sb, sa, sb);
    frag_mma(acc, f1);
  }
}

// single register stage (no prefetch): latency is hidden by occupancy instead (4 waves/SIMD)
__device__ __forceinline__ void mma_64x32_s1(d4 (&acc)[WM][WN], const double* __restrict__ A, size_t lda,
                                             const double* __restrict__ B, size_t ldb, int K) {
  const int nst = __builtin_amdgcn_readfirstlane(K >> 4);
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const double* pa = A + lr + (size_t)lk * lda;
  const double* pb = B + lr + (size_t)lk * ldb;
  const size_t sa = 4 * lda, sb = 4 * ldb;
  for (int it = 0; it < nst; ++it) {
    Frag f;
    frag_load(f, pa + (size_t)it * 4 * sa, pb + (size_t)it * 4 * sb, sa, sb);
    frag_mma(acc, f);
  }
}

// ---------------------------------------------------------------------------------------------
// 64 x 64 wave core (k_gemm, k_lauum_grad): acc[a][b] += A(64 x K) B(64 x K)^T, same operand and
// C maps as mma_64x32 (acc[a][b] lane l reg q = C[16a + (l&15)][16b + (l>>4) + 4q]), 16 MFMAs
// per 8 fragment loads, two register stages of depth 8 (Q4SD = 2 MFMA sub-steps) in ping-pong,
// ~210 VGPRs: two waves per SIMD.  Scheduling barriers pin the two halves of an iteration (stage
// it+1's loads with stage it's MFMAs, stage it+2's loads with stage it+1's MFMAs): without them the
// compiler sinks the prefetch next to the other stage's loads and waits on vmcnt(0) before the
// first MFMA, serialising load and compute.  Inside a half, group barriers interleave one load per
// two MFMAs (round 2: every GEMM 2-3% faster than with the loads issued as one burst before the
// MFMAs, step 43.25 -> 42.7 ms at B=240, same-box A/B).  Measured on MI355X before the interleave
// (scratch/big_core_bench.hip, 192 batched 1024 x 1024 panels, 2 waves/SIMD): 70.9 / 68.5 / 64.2
// TF/s at K = 1024 / 512 / 256, against 64.5 / 67.4 / 63.0 for depth-16 stages without the
// barriers (and 60.2 / 57.4 / 52.7 for depth 16 with them: 25 spills).
// ---------------------------------------------------------------------------------------------
// Buffer resource over [base, base + bytes) (gfx9 word 3: raw, bounds-checked) and a 64-bit load
// at byte offset voff (VGPR) + soff (SGPR): out-of-range reads return 0.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buffer_rsrc(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
}
__device__ __forceinline__ double buffer_load_f64(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}
// 16-B store at byte offset voff (VGPR).  The SGPR offset field is left 0 on purpose: a MUBUF store
// with a register soffset is exempt from the compiler's store-data hazard check (no wait state
// before a VALU overwrites the data VGPRs), and on gfx950 under memory back-pressure (another
// process on the card) the store then read the NEXT exp's intermediate 1.5*2^52 + n as its data:
// K elements ~6.76e15, a non-PD pivot in a few evaluations in ten (scratch/concurrency.py).  With
// soffset 0 the hazard recognizer inserts the wait states.
// 8-B store at byte offset voff (VGPR) + soff (SGPR): 64-bit data, no store-data hazard (a VALU
// overwrite of >64-bit store data needs wait states the compiler skips for a register soffset;
// see buffer_store_f64x2)
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void buffer_store_f64(__amdgpu_buffer_rsrc_t r, int voff, int soff, double x) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, x), r, voff, soff, 0);
}
// -x by the sign bit (exact, as a multiply by -1; an integer VALU op)
__device__ __forceinline__ double neg_f64(double x) {
  return __builtin_bit_cast(double, __builtin_bit_cast(unsigned long long, x) ^ 0x8000000000000000ull);
}
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void buffer_store_f64x2(__amdgpu_buffer_rsrc_t r, int voff, double x, double y) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, make_double2(x, y)), r, voff, 0, 0);
}
constexpr int QM = 4, QN = 4, Q4SD = 2;
struct Frag4 {
  double a[Q4SD][QM], b[Q4SD][QN];
};
// NB < QN: only the first NB 16-column blocks of B (the prediction's last, partly padded test tile)
template <int NB = QN>
__device__ __forceinline__ void frag4_mma(d4 (&acc)[QM][QN], const Frag4& f) {
#pragma unroll
  for (int s = 0; s < Q4SD; ++s)
#pragma unroll
    for (int a = 0; a < QM; ++a)
#pragma unroll
      for (int b = 0; b < NB; ++b) acc[a][b] = mfma(f.b[s][b], f.a[s][a], acc[a][b]);
}
// mma_64x64 with triangular operand tiles and lower-only outputs skipped at 16 x 16-block
// granularity.  A 64-K tile of the K loop is 8 stages (k = 8s..8s+7), i.e. 4 loop trips of 2 stages.
//   TRI_A_FIRST  A's first K tile is upper triangular (explicit zeros below the diagonal): row block
//                a is zero for k < 16a, so trip t of that tile needs rows a <= t (lauum: A = Mt[ti, ti:];
//                TT: A = Mt[ti, ti:]).
//   TRI_AB_FIRST the same with B = A (a diagonal output tile of the lauum), and only the output blocks
//                b <= a are formed (the caller ignores the upper ones): trip t needs blocks a, b <= t.
//   LOWER_SAME   B = A (a diagonal SYRK tile): only the blocks b <= a, dense operands.
//   TRI_A_LAST   A's last K tile is lower triangular: row block a is zero for k > 16a + 15, so trip t
//                of that tile needs rows a >= t (LINV21: A = Linv[ti, :ti]).
//   TRI_B_LAST   the same for B's column blocks (TRSM: B = Linv[tj, :tj]).
// The peeled trips carry compile-time masks; skipped products are exact zeros, so the sums are
// bit-identical to the full core's.  Shared panels (B = A) load the fragments once.
enum CoreMode { PLAIN = 0, TRI_A_FIRST, TRI_AB_FIRST, LOWER_SAME, TRI_A_LAST, TRI_B_LAST, REV_A, REV_B };
// Operand addressing: element (row, k) at base[row + k ld]; lane (lr, lk) of sub-step s of stage st
// reads k = 8 st + 4 s + lk of rows 16 a + lr (a 16-row block reads 128 contiguous bytes).  Round 5:
// buffer loads, the lane's byte offset in a VGPR (fixed), the stage and sub-step offsets in SGPRs
// and the row block in the instruction's offset field, so the K loop has no VALU address
// arithmetic (64-bit global addresses needed a v_lshl_add_u64 per address per stage, and every
// VALU instruction takes issue cycles from the other wave's MFMAs on gfx950: the core pattern on an
// L2-resident panel ran at 76.4 TF/s with global loads and 77.6 with buffer loads,
// scratch/mfma_pattern.hip, profiles/r05_mfma_valu_pattern.txt).
struct CorePtr {
  __amdgpu_buffer_rsrc_t r;  // over the operand from its tile origin
  int vo;                    // this lane's byte offset: row lr, column lk
  int o;                     // byte offset of stage 0, sub-step 0 (wave-uniform)
  int st, sub;               // stage / sub-step strides in bytes (negative: a backward walk)
};
__device__ __forceinline__ CorePtr core_ptr(const double* X, size_t ld) {
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const int L = (int)ld * (int)sizeof(double);
  return CorePtr{buffer_rsrc(X, 0x7ffffff0), lr * (int)sizeof(double) + lk * L, 0, 8 * L, 4 * L};
}
__device__ __forceinline__ CorePtr core_rev(CorePtr c, int nst) {  // stages and sub-steps backward
  c.o += (nst - 1) * c.st + c.sub;
  c.st = -c.st;
  c.sub = -c.sub;
  return c;
}
// The same walk through 64-bit global addresses (the round-4 form): k_node8 keeps it, since its
// GEMM phases sit beside the fused leaf's state and the buffer form's SGPR resources pushed that
// kernel from 8 to 58 spilled VGPRs.
struct CorePtrG {
  const double* p;  // this lane's address of stage 0, sub-step 0, row block 0
  ptrdiff_t st;     // stage stride
  ptrdiff_t sub;    // sub-step stride
};
__device__ __forceinline__ CorePtrG core_ptr_g(const double* X, size_t ld) {
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const ptrdiff_t L = (ptrdiff_t)ld;
  return CorePtrG{X + lr + lk * L, 8 * L, 4 * L};
}
__device__ __forceinline__ CorePtrG core_rev(CorePtrG c, int nst) {
  c.p += (ptrdiff_t)(nst - 1) * c.st + c.sub;
  c.st = -c.st;
  c.sub = -c.sub;
  return c;
}
template <int A0, int A1, int B0, int B1, bool SAME>
__device__ __forceinline__ void frag4_load_r(Frag4& f, const CorePtrG& A, const CorePtrG& B, int st) {
  constexpr int L0 = SAME ? (A0 < B0 ? A0 : B0) : A0, L1 = SAME ? (A1 > B1 ? A1 : B1) : A1;
  const double* pa = A.p + (ptrdiff_t)st * A.st;
  const double* pb = B.p + (ptrdiff_t)st * B.st;
#pragma unroll
  for (int s = 0; s < Q4SD; ++s) {
#pragma unroll
    for (int a = L0; a < L1; ++a) f.a[s][a] = pa[s * A.sub + 16 * a];
    if constexpr (!SAME) {
#pragma unroll
      for (int b = B0; b < B1; ++b) f.b[s][b] = pb[s * B.sub + 16 * b];
    }
  }
}
template <bool BUF>
__device__ __forceinline__ auto core_addr(const double* X, size_t ld) {
  if constexpr (BUF) return core_ptr(X, ld);
  else return core_ptr_g(X, ld);
}
template <int A0, int A1, int B0, int B1, bool SAME>
__device__ __forceinline__ void frag4_load_r(Frag4& f, const CorePtr& A, const CorePtr& B, int st) {
  constexpr int L0 = SAME ? (A0 < B0 ? A0 : B0) : A0, L1 = SAME ? (A1 > B1 ? A1 : B1) : A1;
  const int oa = A.o + st * A.st, ob = B.o + st * B.st;
#pragma unroll
  for (int s = 0; s < Q4SD; ++s) {
#pragma unroll
    for (int a = L0; a < L1; ++a) f.a[s][a] = buffer_load_f64(A.r, A.vo + 128 * a, oa + s * A.sub);
    if constexpr (!SAME) {
#pragma unroll
      for (int b = B0; b < B1; ++b) f.b[s][b] = buffer_load_f64(B.r, B.vo + 128 * b, ob + s * B.sub);
    }
  }
}
template <int A0, int A1, int B0, int B1, bool SAME, bool LOWER>
__device__ __forceinline__ void frag4_mma_r(d4 (&acc)[QM][QN], const Frag4& f) {
#pragma unroll
  for (int s = 0; s < Q4SD; ++s)
#pragma unroll
    for (int a = A0; a < A1; ++a)
#pragma unroll
      for (int b = B0; b < B1; ++b) {
        if (LOWER && b > a) continue;
        acc[a][b] = mfma(SAME ? f.a[s][b] : f.b[s][b], f.a[s][a], acc[a][b]);
      }
}
// the prediction variance's core (k_gemm_pv): NB < QN: only the first NB 16-column blocks of B
// (the last, partly padded test tile); operands through CorePtr like the triangular cores
template <int NB = QN>
__device__ __forceinline__ void mma_64x64(d4 (&acc)[QM][QN], const double* __restrict__ A, size_t lda,
                                          const double* __restrict__ B, size_t ldb, int K) {
  const int nst = __builtin_amdgcn_readfirstlane(K / (4 * Q4SD));  // even: K is whole 64-tiles
  if (nst <= 0) return;
  const CorePtr pa = core_ptr(A, lda), pb = core_ptr(B, ldb);
  Frag4 f0, f1;
  frag4_load_r<0, QM, 0, NB, false>(f0, pa, pb, 0);
  for (int it = 0; it < nst; it += 2) {
    __builtin_amdgcn_sched_barrier(0);
    frag4_load_r<0, QM, 0, NB, false>(f1, pa, pb, it + 1);
    frag4_mma<NB>(acc, f0);
#pragma unroll
    for (int g = 0; g < Q4SD * (QM + NB); ++g) {
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // one VMEM read
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // two MFMAs
    }
    __builtin_amdgcn_sched_barrier(0);
    const int n2 = (it + 2 < nst) ? it + 2 : nst - 1;
    frag4_load_r<0, QM, 0, NB, false>(f0, pa, pb, n2);
    frag4_mma<NB>(acc, f1);
#pragma unroll
    for (int g = 0; g < Q4SD * (QM + NB); ++g) {
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}
// masks of trip T (0..3) of the triangular tile; T = 4: the dense trips
template <int MODE, int T>
struct TripMask {
  static constexpr bool first = MODE == TRI_A_FIRST || MODE == TRI_AB_FIRST || MODE == REV_A || MODE == REV_B;
  static constexpr bool dense = T >= 4 || (first && T == 3);
  static constexpr int a0 = (!dense && MODE == TRI_A_LAST) ? T : (!dense && MODE == REV_A) ? 3 - T : 0;
  static constexpr int a1 = (!dense && (MODE == TRI_A_FIRST || MODE == TRI_AB_FIRST)) ? T + 1 : QM;
  static constexpr int b0 = (!dense && MODE == TRI_B_LAST) ? T : (!dense && MODE == REV_B) ? 3 - T : 0;
  static constexpr int b1 = (!dense && MODE == TRI_AB_FIRST) ? T + 1 : QN;
};
template <int MODE, int T, class CP>
__device__ __forceinline__ void core_load(Frag4& f, const CP& A, const CP& B, int st) {
  constexpr bool same = MODE == TRI_AB_FIRST || MODE == LOWER_SAME;
  using M = TripMask<MODE, T>;
  frag4_load_r<M::a0, M::a1, M::b0, M::b1, same>(f, A, B, st);
}
template <int MODE, int T>
__device__ __forceinline__ void core_mma(d4 (&acc)[QM][QN], const Frag4& f) {
  using M = TripMask<MODE, T>;
  constexpr bool same = MODE == TRI_AB_FIRST || MODE == LOWER_SAME;
  frag4_mma_r<M::a0, M::a1, M::b0, M::b1, same, same>(acc, f);
}
// group barriers of a dense half trip: its loads spread evenly over its MFMAs (one load per two
// MFMAs; shared panels: 8 loads, 20 MFMAs)
template <int MODE>
__device__ __forceinline__ void core_groups() {
  constexpr bool same = MODE == TRI_AB_FIRST || MODE == LOWER_SAME;
  constexpr int la = Q4SD * QM, lb = same ? 0 : Q4SD * QN;
  constexpr int nl = la + lb, nm = Q4SD * (same ? 10 : QM * QN), q = nm / nl, r = nm % nl;
#pragma unroll
  for (int g = 0; g < r; ++g) {
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, q + 1, 0);
  }
#pragma unroll
  for (int g = r; g < nl; ++g) {
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, q, 0);
  }
}
template <int MODE, bool BUF = true>
__device__ __forceinline__ void mma_64x64_m(d4 (&acc)[QM][QN], const double* __restrict__ A, size_t lda,
                                            const double* __restrict__ B, size_t ldb, int K) {
  const int nst = __builtin_amdgcn_readfirstlane(K / (4 * Q4SD));  // multiple of 8: K is whole 64-tiles
  if (nst <= 0) return;
  const auto pa = core_addr<BUF>(A, lda), pb = core_addr<BUF>(B, ldb);
  constexpr bool first = MODE == TRI_A_FIRST || MODE == TRI_AB_FIRST;
  constexpr bool last = MODE == TRI_A_LAST || MODE == TRI_B_LAST;
  Frag4 f0, f1;
  // one peeled trip T of the triangular tile, stages st and st + 1; the prefetch of stage st + 2
  // uses trip T2's masks (NX: whether there is a next stage at all)
#define GPRX_TRIP(M, T, T2, st, NX)                  \
  {                                                  \
    __builtin_amdgcn_sched_barrier(0);               \
    core_load<M, T>(f1, pa, pb, (st) + 1);      \
    core_mma<M, T>(acc, f0);                         \
    __builtin_amdgcn_sched_barrier(0);               \
    if (NX) core_load<M, T2>(f0, pa, pb, (st) + 2); \
    core_mma<M, T>(acc, f1);                         \
  }
  int it = 0, end = nst;
  if constexpr (first) {
    core_load<MODE, 0>(f0, pa, pb, 0);
    GPRX_TRIP(MODE, 0, 1, 0, true)
    GPRX_TRIP(MODE, 1, 2, 2, true)
    GPRX_TRIP(MODE, 2, 3, 4, true)
    it = 6;
  } else {
    core_load<MODE, last ? 0 : 4>(f0, pa, pb, 0);
    if constexpr (last) end = nst - 8;
  }
  for (; it < end; it += 2) {
    __builtin_amdgcn_sched_barrier(0);
    core_load<MODE, 4>(f1, pa, pb, it + 1);
    core_mma<MODE, 4>(acc, f0);
    core_groups<MODE>();
    __builtin_amdgcn_sched_barrier(0);
    const int n2 = (it + 2 < nst) ? it + 2 : nst - 1;
    core_load<MODE, 4>(f0, pa, pb, n2);
    core_mma<MODE, 4>(acc, f1);
    core_groups<MODE>();
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (last) {  // the triangular last tile; f0 holds its stage 0 (dense masks)
    const int st = end;
    GPRX_TRIP(MODE, 0, 1, st, true)
    GPRX_TRIP(MODE, 1, 2, st + 2, true)
    GPRX_TRIP(MODE, 2, 3, st + 4, true)
    GPRX_TRIP(MODE, 3, 3, st + 6, false)
  }
  __builtin_amdgcn_sched_barrier(0);
}
// k_gemm's core: ONE copy of the dense loop and at most one peeled prefix per kernel instance (a
// second inlined copy of the loop, or a second peeled prefix / tail, makes the register allocator
// spill 150-700 VGPRs).  The instance's op (PM) has its triangular tile peeled in front of the
// loop: TT walks K forward from its upper-triangular first tile (Mt[ti,ti]); TRSM and LINV21 walk
// K backward from their lower-triangular last tile (Linv[tj,tj], Linv[ti,ti]: reversed trip T
// needs the row / column blocks >= 3 - T).  tri: this wave's op is PM's.
template <int PM, bool BUF = true>
__device__ __forceinline__ void mma_64x64_pm(d4 (&acc)[QM][QN], Frag4& f0, const double* __restrict__ A, size_t lda,
                                             const double* __restrict__ B, size_t ldb, int K, bool tri, bool pre, bool nxt,
                                             const double* nA, const double* nB, int nK) {
  // pre: f0 already holds this tile's first stage (loaded by the previous tile's last iteration);
  // nxt: the last iteration loads the next tile's first stage (operands nA, nB, K range nK, the
  // same op and walk) into f0 instead of re-reading its own last stage, so the next tile's first
  // MFMAs do not wait for a load issued after this tile's epilogue (round 5)
  const int nst = __builtin_amdgcn_readfirstlane(K / (4 * Q4SD));
  if (nst <= 0) return;
  auto pa = core_addr<BUF>(A, lda), pb = core_addr<BUF>(B, ldb);
  Frag4 f1;
  int it = 0;
  if (tri) {
    if constexpr (PM == REV_A || PM == REV_B) {  // stage j reads the k of stage nst - 1 - j
      pa = core_rev(pa, nst);
      pb = core_rev(pb, nst);
    }
    if (!pre) core_load<PM, 0>(f0, pa, pb, 0);
    GPRX_TRIP(PM, 0, 1, 0, true)
    GPRX_TRIP(PM, 1, 2, 2, true)
    GPRX_TRIP(PM, 2, 3, 4, true)
    it = 6;
  } else {
    if (!pre) core_load<PLAIN, 4>(f0, pa, pb, 0);
  }
  [[maybe_unused]] auto na = pa, nb = pb;
  if constexpr (BUF) {
    if (nxt) {
      const int nn = __builtin_amdgcn_readfirstlane(nK / (4 * Q4SD));
      na = core_addr<BUF>(nA, lda);
      nb = core_addr<BUF>(nB, ldb);
      if constexpr (PM == REV_A || PM == REV_B) {
        if (tri) {
          na = core_rev(na, nn);
          nb = core_rev(nb, nn);
        }
      }
    }
  }
  for (; it < nst; it += 2) {
    __builtin_amdgcn_sched_barrier(0);
    core_load<PLAIN, 4>(f1, pa, pb, it + 1);
    core_mma<PLAIN, 4>(acc, f0);
    core_groups<PLAIN>();
    __builtin_amdgcn_sched_barrier(0);
    const int n2 = (it + 2 < nst) ? it + 2 : nst - 1;
    if constexpr (BUF) {
      const bool nx = nxt && it + 2 >= nst;  // wave-uniform: scalar selects, no branch
      CorePtr la = pa, lb = pb;
      la.r = nx ? na.r : pa.r;
      la.o = nx ? na.o : pa.o + n2 * pa.st;
      la.sub = nx ? na.sub : pa.sub;
      lb.r = nx ? nb.r : pb.r;
      lb.o = nx ? nb.o : pb.o + n2 * pb.st;
      lb.sub = nx ? nb.sub : pb.sub;
      core_load<PLAIN, 4>(f0, la, lb, 0);
    } else {
      core_load<PLAIN, 4>(f0, pa, pb, n2);
    }
    core_mma<PLAIN, 4>(acc, f1);
    core_groups<PLAIN>();
    __builtin_amdgcn_sched_barrier(0);
  }
}
#undef GPRX_TRIP
// 64 x 16 wave core (the fused leaf's column-quarter tasks): acc[a] += A(64 x K) B(16 x K)^T,
// lane l reg q = C[16a + (l&15)][(l>>4) + 4q]; 4 MFMAs per 5 fragment loads, stages of depth 16
// in ping-pong (the same barriers as mma_64x64, groups of 5 loads and 4 MFMAs interleaved: leaf
// 2.18 -> 2.09 ms at B=240, same-box A/B).  K: whole 64-tiles.
struct Frag16 {
  double a[4][QM], b[4];
};
__device__ __forceinline__ void frag16_load(Frag16& f, const double* pa, const double* pb, size_t sa, size_t sb) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
#pragma unroll
    for (int a = 0; a < QM; ++a) f.a[s][a] = pa[s * sa + 16 * a];
    f.b[s] = pb[s * sb];
  }
}
__device__ __forceinline__ void frag16_mma(d4 (&acc)[QM], const Frag16& f) {
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int a = 0; a < QM; ++a) acc[a] = mfma(f.b[s], f.a[s][a], acc[a]);
}
__device__ __forceinline__ void mma_64x16(d4 (&acc)[QM], const double* __restrict__ A, size_t lda,
                                          const double* __restrict__ B, size_t ldb, int K) {
  const int nst = __builtin_amdgcn_readfirstlane(K >> 4);  // even: K is whole 64-tiles
  if (nst <= 0) return;
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const double* pa = A + lr + (size_t)lk * lda;
  const double* pb = B + lr + (size_t)lk * ldb;
  const size_t sa = 4 * lda, sb = 4 * ldb;
  Frag16 f0, f1;
  frag16_load(f0, pa, pb, sa, sb);
  for (int it = 0; it < nst; it += 2) {
    __builtin_amdgcn_sched_barrier(0);
    frag16_load(f1, pa + (size_t)(it + 1) * 4 * sa, pb + (size_t)(it + 1) * 4 * sb, sa, sb);
    frag16_mma(acc, f0);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x020, 5, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    const int n2 = (it + 2 < nst) ? it + 2 : nst - 1;
    frag16_load(f0, pa + (size_t)n2 * 4 * sa, pb + (size_t)n2 * 4 * sb, sa, sb);
    frag16_mma(acc, f1);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x020, 5, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}
// mma_64x16 with the B operand from the wave's LDS buffer: B(j, k) = tb[j * (TS + 1) + k] (a
// column quarter kept transposed in LDS by the producer), K = 64 (one tile)
__device__ __forceinline__ void mma_64x16_ldsb(d4 (&acc)[QM], const double* __restrict__ A, size_t lda, const double* tb) {
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const double* pa = A + lr + (size_t)lk * lda;
  const double* pb = tb + lr * (TS + 1) + lk;
  const size_t sa = 4 * lda;
#pragma unroll
  for (int st = 0; st < TS / 16; ++st) {
    double a[4][QM], b[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int q = 0; q < QM; ++q) a[s][q] = pa[(size_t)(4 * st + s) * sa + 16 * q];
      b[s] = pb[16 * st + 4 * s];
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int q = 0; q < QM; ++q) acc[q] = mfma(b[s], a[s][q], acc[q]);
  }
}
// ---- diagnostic build only (-DGPRX_STAMPS, scratch/clock.py): the in-kernel clock of a main loop
// (MI355X_MICROARCH.md 'DVFS give-back' item 6): s_memtime (shader cycles) and s_memrealtime
// (100 MHz) before and after, per wave, into a buffer no other code reads.  Not in the product build.
#ifdef GPRX_STAMPS
constexpr int STAMP_MAX = 1 << 18;  // waves per stamp region
__device__ unsigned long long g_stamps[3][STAMP_MAX][4];
struct Stamp {
  unsigned long long t, r;
};
__device__ __forceinline__ Stamp stamp_now() {
  __builtin_amdgcn_sched_barrier(0);
  Stamp s{__builtin_amdgcn_s_memtime(), __builtin_amdgcn_s_memrealtime()};
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only
  __builtin_amdgcn_sched_barrier(0);
  return s;
}
__device__ __forceinline__ void stamp_store(int region, const Stamp& a, const Stamp& b) {
  const size_t i = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0 && i < STAMP_MAX) {
    g_stamps[region][i][0] = a.t;
    g_stamps[region][i][1] = b.t;
    g_stamps[region][i][2] = a.r;
    g_stamps[region][i][3] = b.r;
  }
}
// leaf timeline: s_memrealtime of wave 0 at event ev of leaf o / 4 of this slot (slots < 256)
__device__ __forceinline__ void leaf_ts(int o, int slot, int ev) {
  if (threadIdx.x == 0 && slot < 256) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    (&g_stamps[2][0][0])[((size_t)((o >> 2) & 7) * 256 + slot) * 32 + ev] = t;
  }
}
#define LEAF_TS(ev) leaf_ts(o, slot, ev)
// k_leaf9 timeline (scratch/leaf8_timeline.py): lane 0 of the calling wave stamps event ev of
// leaf o / 4 of this slot
__device__ __forceinline__ void leaf9_ts(int o, int slot, int ev) {
  if ((threadIdx.x & 63) == 0 && slot < 256) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    (&g_stamps[2][0][0])[((size_t)((o >> 2) & 7) * 256 + slot) * 32 + ev] = t;
  }
}
#define L9_TS(ev) leaf9_ts(o, slot, ev)
// the single-wave diagonal routine's internal events (after the leaf stamps in region 2)
__device__ __forceinline__ void diag_ts(int jt, int slot, int ev) {
  if ((threadIdx.x & 63) == 0 && slot < 256) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    (&g_stamps[2][0][0])[65536 + ((((size_t)((jt >> 2) & 7) * 256 + slot) * 4 + (jt & 3)) * 16) + ev] = t;
  }
}
#define D_TS1(ev) diag_ts(jt, slot, ev)
// per-wave item events of the leaf's phase B (after the diagonal routine's events)
__device__ __forceinline__ void wave_ts(int o, int slot, int ev) {
  if ((threadIdx.x & 63) == 0 && slot < 256) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    (&g_stamps[2][0][0])[196608 + ((((size_t)((o >> 2) & 7) * 256 + slot) * 8 + (threadIdx.x >> 6)) * 32) + ev] = t;
  }
}
#define W_TS(ev) wave_ts(o, slot, ev)
// whole-node kernels (k_node8 / k_node8h): thread 0 stamps phase ev of slot's node launch (region
// 0 from entry 2^19: 8 per slot: start, after the top leaf, TRSM, SYRK + TT, the bottom leaf, end,
// then the hardware CU id and XCC id)
__device__ __forceinline__ void node_ts(int slot, int ev) {
  if (threadIdx.x == 0 && slot < 32768) {
    unsigned long long t = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    if (ev == 6) t = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
    if (ev == 7) t = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11));
    (&g_stamps[0][0][0])[524288 + (size_t)slot * 8 + ev] = t;
  }
}
#define N_TS(ev) node_ts(slot, ev)
#else
#define N_TS(ev)
#define D_TS1(ev)
#define LEAF_TS(ev)
#define L9_TS(ev)
#define W_TS(ev)
#endif
// ---- diagnostic build only (-DGPRX_GSTAMPS=op*100+n, scratch/gemm_timeline.py): per-wave
// s_memrealtime of the GEMM launch of op at node size n: tile entry, core start, core end (loads
// landed), epilogue end (stores landed), for the wave's first two tiles.  Not in the product build.
#ifdef GPRX_GSTAMPS
constexpr int GTS_MAX = 1 << 17;
__device__ unsigned long long g_gts[GTS_MAX][8];
__device__ __forceinline__ void gts(const GemmGeom& g, int pass, int ev) {
  if (GPRX_GSTAMPS == 1208) {  // k_node8's SYRK + TT phase: every wave (8 per block), 4 tiles, 4 events
    if (!((g.op == OP_SYRK || g.op == OP_TT) && g.n == 8) || pass > 3 || blockDim.x != 512) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    const size_t i = (size_t)blockIdx.x * 8 + (threadIdx.x >> 6);
    if ((threadIdx.x & 63) == 0 && 2 * i + 1 < GTS_MAX) (&g_gts[0][0])[i * 16 + 4 * pass + ev] = t;
    return;
  }
  if (g.op * 100 + g.n != GPRX_GSTAMPS || pass > 1) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long t = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  const size_t i = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0 && i < GTS_MAX) g_gts[i][4 * pass + ev] = t;
}
#define GTS(g, pass, ev) gts(g, pass, ev)
// the gradient GEMM (GPRX_GSTAMPS=999): job entry, then per unit u: main loop start, main loop end,
// unit end, at slots 1 + 3u ..; =998: unit 0 only, with its epilogue phases (gts_d)
__device__ __forceinline__ void gts_d(int gu, int ev) {  // =998: unit 0's epilogue phases at slots 4..7
  if (GPRX_GSTAMPS != 998 || gu != 0) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long t = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  const size_t i = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0 && i < GTS_MAX) g_gts[i][ev] = t;
}
__device__ __forceinline__ void gts_l(int ev) {
  if (GPRX_GSTAMPS != 999 && !(GPRX_GSTAMPS == 998 && ev < 4)) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long t = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  const size_t i = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0 && i < GTS_MAX) g_gts[i][ev] = t;
}
#define GTS_L(ev) gts_l(ev)
#define GTS_D(gu, ev) gts_d(gu, ev)
#else
#define GTS_D(gu, ev)
#define GTS(g, pass, ev)
#define GTS_L(ev)
#endif
__device__ __forceinline__ void acc4_zero(d4 (&acc)[QM][QN]) {
#pragma unroll
  for (int a = 0; a < QM; ++a)
#pragma unroll
    for (int b = 0; b < QN; ++b) acc[a][b] = (d4){0.0, 0.0, 0.0, 0.0};
}

// z = L^-1 y fused into the producers of L^-1: every L^-1 tile (ti, tj) (written exactly once, by
// a diagonal kernel, the leaf or LINV21) also writes its 64-row partial  L^-1[ti,tj] y[tj]  into
// zp[slot][2 tj + half][ti*64 + r] (half: 32-column halves of the pair-unit GEMM; 64-column
// producers write half 0 and zero half 1).  k_alpha phase 0 then sums <= 2(ti+1) partials per row
// instead of re-reading L^-1 from HBM.
// 64 x 64 accumulator tile (mma_64x64 layout) of sgn * L^-1[ti,tj]
__device__ __forceinline__ void zp_acc4(const DevBatch& db, int slot, int ti, int tj, const d4 (&acc)[QM][QN], double sgn) {
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const double* y = db.Y + (size_t)slot * db.Npad + tj * TS;
  double yv[QN][4];
#pragma unroll
  for (int b = 0; b < QN; ++b)
#pragma unroll
    for (int q = 0; q < 4; ++q) yv[b][q] = y[16 * b + lk + 4 * q];
  double* z0 = zp_row(db, slot, 2 * tj) + ti * TS;
  double* z1 = zp_row(db, slot, 2 * tj + 1) + ti * TS;
#pragma unroll
  for (int a = 0; a < QM; ++a) {
    double t = 0.0;
#pragma unroll
    for (int b = 0; b < QN; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) t = fma(acc[a][b][q], yv[b][q], t);
    t = sum_xor32(sum_xor16(t));
    if (lk == 0) {
      z0[16 * a + lr] = sgn * t;
      z1[16 * a + lr] = 0.0;
    }
  }
}
// Units of the 4-wave workgroups of k_gemm / k_lauum_grad: UR x UC output tiles (UR UC = 4), wave w
// = tile (pr + w / UC, pc + w % UC).  The shape follows the op so that the four waves of a unit
// share one K range where it varies by tile: TRSM (K grows with the column) 4 x 1, TT / LINV21 (K
// set by the row) 1 x 4, SYRK (fixed K; lower triangle) and PREDVAR 2 x 2.
__host__ __device__ inline void unit_shape(int op, int& UR, int& UC) {
  UR = op == OP_TRSM ? 4 : ((op == OP_TT || op == OP_LINV21) ? 1 : 2);
  UC = 4 / UR;
}
// rect R x C: ceil(R/UR) x ceil(C/UC) units; lower triangle of R x R (tri: SYRK, fixed K): four
// consecutive tiles of the row-major lower triangle per unit (no idle wave on the diagonal)
__host__ __device__ inline int quad_units(int R, int C, bool tri, int UR = 2, int UC = 2) {
  if (tri) return (R * (R + 1) / 2 + 3) / 4;
  return ((R + UR - 1) / UR) * ((C + UC - 1) / UC);
}
// Triangular-K ops are folded: a workgroup computes the unit with the longest K range and then
// its mirror along the K-varying dimension (TRSM: columns; TT, LINV21, PREDVAR: rows), so every
// workgroup carries about the same K (measured 58.7 -> 67.4 TF/s on a TRSM-shaped launch,
// scratch/gemm3_bench.hip).
__host__ __device__ inline int op_units(const GemmGeom& g, int nt, int mt) {
  int r0, c0, R, C, UR, UC;
  bool tri;
  op_rect(g, nt, mt, r0, c0, R, C, tri);
  unit_shape(g.op, UR, UC);
  if (tri || g.op == OP_SYRK) return quad_units(R, C, tri, UR, UC);
  const int RU = (R + UR - 1) / UR, CU = (C + UC - 1) / UC;
  return g.op == OP_TRSM ? RU * ((CU + 1) / 2) : ((RU + 1) / 2) * CU;
}
__device__ __forceinline__ void quad_tri(int u, int& rp, int& cp) {
  int r = (int)((sqrtf(8.0f * u + 1.0f) - 1.0f) * 0.5f);
  while ((r + 1) * (r + 2) / 2 <= u) ++r;
  while (r * (r + 1) / 2 > u) --r;
  rp = r;
  cp = u - r * (r + 1) / 2;
}

__device__ __forceinline__ void acc_zero(d4 (&acc)[WM][WN]) {
#pragma unroll
  for (int a = 0; a < WM; ++a)
#pragma unroll
    for (int b = 0; b < WN; ++b) acc[a][b] = (d4){0.0, 0.0, 0.0, 0.0};
}

// ============================================================================================
// Gram: lower tiles of K (noise on the diagonal).  grid = B * ntl, 256 threads, each thread
// a 4x4 register block; X tiles in dynamic LDS as [p][64].
// ============================================================================================
// Coordinate images in LDS, dimension-major with row stride CS = 66 doubles: the tile loads write
// them with the dimension as the fast index across lanes, and a stride of 64 put every dimension of
// a point in one bank (26-way conflicts on each ds_write_b64); 66 spreads them over the banks and
// keeps the 16-B alignment of the inner loop's ds_read_b128.
constexpr int CS = TS + 2;
template <int MODE>
__global__ __launch_bounds__(NTHR) void k_gram(DevBatch db) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  __shared__ __attribute__((aligned(16))) double tab[128];  // exp_sf's sf2 2^(j/64) table (static: a
                                                            // known LDS address, no base add)
  const int d = db.d, tid = threadIdx.x;
  double* xi = sm;
  double* xj = xi + d * CS;
  double* pw = xj + d * CS;
  int slot, t, i = 0, j = 0;
  if (!map_slot(db, db.ntl, slot, t)) return;
  {  // t-th lower tile in column-major order
    int c = 0, u = t;
    while (u >= db.nt - c) {
      u -= db.nt - c;
      ++c;
    }
    j = c;
    i = c + u;
  }
  const double* X = db.X + (size_t)slot * db.Npad * d;
  const double* P = db.params + (size_t)slot * db.pst;
  {  // thread -> (dimension p = tid mod 32 + 32 k, rows tid / 32 + 8 m): no per-element division,
     // 16 loads in flight per thread, coalesced over the 32 dimensions of a point row
    // buffer loads: the lane's byte offset in a VGPR, the row step and tile base in SGPRs, so no
    // per-load address arithmetic (64-bit global addresses cost 2-3 VALU per load here)
    const __amdgpu_buffer_rsrc_t xr = buffer_rsrc(X, db.Npad * d * (int)sizeof(double));
    const int bi = i * TS * d * (int)sizeof(double), bj = j * TS * d * (int)sizeof(double);
    const int os = 8 * d * (int)sizeof(double);
    for (int p = tid & 31; p < d; p += 32) {
      double vi[TS / 8], vj[TS / 8];
      const int o0 = ((tid >> 5) * d + p) * (int)sizeof(double);
#pragma unroll
      for (int m = 0; m < TS / 8; ++m) {
        vi[m] = buffer_load_f64(xr, o0, bi + m * os);
        vj[m] = buffer_load_f64(xr, o0, bj + m * os);
      }
      // direct mode: coordinates pre-scaled by 1/(sqrt(2) ell_p) = sqrt(il2_p / 2), so that the
      // sums are r/2, the exponent's magnitude (0.5 il2_p is exact: as accurate as scaling by
      // 1/ell_p); each thread scales its own dimension (no staging barrier)
      const double s = MODE == 1 ? sqrt(0.5 * P[p]) : 1.0;
#pragma unroll
      for (int m = 0; m < TS / 8; ++m) {
        const int r = (tid >> 5) + 8 * m;
        xi[p * CS + r] = vi[m] * s;
        xj[p * CS + r] = vj[m] * s;
      }
    }
  }
  for (int e = tid; e < d + 3; e += NTHR) pw[e] = P[e];
  if (tid < 64) {  // sf2 (hi_j + lo_j) as hi + lo: the product's rounding error by fma, plus sf2 lo_j
    const double s2 = P[d], h = g_exp2tab[2 * tid], lo = g_exp2tab[2 * tid + 1];
    const double th = s2 * h;
    tab[2 * tid] = th;
    tab[2 * tid + 1] = fma(s2, h, -th) + s2 * lo;
  }
  __syncthreads();
  const double noise = pw[d + 1];
  const ExpK ek = g_expk;
  const int rb = tid & 15, cb = tid >> 4;
  double rr[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) rr[a][b] = 0.0;
  for (int p = 0; p < d; ++p) {
    const double2 u0 = *(const double2*)(xi + p * CS + 4 * rb);
    const double2 u1 = *(const double2*)(xi + p * CS + 4 * rb + 2);
    const double2 v0 = *(const double2*)(xj + p * CS + 4 * cb);
    const double2 v1 = *(const double2*)(xj + p * CS + 4 * cb + 2);
    const double av[4] = {u0.x, u0.y, u1.x, u1.y};
    const double bv[4] = {v0.x, v0.y, v1.x, v1.y};
    const double w = pw[p];
    double a2[4], b2[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      a2[a] = av[a] * av[a];
      b2[a] = bv[a] * bv[a];
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        if (MODE == 0) {
          rr[a][b] = wacc<0>(rr[a][b], av[a], a2[a], bv[b], b2[b], w);
        } else {  // r += (a/ell - b/ell)^2: 2 fp64 ops per element and dimension
          const double t = av[a] - bv[b];
          rr[a][b] = __builtin_fma(t, t, rr[a][b]);
        }
      }
  }
  double* K = db.K + (size_t)slot * db.mat;
  // buffer stores over the tile (base uniform): the lane's byte offset in a VGPR (column step
  // added per store), no 64-bit address arithmetic per store
  const __amdgpu_buffer_rsrc_t kr = buffer_rsrc(K + (size_t)j * TS * db.ld + i * TS, 0x7ffffff0);
  const int ldb = (int)db.ld * (int)sizeof(double), lof = 4 * cb * ldb + 4 * rb * (int)sizeof(double);
  if (i != j && (i + 1) * TS <= db.N) {  // off-diagonal tile inside N x N (block-uniform): no tests
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      double kv[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) kv[a] = exp_sf(MODE == 1 ? -rr[a][b] : -rr[a][b] * 0.5, ek, tab);
      buffer_store_f64x2(kr, lof + b * ldb, kv[0], kv[1]);
      buffer_store_f64x2(kr, lof + b * ldb + 16, kv[2], kv[3]);
    }
    return;
  }
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int gj = j * TS + 4 * cb + b;
    double kv[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {  // branch-free: padded points (finite coordinates) are selected away
      const int gi = i * TS + 4 * rb + a;
      const double fv = exp_sf(MODE == 1 ? -rr[a][b] : -rr[a][b] * 0.5, ek, tab);
      const bool pad = gi >= db.N || gj >= db.N;
      kv[a] = (gi == gj) ? (pad ? 1.0 : fv + noise) : (pad ? 0.0 : fv);
    }
    buffer_store_f64x2(kr, lof + b * ldb, kv[0], kv[1]);
    buffer_store_f64x2(kr, lof + b * ldb + 16, kv[2], kv[3]);
  }
}

// Centred copy of the training points: Xc[t][p] = X[t][p] - mean_t X[t][p] for t < N, p < d, and 0
// elsewhere (padded points, padded dimensions up to the stride xs).  grid = B, once per
// gprx_batch_set_train.
__global__ __launch_bounds__(NTHR) void k_center(DevBatch db) {
  __shared__ double mean[DMAX];
  __shared__ double red[4];
  const int slot = blockIdx.x, tid = threadIdx.x, d = db.d, xs = db.xs;
  const double* X = db.X + (size_t)slot * db.Npad * d;
  double* Xc = db.Xc + (size_t)slot * db.Npad * xs;
  for (int p = 0; p < d; ++p) {
    double s = 0.0;
    for (int t = tid; t < db.N; t += NTHR) s += X[(size_t)t * d + p];
    s = wave_sum(s);
    __syncthreads();
    if ((tid & 63) == 0) red[tid >> 6] = s;
    __syncthreads();
    if (tid == 0) mean[p] = (((red[0] + red[1]) + red[2]) + red[3]) / db.N;
  }
  __syncthreads();
  for (int e = tid; e < db.Npad * xs; e += NTHR) {
    const int t = e / xs, p = e - t * xs;
    Xc[e] = (t < db.N && p < d) ? X[(size_t)t * d + p] - mean[p] : 0.0;
  }
}

// ============================================================================================
// Leaf of the recursion: Cholesky of the 64x64 diagonal tile jt (already reduced by the SYRK
// updates of its ancestors) and its inverse, one workgroup (4 waves) per slot, blocked by 16:
// the 16x16 diagonal blocks are factored and inverted in registers by wave 0 (lane = row /
// column, pivots and row values broadcast by readlane), the panel TRSM / trailing SYRK and the
// off-diagonal blocks of the inverse run on the MFMA pipe from an LDS image of the tile.
// 4 + 3 barrier-separated phases per panel instead of 128 steps.
//   panel P (c0 = 16P):  D = chol(A_PP), Dinv = D^-1               (wave 0)
//                        A_iP <- A_iP Dinv^T  (i > P)              (TRSM, one wave per block)
//                        A_ij -= A_iP A_jP^T  (i >= j > P)          (SYRK)
//   inverse:  X_PP = Dinv_P ;  X_ij = -Dinv_i sum_{k=j}^{i-1} L_ik X_kj   by sub-diagonal i - j
// Failure (first pivot <= 0 or NaN, as LAPACK dpotrf) records status 1 and the 1-based global
// pivot index and continues with pivot 1.  Writes Linv[jt,jt] = L_jj^-1 and Mt[jt,jt] = L_jj^-T
// (full tiles, explicit zeros) and the tile's sum_c log L_cc.
// 16x16x4 f64 MFMA operand maps (gfx950): A lane l = A[l&15][l>>4], B lane l = B[l>>4][l&15],
// D lane l reg q = D[(l>>4) + 4q][l&15].
// ============================================================================================
constexpr int FS = TS + 1;  // LDS column stride of the tile images
// LDS of the diagonal routine (the caller's): T[c*FS + r] = A[r][c], then L (lower); Xi[c*FS + r]
// = X[r][c] = (L^-1)[r][c] (the inverse stays there until the next call); cbs: [256] scratch.
// t_ready: T already holds the tile's lower triangle (zeros above), written by the caller; else
// it is read from Ksrc (K, or S when a SYRK updated it).
__device__ __forceinline__ void diag_tile_fast(const DevBatch& db, int slot, int jt, double* T, double* Xi, double* cbs,
                                               bool t_ready, const double* Ksrc, bool store = true);
__device__ __forceinline__ void diag_store(const DevBatch& db, int slot, int jt, const double* Xi, double* cbs);
__global__ __launch_bounds__(NTHR) void k_diag_f(DevBatch db, int jt, int upd) {
  __shared__ double T[TS * FS], Xi[TS * FS];
  __shared__ __attribute__((aligned(16))) double cbs[256];
  if (slot_active(db, blockIdx.x)) diag_tile_fast(db, blockIdx.x, jt, T, Xi, cbs, false, upd ? db.S : db.K);
}
__device__ __forceinline__ void diag_tile_fast(const DevBatch& db, int slot, int jt, double* T, double* Xi, double* cbs,
                                               bool t_ready, const double* Ksrc, bool store) {
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lr = l & 15, lk = l >> 4;
  const size_t ld = db.ld;
  const double* A = Ksrc + (size_t)slot * db.mat + (size_t)jt * TS * ld + jt * TS;
  if (!t_ready) {  // all 16 loads of a thread in flight before the LDS stores (one latency, not 16)
    double v[TS * TS / NTHR];
#pragma unroll
    for (int k = 0; k < TS * TS / NTHR; ++k) {
      const int e = tid + k * NTHR, r = e & 63, c = e >> 6;
      v[k] = (r >= c) ? A[(size_t)c * ld + r] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < TS * TS / NTHR; ++k) {
      const int e = tid + k * NTHR, r = e & 63, c = e >> 6;
      T[c * FS + r] = v[k];
    }
  }
  for (int e = tid; e < TS * TS; e += NTHR) Xi[(e >> 6) * FS + (e & 63)] = 0.0;
  __syncthreads();
  int fail = -1;
  double lsum = 0.0;  // wave 0: sum log l_jj
  for (int P = 0; P < 4; ++P) {
    const int c0 = 16 * P;
    if (w == 0) {
      // ---- factor and invert the diagonal block together, by elimination on 16 lanes: lane i
      //      holds row i of the block (a[k] = A[c0+i][c0+k], becoming L) and column i of its
      //      inverse (y[m] = X[m][i], starting from the identity).  Step j scales column j of L and
      //      row j of X by 1/l_jj, then L[m][j] (lane m's a[j]) is broadcast to the row of 16 lanes
      //      by DPP (row_newbcast: no LDS round trip) and updates both A (a[m] -= L[i][j] L[m][j])
      //      and X (X[m][i] -= L[m][j] X[j][i]).  The operations and their order are those of the
      //      column-by-column factor followed by the row-oriented forward substitution, so the
      //      results are bit-identical to that form. ----
      double a[16], y[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        a[k] = T[(c0 + k) * FS + c0 + lr];
        y[k] = (k == lr) ? 1.0 : 0.0;
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const double p = readlane_d(a[j], j);
        const double pk = (p > 0.0) ? p : 1.0;
        if (!(p > 0.0) && fail < 0) fail = c0 + j;
        double ljj, rj;
        sqrt_rsqrt(pk, ljj, rj);
        a[j] = (lr > j) ? a[j] * rj : (lr == j ? ljj : 0.0);
        y[j] = y[j] * rj;
#pragma unroll
        for (int m = j + 1; m < 16; ++m) {
          const double b = row_bcast16(a[j], m);  // L[m][j]
          a[m] = fma(-a[j], b, a[m]);
          y[m] = fma(-b, y[j], y[m]);
        }
      }
      double (&x)[16] = y;
      if (l < 16) {
#pragma unroll
        for (int k = 0; k < 16; ++k) T[(c0 + k) * FS + c0 + l] = (k <= l) ? a[k] : 0.0;  // row l of L_PP
      }
      __builtin_amdgcn_wave_barrier();
      if (l < 16) {
#pragma unroll
        for (int r = 0; r < 16; ++r) Xi[(c0 + l) * FS + c0 + r] = x[r];    // column l of Dinv
      }
    }
    __syncthreads();
    // ---- TRSM: block row i > P:  A_iP <- A_iP Dinv^T   (D[r][c] = sum_k A_iP[r][k] Dinv[c][k]) ----
    {
      const int i = P + 1 + w;
      if (i < 4) {
        d4 acc = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int k = 4 * s + lk;
          const double av = T[(c0 + k) * FS + 16 * i + lr];   // A_iP[lr][k]
          const double bv = Xi[(c0 + k) * FS + c0 + lr];      // B[k][j=lr] = Dinv[lr][k]
          acc = mfma(av, bv, acc);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) T[(c0 + lr) * FS + 16 * i + lk + 4 * q] = acc[q];  // D[lk+4q][lr]
      }
    }
    __syncthreads();
    // ---- SYRK: A_ij -= A_iP A_jP^T for P < j <= i < 4 ----
    {
      const int m = 3 - P;  // trailing blocks per edge
      for (int t = w; t < m * (m + 1) / 2; t += 4) {
        int u = t, j = 0;
        while (u >= m - j) {
          u -= m - j;
          ++j;
        }
        const int bj = P + 1 + j, bi = bj + u;
        d4 acc = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int k = 4 * s + lk;
          const double av = T[(c0 + k) * FS + 16 * bi + lr];  // A_iP[lr][k]
          const double bv = T[(c0 + k) * FS + 16 * bj + lr];  // B[k][lr] = A_jP[lr][k]
          acc = mfma(av, bv, acc);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          double* pp = &T[(16 * bj + lr) * FS + 16 * bi + lk + 4 * q];
          *pp = *pp - acc[q];
        }
      }
    }
    __syncthreads();
  }
  // ---- off-diagonal blocks of the inverse, by sub-diagonal s = i - j ----
  for (int sd = 1; sd < 4; ++sd) {
    const int j = w, i = w + sd;
    if (i < 4) {
      // Y = sum_{k=j}^{i-1} L_ik X_kj
      d4 y = (d4){0.0, 0.0, 0.0, 0.0};
      for (int kb = j; kb < i; ++kb)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int k = 4 * s + lk;
          const double av = T[(16 * kb + k) * FS + 16 * i + lr];    // L_ik[lr][k]
          const double bv = Xi[(16 * j + lr) * FS + 16 * kb + k];   // X_kj[k][lr]
          y = mfma(av, bv, y);
        }
      // X_ij = -Dinv_i Y ; Y's D layout (reg q = Y[lk+4q][lr]) is the B operand of k-chunk q
      d4 x = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const double av = Xi[(16 * i + 4 * s + lk) * FS + 16 * i + lr];  // Dinv_i[lr][4s+lk]
        x = mfma(av, y[s], x);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) Xi[(16 * j + lr) * FS + 16 * i + lk + 4 * q] = -x[q];
    }
    __syncthreads();
  }
  if (w == 0) {  // fail: uniform over wave 0; sum log l_jj from the diagonal of T, one per lane
    lsum = wave_sum(log(T[l * FS + l]));
    if (l == 0) {
      db.logdet_part[(size_t)slot * db.nt + jt] = lsum;
      if (fail >= 0 && db.status[slot] == 0) {
        db.status[slot] = 1;
        db.info[slot] = jt * TS + fail + 1;
      }
    }
  }
  if (store) diag_store(db, slot, jt, Xi, cbs);
}
// The diagonal routine's results to HBM: Linv[jt,jt], Mt[jt,jt] and the tile's z partial, from the
// inverse image Xi (LDS).  The fused leaf issues them after its TRSM tasks' loads: issued first, the
// stores sat ahead of those loads in the in-order counter and zp_diag's barriers drained them.
__device__ __forceinline__ void diag_store(const DevBatch& db, int slot, int jt, const double* Xi, double* cbs) {
  const int tid = threadIdx.x;
  const size_t ld = db.ld;
  double* Li = db.Linv + (size_t)slot * db.mat + (size_t)jt * TS * ld + jt * TS;
  double* Mj = db.Mt + (size_t)slot * db.mat + (size_t)jt * TS * ld + jt * TS;
  for (int e = tid; e < TS * TS; e += NTHR) {
    const int r = e & 63, c = e >> 6;
    const double v = (r >= c) ? Xi[c * FS + r] : 0.0;
    Li[(size_t)c * ld + r] = v;                              // Linv[r][c]
    Mj[(size_t)c * ld + r] = (c >= r) ? Xi[r * FS + c] : 0.0;  // Mt[r][c] = X[c][r]
  }
  zp_diag(db, slot, jt, Xi, 1, FS, cbs);
}


// ============================================================================================
// Generic batched tile GEMM of the recursion (see GemmOp).  Unit = 4 output tiles (unit_shape;
// a triangular SYRK: 4 consecutive lower tiles); each wave computes one 64 x 64 tile with its own
// K range (triangular operands are skipped at tile granularity).  Waves of tiles outside the rectangle / above the diagonal
// return at once (no workgroup barrier in this kernel).
// ============================================================================================
// One 64 x 64 output tile (ti, tj) of a GemmOp on one wave.
constexpr int TT_S = TS + 2;  // row stride of k_gemm's per-wave transpose buffer (LINV21's Mt store)
constexpr size_t linv21_lds_bytes() { return (size_t)4 * 32 * TT_S * sizeof(double); }  // 4 waves x [32][66]
// operands of tile (ti, tj) of a GemmOp: A and B at the K range's start, B's leading dimension,
// the K range (elements)
struct TileOps {
  const double *A, *B;
  size_t ldb;
  int Kn;
};
__device__ __forceinline__ TileOps tile_ops(const DevBatch& db, int op, const GemmGeom& g, int slot, int ti, int tj) {
  const size_t ld = db.ld, so = (size_t)slot * db.mat;
  int kb, ke;  // K range in tiles
  const double *A, *Bm;
  size_t ldb = ld;
  switch (op) {
    case OP_TRSM: kb = g.o; ke = tj + 1; A = (g.upd ? db.S : db.K) + so; Bm = db.Linv + so; break;
    case OP_SYRK: kb = g.o; ke = g.o + g.h; A = db.Lw + so; Bm = db.Lw + so; break;
    case OP_TT: kb = ti; ke = g.o + g.h; A = db.Mt + so; Bm = db.Lw + so; break;
    case OP_LINV21: kb = g.o + g.h; ke = ti + 1; A = db.Linv + so; Bm = db.Lw + so; break;
    default:
      kb = 0;
      ke = ti + 1;
      A = db.Linv + so;
      Bm = db.KsT + (size_t)slot * db.Npad * db.Mpad;
      ldb = db.Mpad;
      break;
  }
  return TileOps{A + (size_t)kb * TS * ld + ti * TS, Bm + (size_t)kb * TS * ldb + tj * TS, ldb, (ke - kb) * TS};
}
// f0 / pre / nxt / (nti, ntj): the register stage handed from one tile of a wave's folded pair to
// the next (mma_64x64_pm)
template <bool PV, int PM = PLAIN, bool BUF = true>
__device__ __forceinline__ void gemm_tile(const DevBatch& db, const GemmGeom& g, int slot, int ti, int tj, int pass, Frag4& f0,
                                          bool pre, bool nxt, int nti, int ntj) {
  GTS(g, pass, 0);
  const int op = PV ? (int)OP_PREDVAR : g.op;
  const size_t ld = db.ld, so = (size_t)slot * db.mat;
  const TileOps to = tile_ops(db, op, g, slot, ti, tj);
  const size_t ldb = to.ldb;
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  // the output tile's addressing (the SYRK's C and every op's stores): buffer ops over the tile,
  // the lane's byte offset per q in a VGPR, the 16-column block b in an SGPR, the row block a in the
  // offset field: no per-element 64-bit address arithmetic
  const int Lb = (int)ld * (int)sizeof(double);
  const int vl = lk * Lb + lr * (int)sizeof(double);  // + 4 q Lb (formed where used: not live across the K loop)
  d4 acc[QM][QN];
  if (op == OP_SYRK) {  // acc = -C, loaded before the K loop so its latency overlaps the first stage
    const __amdgpu_buffer_rsrc_t cr = buffer_rsrc((g.upd ? db.S : db.K) + so + (size_t)(tj * TS) * ld + ti * TS, 0x7ffffff0);
#pragma unroll
    for (int a = 0; a < QM; ++a)
#pragma unroll
      for (int b = 0; b < QN; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[a][b][q] = neg_f64(buffer_load_f64(cr, vl + 128 * a, (16 * b + 4 * q) * Lb));
  } else {
    acc4_zero(acc);
  }
  const double* Ak = to.A;
  const double* Bk = to.B;
  if constexpr (PV) {  // prediction (own kernel instance): skip the last test tile's all-padding blocks
    const int nbv = __builtin_amdgcn_readfirstlane((db.M - tj * TS + 15) >> 4);
    if (nbv >= QN) mma_64x64(acc, Ak, ld, Bk, ldb, to.Kn);
    else if (nbv == 3) mma_64x64<3>(acc, Ak, ld, Bk, ldb, to.Kn);
    else if (nbv == 2) mma_64x64<2>(acc, Ak, ld, Bk, ldb, to.Kn);
    else mma_64x64<1>(acc, Ak, ld, Bk, ldb, to.Kn);
  } else {
#ifdef GPRX_STAMPS
    const Stamp st0 = stamp_now();
#endif
    // the operands' triangular tiles (diagonal tiles of Linv / Mt) and SYRK's upper blocks of a
    // diagonal tile are skipped (mma_64x64_m); op and ti == tj are wave-uniform
    const bool tri = (PM == TRI_A_FIRST && op == OP_TT) || (PM == REV_A && op == OP_LINV21) || (PM == REV_B && op == OP_TRSM);
    TileOps tn = to;
    if (nxt) tn = tile_ops(db, op, g, slot, nti, ntj);
    GTS(g, pass, 1);
    mma_64x64_pm<PM, BUF>(acc, f0, Ak, ld, Bk, ldb, to.Kn, tri, pre, nxt, tn.A, tn.B, tn.Kn);
    GTS(g, pass, 2);
#ifdef GPRX_STAMPS
    if ((op == OP_SYRK || op == OP_TT) && g.n == db.nt) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      stamp_store(1, st0, stamp_now());
    }
#endif
  }
  if (PV) {  // OP_PREDVAR runs only in the k_gemm_pv instance
#pragma unroll
    for (int b = 0; b < QN; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        double v = 0.0;
#pragma unroll
        for (int a = 0; a < QM; ++a) v = fma(acc[a][b][q], acc[a][b][q], v);
        // the 16 lanes' sum by DPP (round 5: was four ds_bpermute exchanges per 32-bit half); the
        // same partners and operand order as the xor-1/2/4/8 tree, so the same sums
        v = row_sum16(v);
        if (lr == 0) db.var_part[((size_t)slot * db.nt + ti) * db.Mpad + tj * TS + 16 * b + lk + 4 * q] = v;
      }
    return;
  }
  double* Cm;
  switch (op) {
    case OP_TRSM: Cm = db.Lw + so; break;
    case OP_SYRK: Cm = db.S + so; break;
    case OP_TT: Cm = db.Lw + so; break;
    default: Cm = db.Linv + so; break;
  }
  // SYRK: C - L L^T = -acc; LINV21: L^-1_21 = -acc.  The sign flips the sign bit (an integer op:
  // an fp64 multiply by -1 takes issue cycles from the MFMA pipe of the SIMD's other wave)
  if (op == OP_SYRK || op == OP_LINV21) {  // wave-uniform
#pragma unroll
    for (int a = 0; a < QM; ++a)
#pragma unroll
      for (int b = 0; b < QN; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[a][b][q] = neg_f64(acc[a][b][q]);
  }
  const __amdgpu_buffer_rsrc_t crw = buffer_rsrc(Cm + (size_t)(tj * TS) * ld + ti * TS, 0x7ffffff0);
#pragma unroll
  for (int a = 0; a < QM; ++a)
#pragma unroll
    for (int b = 0; b < QN; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) buffer_store_f64(crw, vl + 128 * a, (16 * b + 4 * q) * Lb, acc[a][b][q]);
  if (op == OP_LINV21) zp_acc4(db, slot, ti, tj, acc, 1.0);
  if (op != OP_LINV21) GTS(g, pass, 3);
  if (op == OP_LINV21) {  // Mt[tj, ti] = Linv[ti, tj]^T, transposed through LDS 32 rows at a time
    // (round 5: two rounds instead of four 16-row ones, and 16-B reads and stores: every store
    // instruction writes two contiguous 512-B column segments of Mt)
    extern __shared__ __attribute__((aligned(16))) double gsm[];
    // this wave's [32][66] buffer: at row stride 66 the 16 x 4 lanes of a write hit 64 distinct
    // banks per half-wave (stride 65 put lanes with equal lr + lk in one bank); 528-B rows keep the
    // 16-B reads aligned
    double* tb = gsm + (threadIdx.x >> 6) * (32 * TT_S);
    double* Mtt = db.Mt + so + (size_t)(ti * TS) * ld + tj * TS;
    const int hr = l >> 5, c2 = 2 * (l & 31);  // 16-B lane: row parity, column pair
    const int vst = (hr * (int)ld + c2) * (int)sizeof(double);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int aa = 0; aa < 2; ++aa)
#pragma unroll
        for (int b = 0; b < QN; ++b)
#pragma unroll
          for (int q = 0; q < 4; ++q) tb[(16 * aa + lr) * TT_S + 16 * b + lk + 4 * q] = acc[2 * h + aa][b][q];
      __builtin_amdgcn_wave_barrier();
      // all 16 reads in flight before the stores (one LDS round trip per round, not one per row
      // pair); rows 32h + 2 r2 .. + 1: the pair's base in the resource (SGPRs), the lane's row
      // parity and column pair in the VGPR offset (soffset 0: see buffer_store_f64x2)
      double2 v[16];
#pragma unroll
      for (int r2 = 0; r2 < 16; ++r2) v[r2] = *(const double2*)(tb + (2 * r2 + hr) * TT_S + c2);
#pragma unroll
      for (int r2 = 0; r2 < 16; ++r2)
        buffer_store_f64x2(buffer_rsrc(Mtt + (size_t)(32 * h + 2 * r2) * ld, 0x7ffffff0), vst, v[r2].x, v[r2].y);
      __builtin_amdgcn_wave_barrier();
    }
    GTS(g, pass, 3);
  }
}

// The SYRK + TT launch of an 8-tile node (m1 = m2 = 4 tiles): 10 SYRK tiles of K = 4 tiles and 16 TT
// tiles of K = 4 - i (row i), 80 tile-K in all.  The unit decomposition below gives 5 workgroups
// per slot (1200 at B = 240: 2.34 rounds of 512 resident workgroups, i.e. three); this fixed plan
// packs them into 2 workgroups per slot (one round), every wave a list of 3-4 tiles.  Round 6: the
// lists balance issued MFMAs, not tile-K (a diagonal SYRK tile forms 10 of its 16 blocks, a TT
// tile skips 96 of its first K tile's 256 MFMAs): 2112-2240 MFMAs per wave, and 4352 on each SIMD,
// whose two waves are w and w + 4 in k_node8 (scratch/hwid_probe.hip); the round-5 lists had
// 1984-2464 per wave and 4064-4640 per SIMD, and k_node8's SYRK + TT phase ended 45 us apart on a
// slot's waves (scratch/node8_gts.py).  Entry: sel * 16 + 4 i + j, tile (i, j) of the SYRK (sel 0)
// or TT (sel 1) rectangle, each list longest first.
__constant__ int N8_PLAN[8][4] = {{13, 18, 30, -1}, {17, 20, 0, -1},  {8, 10, 24, 28}, {19, 22, 15, -1},
                                   {9, 5, 27, 31},   {14, 21, 26, -1}, {12, 23, 25, -1}, {4, 16, 29, -1}};
__host__ __device__ inline bool n8_plan(const GemmGeom& g1, const GemmGeom& g2) {
  return g1.op == OP_SYRK && g2.op == OP_TT && g1.n == 8 && g1.h == 4;
}
// units per slot of a launch (g2: the appended op; the n = 8 SYRK + TT launch: its fixed plan)
template <bool PV>
__device__ __forceinline__ int gemm_units(const DevBatch& db, const GemmGeom& g1, const GemmGeom& g2, int& T1) {
  const bool plan = !PV && n8_plan(g1, g2);
  T1 = plan ? 2 : op_units(g1, db.nt, db.mt);
  return T1 + ((plan || g2.op == OP_NONE) ? 0 : op_units(g2, db.nt, db.mt));
}
// unit u of a slot on the four waves w = 0..3 that share it
template <bool PV, int PM = PLAIN, bool BUF = true>
__device__ __forceinline__ void gemm_unit(const DevBatch& db, const GemmGeom& g1, const GemmGeom& g2, int slot, int u, int w,
                                          int T1) {
  int r0, c0, R, C, r02, c02, R2, C2;
  bool tri, tri2;
  op_rect(g1, db.nt, db.mt, r0, c0, R, C, tri);
  op_rect(g2, db.nt, db.mt, r02, c02, R2, C2, tri2);
  const bool plan = !PV && n8_plan(g1, g2);
  int pr, pc;
  // the wave's tiles: the plan's list, or the unit (and its folded mirror) of the decomposition
  // below; ONE call site of gemm_tile (its cores are inlined once per kernel instance)
  int np = 1, pr2 = 0, pc2 = 0, sel0 = 0, w8 = 0, wr = 0, wc = 0;
  if (plan) {
    w8 = 4 * u + w;
    np = 4;
  } else {
    if (u >= T1) {
      u -= T1;
      sel0 = 1;
      r0 = r02; c0 = c02; R = R2; C = C2; tri = tri2;
    }
    const int op = (sel0 ? g2 : g1).op;  // block-uniform
    int UR, UC;
    unit_shape(op, UR, UC);
    wr = w / UC;
    wc = w - wr * UC;
    if (tri) {  // lower-triangle tile 4u + w in row-major order
      const int t = 4 * u + w;
      if (t >= R * (R + 1) / 2) return;  // wave-uniform: the last unit's missing tiles
      quad_tri(t, pr, pc);
      wr = wc = 0;
    } else {
      const int RU = (R + UR - 1) / UR, CU = (C + UC - 1) / UC;
      if (op == OP_SYRK) {
        pr = UR * (u / CU);
        pc = UC * (u % CU);
      } else if (op == OP_TRSM) {  // K grows with the column: fold columns
        const int nf = (CU + 1) / 2, pi = u / nf, f = u - pi * nf;
        pr = pr2 = UR * pi;
        pc = UC * (CU - 1 - f);
        pc2 = UC * f;
        np = (CU - 1 - f != f) ? 2 : 1;
      } else {  // fold rows; TT: K shrinks with the row, LINV21 / PREDVAR: K grows with the row
        const int f = u / CU, pj = u - f * CU;
        const int lo = f, hi = RU - 1 - f;
        pr = UR * (op == OP_TT ? lo : hi);
        pr2 = UR * (op == OP_TT ? hi : lo);
        pc = pc2 = UC * pj;
        np = (lo != hi) ? 2 : 1;
      }
    }
  }
  // the register stage handed from tile k to tile k + 1 (mma_64x64_pm), in the SYRK + TT instance:
  // syrk_tt 9.97-10.04 -> 9.84-9.90 ms; TRSM 4.93-4.97 -> 5.03-5.09 and LINV21 unchanged (same-box
  // A/B, scratch/gemm_ab.sh), so those keep the reload
  Frag4 f0;
  bool pre = false;  // f0 holds this tile's first stage
#pragma unroll 1
  for (int k = 0; k < np; ++k) {
    int sel, ti, tj;
    bool nxt = false;  // the next tile of the fold exists on this wave: prefetch its first stage
    int nti = 0, ntj = 0;
    if (plan) {
      const int e = N8_PLAN[w8][k];
      if (e < 0) break;
      sel = e >> 4;
      ti = (sel ? r02 : r0) + ((e >> 2) & 3);
      tj = (sel ? c02 : c0) + (e & 3);
    } else {
      const int ur = k ? pr2 : pr, uc = k ? pc2 : pc;
      if (ur + wr >= R || uc + wc >= C) continue;  // wave-uniform: partial unit
      sel = sel0;
      ti = r0 + ur + wr;
      tj = c0 + uc + wc;
      if (!PV && BUF && PM == TRI_A_FIRST && k + 1 < np && pr2 + wr < R && pc2 + wc < C) {  // TT's folds (see below)
        nxt = true;
        nti = r0 + pr2 + wr;
        ntj = c0 + pc2 + wc;
      }
    }
    // wave-uniform tile indices in SGPRs (the 64 x 64 core needs every VGPR)
    gemm_tile<PV, PM, BUF>(db, sel ? g2 : g1, slot, __builtin_amdgcn_readfirstlane(ti), __builtin_amdgcn_readfirstlane(tj), k, f0,
                           pre, nxt, __builtin_amdgcn_readfirstlane(nti), __builtin_amdgcn_readfirstlane(ntj));
    pre = nxt;
  }
}

template <bool PV, int PM = PLAIN>
__device__ __forceinline__ void gemm_body(const DevBatch& db, const GemmGeom& g1, const GemmGeom& g2) {
  int T1;
  const int T = gemm_units<PV>(db, g1, g2, T1);
  int slot, u;
  if (!map_slot(db, T, slot, u)) return;
  gemm_unit<PV, PM>(db, g1, g2, slot, u, __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), T1);
}

// 64 x 32 accumulator half-tile (mma_64x32 layout, columns 32 half ..) of sgn * L^-1[ti,tj]
__device__ __forceinline__ void zp_acc2(const DevBatch& db, int slot, int ti, int tj, int half, const d4 (&acc)[WM][WN],
                                        double sgn) {
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const double* y = db.Y + (size_t)slot * db.Npad + tj * TS + 32 * half;
  double yv[WN][4];
#pragma unroll
  for (int b = 0; b < WN; ++b)
#pragma unroll
    for (int q = 0; q < 4; ++q) yv[b][q] = y[16 * b + lk + 4 * q];
  double* z = zp_row(db, slot, 2 * tj + half) + ti * TS;
#pragma unroll
  for (int a = 0; a < WM; ++a) {
    double t = 0.0;
#pragma unroll
    for (int b = 0; b < WN; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) t = fma(acc[a][b][q], yv[b][q], t);
    t = sum_xor32(sum_xor16(t));
    if (lk == 0) z[16 * a + lr] = sgn * t;
  }
}
// Small recursion nodes: unit = 2 vertically adjacent 64 x 64 tiles, wave = 64 x 32, single-stage
// core at 4 waves/SIMD (more, shorter units than the 2 x 2 form: better for K <= 512).
__device__ __forceinline__ void gemm_tile_pair(const DevBatch& db, const GemmGeom& g, int slot, int ti, int tj, int wc);
// units: tri (SYRK) as pair_unit; TRSM folds column c with C-1-c; TT / LINV21 / PREDVAR fold
// row pair p with P-1-p (the folding of gemm_body, for 2 x 1 units)
__host__ __device__ inline int pair_op_units(const GemmGeom& g, int nt, int mt) {
  int r0, c0, R, C;
  bool tri;
  op_rect(g, nt, mt, r0, c0, R, C, tri);
  if (tri || g.op == OP_SYRK) return pair_units(R, C, tri);
  const int P = (R + 1) / 2;
  return g.op == OP_TRSM ? P * ((C + 1) / 2) : ((P + 1) / 2) * C;
}
__device__ __forceinline__ void gemm_body_pair(const DevBatch& db, const GemmGeom& g1, const GemmGeom& g2) {
  int r0, c0, R, C, r02, c02, R2, C2;
  bool tri, tri2;
  op_rect(g1, db.nt, db.mt, r0, c0, R, C, tri);
  op_rect(g2, db.nt, db.mt, r02, c02, R2, C2, tri2);
  const int T1 = pair_op_units(g1, db.nt, db.mt), T2 = g2.op == OP_NONE ? 0 : pair_op_units(g2, db.nt, db.mt);
  int slot, u, pr, pc;
  if (!map_slot(db, T1 + T2, slot, u)) return;
  const GemmGeom g = u < T1 ? g1 : g2;  // block-uniform
  if (u >= T1) {
    u -= T1;
    r0 = r02; c0 = c02; R = R2; C = C2; tri = tri2;
  }
  const int op = g.op;
  int np = 1, pr2 = 0, pc2 = 0;
  if (tri) {
    pair_unit(u, R, C, tri, pr, pc);
  } else if (op == OP_SYRK) {
    const int P = (R + 1) / 2, pi = u / C;
    pr = 2 * (P - 1 - pi);
    pc = u - pi * C;
  } else if (op == OP_TRSM) {  // K grows with the column: fold columns
    const int nf = (C + 1) / 2, pi = u / nf, f = u - pi * nf;
    pr = pr2 = 2 * pi;
    pc = C - 1 - f;
    pc2 = f;
    np = (pc != pc2) ? 2 : 1;
  } else {  // fold row pairs; TT: K shrinks with the row, LINV21 / PREDVAR: K grows with the row
    const int P = (R + 1) / 2, f = u / C;
    pc = pc2 = u - f * C;
    const int lo = f, hi = P - 1 - f;
    pr = 2 * (op == OP_TT ? lo : hi);
    pr2 = 2 * (op == OP_TT ? hi : lo);
    np = (lo != hi) ? 2 : 1;
  }
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), wr = w >> 1, wc = w & 1;
#pragma unroll 1
  for (int pass = 0; pass < np; ++pass) {
    const int ur = pass ? pr2 : pr, uc = pass ? pc2 : pc;
    if (ur + wr >= R) continue;  // wave-uniform: second tile of an odd pair
    gemm_tile_pair(db, g, slot, __builtin_amdgcn_readfirstlane(r0 + ur + wr), __builtin_amdgcn_readfirstlane(c0 + uc), wc);
  }
}
__device__ __forceinline__ void gemm_tile_pair(const DevBatch& db, const GemmGeom& g, int slot, int ti, int tj, int wc) {
  const int op = g.op;
  const size_t ld = db.ld, so = (size_t)slot * db.mat;
  int kb, ke;  // K range in tiles
  const double *A, *Bm;
  size_t ldb = ld;
  switch (op) {
    case OP_TRSM: kb = g.o; ke = tj + 1; A = (g.upd ? db.S : db.K) + so; Bm = db.Linv + so; break;
    case OP_SYRK: kb = g.o; ke = g.o + g.h; A = db.Lw + so; Bm = db.Lw + so; break;
    case OP_TT: kb = ti; ke = g.o + g.h; A = db.Mt + so; Bm = db.Lw + so; break;
    case OP_LINV21: kb = g.o + g.h; ke = ti + 1; A = db.Linv + so; Bm = db.Lw + so; break;
    default:
      kb = 0;
      ke = ti + 1;
      A = db.Linv + so;
      Bm = db.KsT + (size_t)slot * db.Npad * db.Mpad;
      ldb = db.Mpad;
      break;
  }
  d4 acc[WM][WN];
  acc_zero(acc);
  mma_64x32_s1(acc, A + (size_t)kb * TS * ld + ti * TS, ld, Bm + (size_t)kb * TS * ldb + tj * TS + 32 * wc, ldb,
           (ke - kb) * TS);
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  if (op == OP_PREDVAR) {
#pragma unroll
    for (int b = 0; b < WN; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        double v = 0.0;
#pragma unroll
        for (int a = 0; a < WM; ++a) v = fma(acc[a][b][q], acc[a][b][q], v);
        v = row_sum16(v);  // the xor-1/2/4/8 tree's partners and order, by DPP
        if (lr == 0)
          db.var_part[((size_t)slot * db.nt + ti) * db.Mpad + tj * TS + 32 * wc + 16 * b + lk + 4 * q] = v;
      }
    return;
  }
  double* Cm;
  double sgn = 1.0;
  switch (op) {
    case OP_TRSM: Cm = db.Lw + so; break;
    case OP_SYRK: Cm = db.S + so; break;
    case OP_TT: Cm = db.Lw + so; break;
    default: Cm = db.Linv + so; sgn = -1.0; break;
  }
  const size_t co = (size_t)(tj * TS + 32 * wc) * ld + ti * TS;
  double* Ct = Cm + co;
  if (op == OP_SYRK) {  // C (from K, or S once updated) - L L^T into S
    const double* Cs = (g.upd ? db.S : db.K) + so + co;
#pragma unroll
    for (int a = 0; a < WM; ++a)
#pragma unroll
      for (int b = 0; b < WN; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const size_t e = (size_t)(16 * b + lk + 4 * q) * ld + 16 * a + lr;
          Ct[e] = Cs[e] - acc[a][b][q];
        }
  } else {
#pragma unroll
    for (int a = 0; a < WM; ++a)
#pragma unroll
      for (int b = 0; b < WN; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) Ct[(size_t)(16 * b + lk + 4 * q) * ld + 16 * a + lr] = sgn * acc[a][b][q];
  }
  if (op == OP_LINV21) zp_acc2(db, slot, ti, tj, wc, acc, -1.0);
  if (op == OP_LINV21) {  // Mt[tj, ti] = Linv[ti, tj]^T (direct: an LDS transpose measured slower here)
    double* Mtt = db.Mt + so + (size_t)(ti * TS) * ld + tj * TS + 32 * wc;
#pragma unroll
    for (int a = 0; a < WM; ++a)
#pragma unroll
      for (int b = 0; b < WN; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) Mtt[(size_t)(16 * a + lr) * ld + 16 * b + lk + 4 * q] = -acc[a][b][q];
  }
}

__global__ __launch_bounds__(NTHR) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_gemm_p(DevBatch db, GemmGeom g, GemmGeom g2) {
  gemm_body_pair(db, g, g2);
}
// PM: the op whose triangular operand tile the instance peels (TRI_A_FIRST: TT of the SYRK + TT
// launches; REV_B: TRSM; REV_A: LINV21)
template <int PM>
__global__ __launch_bounds__(NTHR) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_gemm(DevBatch db, GemmGeom g, GemmGeom g2) {
  gemm_body<false, PM>(db, g, g2);
}
__global__ __launch_bounds__(NTHR) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_gemm_pv(DevBatch db, GemmGeom g, GemmGeom g2) {
  gemm_body<true>(db, g, g2);
}

// ============================================================================================
// Fused leaf node: Cholesky + inverse of the n <= 4 diagonal tiles o..o+n-1 (a 256x256 block at
// most) in ONE workgroup per slot, replacing ~4n latency-bound launches of the recursion.
//   for k: diag(o+k); Lw[i,k] = K[i,k] Linv[k,k]^T (i > k); K[i,j] -= Lw[i,k] Lw[j,k]^T (i >= j > k)
//   then the off-diagonal inverse tiles by sub-diagonal s = i - j:
//     X = sum_{t=j}^{i-1} L[i,t] Linv[t,j]  (per wave quarter, in LDS),  Linv[i,j] = -Linv[i,i] X
// Each 64x64 tile task is split into four 64x16 column quarters, one per wave.  The X of a task is
// only re-read by the wave that computed it (its own 16 columns, kept in the wave's LDS buffer), so
// a wave-level barrier replaces a workgroup barrier between the two products.
// ============================================================================================
// 64 x 16 column-quarter stores (C layout of mma_64x16, quarter columns 16w..): C[r + c ld] =
// sgn acc, C -= acc, and the transposed Ct[c + r ld] through the wave's [16][65] LDS buffer (four
// 128-B row segments per store instruction)
__device__ __forceinline__ void accq_store(double* C, size_t ld, const d4 (&acc)[QM], double sgn) {
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
#pragma unroll
  for (int a = 0; a < QM; ++a)
#pragma unroll
    for (int q = 0; q < 4; ++q) C[(size_t)(lk + 4 * q) * ld + 16 * a + lr] = sgn * acc[a][q];
}
__device__ __forceinline__ void accq_store_t(double* Ct, size_t ld, const d4 (&acc)[QM], double sgn, double* tb) {
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
#pragma unroll
  for (int a = 0; a < QM; ++a)
#pragma unroll
    for (int q = 0; q < 4; ++q) tb[(lk + 4 * q) * (TS + 1) + 16 * a + lr] = sgn * acc[a][q];  // tb[c][r]
  __builtin_amdgcn_wave_barrier();
  const int c = l & 15, r4 = l >> 4;
#pragma unroll
  for (int r = 0; r < TS; r += 4) Ct[(size_t)(r + r4) * ld + c] = tb[c * (TS + 1) + r + r4];
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ void leaf_body(const DevBatch& db, int o, int n, int upd) {
  // every 64 x 64 tile task is split into four 64 x 16 column quarters, one per wave (wave w:
  // columns 16w..16w+15 of every tile of a step), so a step with fewer tiles than waves keeps
  // all four SIMDs busy; quarter-transposed stores through the wave's LDS buffer
  __shared__ double tbs[4 * 16 * (TS + 1)];
  __shared__ double zq[6][4][TS];  // n <= 4: z partials of the off-diagonal L^-1 quarters [tile][wave][row]
  __shared__ double dT[TS * FS], dXi[TS * FS];  // the diagonal routine's tile and inverse images
  __shared__ __attribute__((aligned(16))) double dcb[256];
  const int slot = blockIdx.x;
  if (!slot_active(db, slot)) return;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), cq = 16 * w;
  double* tb = tbs + w * 16 * (TS + 1);
  const size_t ld = db.ld, so = (size_t)slot * db.mat;
  // the leaf's tiles: from K (or S, upd) in step 0; every later step reads what this leaf's own
  // SYRK wrote to S
  double* S = db.S + so;
  const double* K0 = (upd ? db.S : db.K) + so;
  double* Lw = db.Lw + so;
  double* Li = db.Linv + so;
  double* Mt = db.Mt + so;
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  LEAF_TS(0);
  for (int k = 0; k < n; ++k) {
    const int tk = o + k, m = n - 1 - k;
    const double* xi = dXi;  // Linv[tk,tk] in LDS, read by the TRSM tasks below
    const double* K = k > 0 ? S : K0;
    diag_tile_fast(db, slot, tk, dT, dXi, dcb, k > 0, upd ? db.S : db.K, false);  // k > 0: the SYRK below left the tile in dT
    __syncthreads();
    LEAF_TS(1 + 3 * k);
    for (int t = 0; t < m; ++t) {  // TRSM: L[ti,tk] = K[ti,tk] Linv[tk,tk]^T
      const int ti = tk + 1 + t;
      d4 acc[QM];
#pragma unroll
      for (int a = 0; a < QM; ++a) acc[a] = (d4){0.0, 0.0, 0.0, 0.0};
      mma_64x16(acc, K + (size_t)tk * TS * ld + ti * TS, ld, xi + cq, FS, TS);
      accq_store(Lw + (size_t)(tk * TS + cq) * ld + ti * TS, ld, acc, 1.0);
    }
    diag_store(db, slot, tk, dXi, dcb);  // after the TRSM loads (dXi stays until the next diagonal)
    __syncthreads();
    LEAF_TS(2 + 3 * k);
    for (int c = 0; c < m; ++c)  // SYRK (lower trailing tiles)
      for (int a0 = 0; a0 < m - c; ++a0) {
        const int tj = tk + 1 + c, ti = tj + a0;
        const double* Cs = K + (size_t)(tj * TS + cq) * ld + ti * TS;
        double* Ct = S + (size_t)(tj * TS + cq) * ld + ti * TS;
        d4 acc[QM];  // -C - L L^T, stored negated
#pragma unroll
        for (int a = 0; a < QM; ++a)
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[a][q] = -Cs[(size_t)(lk + 4 * q) * ld + 16 * a + lr];
        mma_64x16(acc, Lw + (size_t)tk * TS * ld + ti * TS, ld, Lw + (size_t)tk * TS * ld + tj * TS + cq, ld, TS);
        if (c == 0 && a0 == 0) {  // the next diagonal tile: straight into the diagonal routine's LDS
#pragma unroll
          for (int a = 0; a < QM; ++a)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int r = 16 * a + lr, cc = cq + lk + 4 * q;
              dT[cc * FS + r] = r >= cc ? -acc[a][q] : 0.0;
            }
        } else {
          accq_store(Ct, ld, acc, -1.0);
        }
      }
    __syncthreads();
    LEAF_TS(3 + 3 * k);
  }
  // off-diagonal inverse tiles by sub-diagonal s:  X = sum_{k=tj}^{ti-1} L[ti,k] Linv[k,tj] (kept
  // transposed in the wave's LDS buffer), Linv[ti,tj] = -Linv[ti,ti] X.  Wave w's quarter of
  // Linv[ti,tj] needs only its own quarter of X: no barrier between the two products.
  int kz = 0;  // off-diagonal tile index in (s, t) order
  for (int s = 1; s < n; ++s) {
    for (int t = 0; t < n - s; ++t, ++kz) {
      const int tj = o + t, ti = tj + s;
      double* Xt = Mt + (size_t)(ti * TS) * ld + tj * TS;  // Mt[tj,ti]
      d4 acc[QM];
#pragma unroll
      for (int a = 0; a < QM; ++a) acc[a] = (d4){0.0, 0.0, 0.0, 0.0};
      mma_64x16(acc, Lw + (size_t)tj * TS * ld + ti * TS, ld, Mt + (size_t)tj * TS * ld + tj * TS + cq, ld, s * TS);
      // this wave's quarter of X stays in its LDS buffer, transposed (tb[c][r] = X[r][cq + c]):
      // the second product reads it from there instead of a global round trip
#pragma unroll
      for (int a = 0; a < QM; ++a)
#pragma unroll
        for (int q = 0; q < 4; ++q) tb[(lk + 4 * q) * (TS + 1) + 16 * a + lr] = acc[a][q];
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int a = 0; a < QM; ++a) acc[a] = (d4){0.0, 0.0, 0.0, 0.0};
      mma_64x16_ldsb(acc, Li + (size_t)ti * TS * ld + ti * TS, ld, tb);
      __builtin_amdgcn_wave_barrier();  // the reads of X precede accq_store_t's writes to tb
      if (n <= 4) {  // this quarter's z partial, from the registers: sum_c Linv[r][cq + c] y[cq + c]
        const double* yq = db.Y + (size_t)slot * db.Npad + tj * TS + cq;
        double yv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) yv[q] = yq[lk + 4 * q];
#pragma unroll
        for (int a = 0; a < QM; ++a) {
          double zt = 0.0;
#pragma unroll
          for (int q = 0; q < 4; ++q) zt = fma(-acc[a][q], yv[q], zt);
          zt = sum_xor32(sum_xor16(zt));
          if (lk == 0) zq[kz][w][16 * a + lr] = zt;
        }
      }
      accq_store(Li + (size_t)(tj * TS + cq) * ld + ti * TS, ld, acc, -1.0);
      accq_store_t(Xt + cq, ld, acc, -1.0, tb);
    }
    __syncthreads();
    LEAF_TS(12 + s);
  }
  // z partials of the off-diagonal L^-1 tiles of this leaf (the diagonal tiles' come from
  // diag_tile_fast).  n <= 4: the four quarters' partials from zq, summed in wave order.
  if (n <= 4) {
    const int r = threadIdx.x & 63;
    for (int k = threadIdx.x >> 6; k < n * (n - 1) / 2; k += 4) {
      int s = 1, t = k;
      while (t >= n - s) {
        t -= n - s;
        ++s;
      }
      const int tj = o + t, ti = tj + s;
      zp_row(db, slot, 2 * tj)[ti * TS + r] = ((zq[k][0][r] + zq[k][1][r]) + zq[k][2][r]) + zq[k][3][r];
      zp_row(db, slot, 2 * tj + 1)[ti * TS + r] = 0.0;
    }
    LEAF_TS(16);
    return;
  }
  // larger leaves: read the tiles back from L2 (this workgroup wrote them); 16 tiles per round
  // (the [4][16][65] buffer)
  __threadfence_block();
  {
    const int r = threadIdx.x & 63, qc = threadIdx.x >> 6;  // 4 quarters of 16 columns
    const int nod = n * (n - 1) / 2;
    for (int k0 = 0; k0 < nod; k0 += 16) {
      int k = 0;
      for (int s = 1; s < n; ++s)
        for (int t = 0; t < n - s; ++t, ++k) {
          if (k < k0 || k >= k0 + 16) continue;
          const int tj = o + t, ti = tj + s;
          const double* Lt = Li + (size_t)(tj * TS) * ld + ti * TS;
          const double* y = db.Y + (size_t)slot * db.Npad + tj * TS;
          double acc = 0.0;
#pragma unroll
          for (int c = 16 * qc; c < 16 * qc + 16; ++c) acc = fma(Lt[(size_t)c * ld + r], y[c], acc);
          tbs[(4 * (k - k0) + qc) * TS + r] = acc;
        }
      __syncthreads();
      k = 0;
      for (int s = 1; s < n; ++s)
        for (int t = 0; t < n - s; ++t, ++k)
          if (qc == 0 && k >= k0 && k < k0 + 16) {
            const int tj = o + t, ti = tj + s;
            const double* pk = tbs + 4 * (k - k0) * TS;
            zp_row(db, slot, 2 * tj)[ti * TS + r] = ((pk[r] + pk[TS + r]) + pk[2 * TS + r]) + pk[3 * TS + r];
            zp_row(db, slot, 2 * tj + 1)[ti * TS + r] = 0.0;
          }
      __syncthreads();
    }
  }
}

__global__ __launch_bounds__(NTHR) void k_leaf(DevBatch db, int o, int n, int upd) { leaf_body(db, o, n, upd); }
// ============================================================================================
// Workgroup-local hand-offs of the fused leaf (k_leaf9): progress words and counter barriers in
// LDS, polled by the waiting waves.  Every wait is bounded (2^24 polls, about half a second): a
// hand-off that never comes ends the kernel with status GPRX_DEVICE_ERROR (3) for the slot instead
// of a hung launch.
// ============================================================================================
__device__ __forceinline__ int lds_load(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void l9_release() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup"); }
__device__ __forceinline__ void l9_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup"); }
__device__ __forceinline__ void lds_publish(int* p, int v) {
  // the writer's LDS and global stores are complete before the word changes
  l9_release();
  if ((threadIdx.x & 63) == 0) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
constexpr int LW_SPIN = 1 << 24;
__device__ __forceinline__ void lw_timeout(const DevBatch& db, int slot) {
  if ((threadIdx.x & 63) == 0) db.status[slot] = 3;
}
__device__ __forceinline__ void lds_wait_gt(const int* p, int v, const DevBatch& db, int slot) {
  for (int it = 0; lds_load(p) <= v; ++it) {
    if (it > LW_SPIN) {
      lw_timeout(db, slot);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  l9_acquire();
}
// ---- k_leaf9's diagonal wave: the diagonal routine of diag_tile_fast on one wave.  The 16 x 16
// factor+inverse is an unscaled elimination (no square root inside the 16-step loop: the columns
// are scaled by 1/sqrt(p_j) once at the end) with v_fmac_f64 taking the DPP row broadcast
// directly, one instruction per update instead of a 64-bit broadcast move and an fma.  A single
// wave issues one VALU instruction per ~4.5 cycles here, so the instruction count sets the time
// (scratch/factbench: 4346 -> about 3500 cycles per 16 x 16 block).  The TRSM, SYRK and inverse
// blocks of a panel are issued as one batch (all operand reads, then the MFMA chains interleaved,
// then the stores) instead of block after block.  The inverse image's upper blocks are never
// written (no reader touches them), and the tile's diagonal goes to ldiag[64] for the
// log-determinant, which a task wave sums.
// LDS writes of this wave complete and visible to its later reads (the compiler keeps the order)
__device__ __forceinline__ void wave_sync() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}
template <int M>
__device__ __forceinline__ void fmac_bcast(double& acc, double src, double f) {
  // acc += src[lane M of this row] * f.  A VALU write followed by a DPP read of the same register
  // needs two wait states, which the compiler does not insert around inline assembly.  The only
  // DPP source is a step's pivot column u[.][j], last written by the previous step's update for
  // m = j; volatile keeps the updates in program order, so at least three updates (its X partner
  // and the m = j+1 pair) separate that write from the first read.
  asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(src), "v"(f), "i"(M));
}
template <int J, int M>
__device__ __forceinline__ void fact_updates(double (&a)[16], double (&y)[16], double au, double fa, double fy) {
  if constexpr (M < 16) {
    fmac_bcast<M>(a[M], au, fa);  // a[m] -= u[m][j] u[i][j] / p_j   (fa = -u[i][j] / p_j)
    fmac_bcast<M>(y[M], au, fy);  // W^-1[m][i] -= (u[m][j] / p_j) W^-1[j][i]   (fy = -W^-1[j][i] / p_j)
    fact_updates<J, M + 1>(a, y, au, fa, fy);
  }
}
template <int J>
__device__ __forceinline__ double row_bcast_c(double v) { return __builtin_amdgcn_mov_dpp(v, 0x150 + J, 0xF, 0xF, true); }
// Step J of the unscaled elimination A = U D^-1 U^T (U = L D^1/2, D = diag(p)): lane i holds row i
// of U (a) and column i of W^-1 (y; W = U D^-1 unit lower) and d = its running diagonal, so the
// next pivot is one DPP broadcast away and the step's critical path is the reciprocal of p_J (no
// square root: the columns are scaled by 1/sqrt(p_J) once, after the last step).
template <int J>
__device__ __forceinline__ void fact_step(double (&a)[16], double (&y)[16], double& d, double& pv, int lr, int& fl) {
  if constexpr (J < 16) {
    const double au = a[J], yu = y[J];
    const double p = row_bcast_c<J>(d);
    const double pk = (p > 0.0) ? p : 1.0;
    fl = (fl < 0 && !(p > 0.0)) ? J : fl;  // the first pivot <= 0 or NaN (continue with 1)
    pv = (lr == J) ? pk : pv;
    const double r0 = __builtin_amdgcn_rcp(pk);
    const double e = fma(-pk, r0, 1.0);
    const double ip = fma(r0, fma(e, e, e), r0);  // 1/p to the rounding level (error e^3)
    d = fma(-au * au, ip, d);
    fact_updates<J, J + 1>(a, y, au, -au * ip, -yu * ip);
    fact_step<J + 1>(a, y, d, pv, lr, fl);
  }
}
template <int J>
__device__ __forceinline__ void fact_scale(double (&a)[16], double (&y)[16], double rl, double sl, int lr) {
  if constexpr (J < 16) {
    const double rJ = row_bcast_c<J>(rl);  // 1/sqrt(p_J)
    a[J] = (lr > J) ? a[J] * rJ : (lr == J ? sl : 0.0);
    y[J] = y[J] * rJ;
    fact_scale<J + 1>(a, y, rl, sl, lr);
  }
}
template <int P>
__device__ __forceinline__ void w1_panel(double* T, const double* Xi, int lr, int lk) {
  constexpr int NT = 3 - P;  // trailing blocks
  if constexpr (NT > 0) {
    constexpr int c0 = 16 * P;
    // TRSM: A_iP <- A_iP Dinv^T, i = P+1 .. 3
    double bv[4], av[NT][4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bv[s] = Xi[(c0 + 4 * s + lk) * FS + c0 + lr];
#pragma unroll
      for (int i = 0; i < NT; ++i) av[i][s] = T[(c0 + 4 * s + lk) * FS + 16 * (P + 1 + i) + lr];
    }
    d4 acc[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) acc[i] = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < NT; ++i) acc[i] = mfma(av[i][s], bv[s], acc[i]);
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) T[(c0 + lr) * FS + 16 * (P + 1 + i) + lk + 4 * q] = acc[i][q];
    wave_sync();
    // SYRK: A_ij -= A_iP A_jP^T for P < j <= i < 4
    double pv[NT][4];
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int s = 0; s < 4; ++s) pv[i][s] = T[(c0 + 4 * s + lk) * FS + 16 * (P + 1 + i) + lr];
    constexpr int NB = NT * (NT + 1) / 2;
    d4 sacc[NB], old[NB];
#pragma unroll
    for (int b = 0, j = 0; j < NT; ++j)
#pragma unroll
      for (int i = j; i < NT; ++i, ++b) {
#pragma unroll
        for (int q = 0; q < 4; ++q) old[b][q] = T[(16 * (P + 1 + j) + lr) * FS + 16 * (P + 1 + i) + lk + 4 * q];
        sacc[b] = (d4){0.0, 0.0, 0.0, 0.0};
      }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int b = 0, j = 0; j < NT; ++j)
#pragma unroll
        for (int i = j; i < NT; ++i, ++b) sacc[b] = mfma(pv[i][s], pv[j][s], sacc[b]);
#pragma unroll
    for (int b = 0, j = 0; j < NT; ++j)
#pragma unroll
      for (int i = j; i < NT; ++i, ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) T[(16 * (P + 1 + j) + lr) * FS + 16 * (P + 1 + i) + lk + 4 * q] = old[b][q] - sacc[b][q];
    wave_sync();
  }
}
// off-diagonal inverse blocks of sub-diagonal SD: X_ij = -Dinv_i sum_{k=j}^{i-1} L_ik X_kj, j = 0 .. 3-SD
template <int SD>
__device__ __forceinline__ void w1_inverse(const double* T, double* Xi, int lr, int lk) {
  constexpr int NJ = 4 - SD;
  d4 y[NJ], x[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) y[j] = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int kk = 0; kk < SD; ++kk) {
    double av[NJ][4], bv[NJ][4];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int i = j + SD, kb = j + kk;
        av[j][s] = T[(16 * kb + 4 * s + lk) * FS + 16 * i + lr];   // L_ik[lr][k]
        bv[j][s] = Xi[(16 * j + lr) * FS + 16 * kb + 4 * s + lk];  // X_kj[k][lr]
      }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int j = 0; j < NJ; ++j) y[j] = mfma(av[j][s], bv[j][s], y[j]);
  }
  double dv[NJ][4];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int s = 0; s < 4; ++s) dv[j][s] = Xi[(16 * (j + SD) + 4 * s + lk) * FS + 16 * (j + SD) + lr];  // Dinv_i[lr][4s+lk]
#pragma unroll
  for (int j = 0; j < NJ; ++j) x[j] = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int j = 0; j < NJ; ++j) x[j] = mfma(dv[j][s], y[j][s], x[j]);
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) Xi[(16 * j + lr) * FS + 16 * (j + SD) + lk + 4 * q] = -x[j][q];
  wave_sync();
}
__device__ __forceinline__ void diag_w1(const DevBatch& db, int slot, int jt, double* T, double* Xi, double* ldiag) {
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  int fail = -1;
  D_TS1(0);
  for (int P = 0; P < 4; ++P) {
    const int c0 = 16 * P;
    double a[16], y[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      a[k] = T[(c0 + k) * FS + c0 + lr];
      y[k] = (k == lr) ? 1.0 : 0.0;
    }
    double d = T[(c0 + lr) * FS + c0 + lr], pv = 1.0;
    int fl = -1;
    fact_step<0>(a, y, d, pv, lr, fl);
    fl = __builtin_amdgcn_readfirstlane(fl);
    if (fail < 0 && fl >= 0) fail = c0 + fl;
    {
      double sl, rl;
      sqrt_rsqrt(pv, sl, rl);  // lane i: sqrt(p_i), 1/sqrt(p_i)
      fact_scale<0>(a, y, rl, sl, lr);
    }
    if (l < 16) {
#pragma unroll
      for (int k = 0; k < 16; ++k) T[(c0 + k) * FS + c0 + l] = (k <= l) ? a[k] : 0.0;  // row l of L_PP
      ldiag[c0 + l] = a[l];
    }
    __builtin_amdgcn_wave_barrier();
    if (l < 16) {
#pragma unroll
      for (int r = 0; r < 16; ++r) Xi[(c0 + l) * FS + c0 + r] = y[r];  // column l of Dinv
    }
    wave_sync();
    D_TS1(1 + 2 * P);
    switch (P) {
      case 0: w1_panel<0>(T, Xi, lr, lk); break;
      case 1: w1_panel<1>(T, Xi, lr, lk); break;
      case 2: w1_panel<2>(T, Xi, lr, lk); break;
      default: break;
    }
    D_TS1(2 + 2 * P);
  }
  w1_inverse<1>(T, Xi, lr, lk);
  w1_inverse<2>(T, Xi, lr, lk);
  w1_inverse<3>(T, Xi, lr, lk);
  D_TS1(9);
  if (fail >= 0 && l == 0 && db.status[slot] == 0) {
    db.status[slot] = 1;
    db.info[slot] = jt * TS + fail + 1;
  }
}

struct Leaf9Sync {
  int tk;          // task-wave barrier counter (monotonic, 7 per barrier)
  int ch;          // chain-wave barrier counter (4 per barrier)
  int diag_done;   // diagonal tiles factored and inverted
  int tile_ready;  // diagonal tiles handed to wave 0 (tile 0 at the start)
  int xfree;       // steps whose readers of dX[k & 1] are done
  int crit;        // critical SYRK items done (monotonic over the steps)
};
constexpr int L9_TW = 7;
// Items go round the task waves (L9_HW of them), the three off the chain first: 5, 6, 7, 1, 2, 3
// (round 6: L9_HW = 6), or 5, 6, 7, 1, 2, 3, 4 (L9_HW = 7, rounds 4-5).  Wave 4 is the diagonal
// wave's SIMD-mate (waves w and w + 4 of a workgroup share a SIMD, scratch/hwid_probe.hip), and the
// fp64 VALU of the diagonal routine shares that SIMD's one fp64 pipe with the mate's MFMAs: without
// items on wave 4 (it keeps its chain quarter, while wave 0 waits), node8 2.741 -> 2.723 ms per
// step at B = 240 and 2.998 -> 2.957 ms for CP at B = 1014 (same box, two pairs each; the same
// items, so bit-identical).
#ifndef GPRX_L9_HW
#define GPRX_L9_HW 6
#endif
constexpr int L9_HW = GPRX_L9_HW;
// Phase B (the SYRK items and the Y items of the next inverse row) runs while the diagonal wave
// waits for the next chain, so its round robin keeps wave 4 (L9_HWB = 7): otherwise its SIMD idles
// through phase B.
#ifndef GPRX_L9_HWB
#define GPRX_L9_HWB 7
#endif
constexpr int L9_HWB = GPRX_L9_HWB;
// position of task wave w in a round robin over nw task waves (-1: no items)
__device__ __forceinline__ int l9_pos(int w, int nw = L9_HW) { return w >= 5 ? w - 5 : (w <= 3 ? w + 2 : (nw == 7 ? 6 : -1)); }
// phase B of step k (m = n - 1 - k trailing tiles per edge): the SYRK tiles the next step needs,
// column k + 1 below the diagonal and the next diagonal tile, are its first nc tiles in the
// column-major enumeration that skips (k + 1, k + 1)
__host__ __device__ constexpr int l9_crit_tiles(int m) { return m <= 0 ? 0 : (m - 1) + (m >= 2 ? 1 : 0); }
__device__ __forceinline__ void lds_wait_ge(const int* p, int v, const DevBatch& db, int slot) {
  for (int it = 0; lds_load(p) < v; ++it) {
    if (it > LW_SPIN) {
      lw_timeout(db, slot);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  l9_acquire();
}
__device__ __forceinline__ void lds_count(int* p) {  // one more item done (its stores before the count)
  l9_release();
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(p, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// The diagonal tile's four store quarters go to waves 4..7 (L9_HW = 6: 1, 5, 6, 7).
__device__ __forceinline__ int l9_store_wave(int e) { return L9_HW == 7 || e > 0 ? 4 + e : 1; }
__device__ __forceinline__ int l9_wave_of(int e) {
  const int r = e % L9_HW;
  return r < 3 ? 5 + r : (r < 6 ? r - 2 : 4);
}
__device__ __forceinline__ void ctr_barrier(int* ctr, int& gen, int nw, const DevBatch& db, int slot) {
  gen += nw;
  l9_release();
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  for (int it = 0; lds_load(ctr) < gen; ++it) {
    if (it > LW_SPIN) {
      lw_timeout(db, slot);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  l9_acquire();
}
// acc[a] += sum_k Lx[16a + lk + 4q][k] b(k) for a triangular Lx (lower; LDS image Lx[c * FS + r]):
// chunk s (k = 4s .. 4s + 3) reaches only the blocks a >= s / 4.  b[s] is lane (lr, lk)'s B operand
// of chunk s.
__device__ __forceinline__ void lmma_tri(d4 (&acc)[QM], const double* Lx, const double (&b)[16]) {
  const int l = threadIdx.x & 63, llo = (l >> 4) * FS + (l & 15);
#pragma unroll
  for (int s = 0; s < 16; ++s)
#pragma unroll
    for (int a = s >> 2; a < QM; ++a) acc[a] = mfma(Lx[4 * s * FS + 16 * a + llo], b[s], acc[a]);
}
// Row-block core over global operands: acc[a] lane (lr, lk) reg q += sum_k M[16a + lk + 4q][k]
// N[lr][k] (M, N column-major, K a multiple of 16).  Operands
// one 16-deep stage ahead in registers, as mma_64x16 (whose MFMA operands are the other way round).
__device__ __forceinline__ void frag16_load_rd(Frag16& f, const double* pa, const double* pb, size_t sa, size_t sb) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
#pragma unroll
    for (int a = 0; a < QM; ++a) f.a[s][a] = pa[s * sa + 16 * a];
    f.b[s] = pb[s * sb];
  }
}
__device__ __forceinline__ void frag16_mma_rd(d4 (&acc)[QM], const Frag16& f) {
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int a = 0; a < QM; ++a) acc[a] = mfma(f.a[s][a], f.b[s], acc[a]);
}
__device__ __forceinline__ void mma_rd(d4 (&acc)[QM], const double* __restrict__ M, size_t ldm, const double* __restrict__ N,
                                       size_t ldn, int K) {
  const int nst = __builtin_amdgcn_readfirstlane(K >> 4);
  if (nst <= 0) return;
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const double* pa = M + lr + (size_t)lk * ldm;
  const double* pb = N + lr + (size_t)lk * ldn;
  const size_t sa = 4 * ldm, sb = 4 * ldn;
  Frag16 f0, f1;
  frag16_load_rd(f0, pa, pb, sa, sb);
  int it = 0;
  for (; it + 1 < nst; it += 2) {
    __builtin_amdgcn_sched_barrier(0);
    frag16_load_rd(f1, pa + (size_t)(it + 1) * 4 * sa, pb + (size_t)(it + 1) * 4 * sb, sa, sb);
    frag16_mma_rd(acc, f0);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x020, 5, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    const int n2 = (it + 2 < nst) ? it + 2 : it + 1;
    frag16_load_rd(f0, pa + (size_t)n2 * 4 * sa, pb + (size_t)n2 * 4 * sb, sa, sb);
    frag16_mma_rd(acc, f1);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x020, 5, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  if (it < nst) frag16_mma_rd(acc, f0);
}
// Row-packed mma_rd, for products whose output row order is free (the leaf's SYRK items): block a =
// (h = a / 2, p = a % 2) holds rows 32 h + 2 i + p (i = lk + 4 q in the C layout), so a lane's two
// rows 32 h + 2 lr, + 1 of an M column arrive by one 16-B load: 8 A loads per 16-deep stage instead
// of 16.  Every output element sums its k in mma_rd's order: the same results.
struct Frag16p {
  double2 a[4][2];
  double b[4];
};
__device__ __forceinline__ void frag16p_load_rd(Frag16p& f, const double* pa, const double* pb, size_t sa, size_t sb) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
#pragma unroll
    for (int h = 0; h < 2; ++h) f.a[s][h] = *(const double2*)(pa + s * sa + 32 * h);
    f.b[s] = pb[s * sb];
  }
}
__device__ __forceinline__ void frag16p_mma_rd(d4 (&acc)[QM], const Frag16p& f) {
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      acc[2 * h] = mfma(f.a[s][h].x, f.b[s], acc[2 * h]);
      acc[2 * h + 1] = mfma(f.a[s][h].y, f.b[s], acc[2 * h + 1]);
    }
}
// M's rows in pairs (16-B aligned: M's offset and ldm even)
__device__ __forceinline__ void mma_rd_pk(d4 (&acc)[QM], const double* __restrict__ M, size_t ldm, const double* __restrict__ N,
                                          size_t ldn, int K) {
  const int nst = __builtin_amdgcn_readfirstlane(K >> 4);
  if (nst <= 0) return;
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const double* pa = M + 2 * lr + (size_t)lk * ldm;
  const double* pb = N + lr + (size_t)lk * ldn;
  const size_t sa = 4 * ldm, sb = 4 * ldn;
  Frag16p f0, f1;
  frag16p_load_rd(f0, pa, pb, sa, sb);
  int it = 0;
  for (; it + 1 < nst; it += 2) {
    __builtin_amdgcn_sched_barrier(0);
    frag16p_load_rd(f1, pa + (size_t)(it + 1) * 4 * sa, pb + (size_t)(it + 1) * 4 * sb, sa, sb);
    frag16p_mma_rd(acc, f0);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x020, 3, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (it + 2 < nst) frag16p_load_rd(f0, pa + (size_t)(it + 2) * 4 * sa, pb + (size_t)(it + 2) * 4 * sb, sa, sb);
    frag16p_mma_rd(acc, f1);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x020, 3, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  if (it < nst) frag16p_mma_rd(acc, f0);
}
__device__ __forceinline__ void acc_zero4(d4 (&acc)[QM]) {
#pragma unroll
  for (int a = 0; a < QM; ++a) acc[a] = (d4){0.0, 0.0, 0.0, 0.0};
}

__device__ __forceinline__ void leaf9_body(const DevBatch& db, int o, int upd) {
  constexpr int n = 4;
  extern __shared__ __attribute__((aligned(16))) double l9a[];
  double* dT = l9a;                  // wave 0's tile image
  double* dXb = dT + TS * FS;        // two inverse images
  double* Tc = dXb + 2 * TS * FS;    // the chain's L(k+1,k), Tc[c * FS + r] = L[r][c]
  double(*zq)[4][TS] = (double(*)[4][TS])(Tc + TS * FS);  // z partials: 6 off-diagonal tiles
  double(*zqd)[4][TS] = zq + 6;                            // ... and the 4 diagonal tiles
  double* ldiag = (double*)(zqd + 4);  // [2][64]: the diagonal of L_kk (log-determinant)
  Leaf9Sync& sy = *(Leaf9Sync*)(ldiag + 2 * TS);
  const int slot = blockIdx.x;
  if (slot >= db.B || !slot_active(db, slot)) return;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const size_t ld = db.ld, so = (size_t)slot * db.mat;
  // 32-bit element offsets within a slot's matrix: a uniform part plus one of three lane parts
  const int ldi = (int)ld;
  const int lo = lk * ldi + lr;   // row + lr, column + lk
  const int lo2 = lr * ldi + lk;  // row + lk, column + lr
  const int llo = lk * FS + lr;   // LDS images: row + lr, column + lk
  double* S = db.S + so;
  const double* K0 = (upd ? db.S : db.K) + so;
  double* Lw = db.Lw + so;
  double* Li = db.Linv + so;
  double* Mt = db.Mt + so;
  const double* Y = db.Y + (size_t)slot * db.Npad;
  {  // tile o into wave 0's image (all eight waves, all loads in flight first)
    const double* A = K0 + (size_t)o * TS * ld + o * TS;
    double v[TS * TS / (2 * NTHR)];
#pragma unroll
    for (int k = 0; k < TS * TS / (2 * NTHR); ++k) {
      const int e = threadIdx.x + k * 2 * NTHR, r = e & 63, c = e >> 6;
      v[k] = (r >= c) ? A[(size_t)c * ld + r] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < TS * TS / (2 * NTHR); ++k) {
      const int e = threadIdx.x + k * 2 * NTHR, r = e & 63, c = e >> 6;
      dT[c * FS + r] = v[k];
    }
    if (threadIdx.x == 0) {
      sy.tk = 0;
      sy.ch = 0;
      sy.diag_done = 0;
      sy.tile_ready = 1;
      sy.xfree = 0;
      sy.crit = 0;
    }
  }
  __syncthreads();
  if (wave == 0) {  // ---- wave 0: the diagonal tiles
    L9_TS(0);
    for (int k = 0; k < n; ++k) {
      lds_wait_gt(&sy.tile_ready, k, db, slot);
      if (k >= 2) lds_wait_gt(&sy.xfree, k - 2, db, slot);  // step k-2's readers of dX[k & 1] done
      L9_TS(1 + 2 * k);
      diag_w1(db, slot, o + k, dT, dXb + (k & 1) * TS * FS, ldiag + (k & 1) * TS);
      L9_TS(2 + 2 * k);
      lds_publish(&sy.diag_done, k + 1);
    }
  } else {  // ---- the task waves
    // chain quarter of this wave (-1: off the chain): waves 4, 1, 2, 3 -> 0, 1, 2, 3
    const int cw = wave == 4 ? 0 : (wave <= 3 ? wave : -1);
    const int cq = 16 * (cw < 0 ? 0 : cw);
    int gen = 0, cgen = 0;
    d4 yh[2][QM];       // held Y items (inverse row of the next step)
#pragma unroll
    for (int h = 0; h < 2; ++h) acc_zero4(yh[h]);
    // the chain's first operand of step k, A(o+k+1, o+k) rows cq.., staged in the idle inverse
    // image dX[(k+1) & 1] (its step k-1 readers are past their barrier; wave 0 writes it again only
    // after this chain hands tile k+1 over), Bs[c * FS + r] = A[r][c], this wave's rows only
    auto preload = [&](int k) {
      const double* Kc = k > 0 ? S : K0;
      const int kk = o + k, k1 = kk + 1;
      double* Bs = dXb + ((k + 1) & 1) * TS * FS;
      double v[16];
#pragma unroll
      for (int s = 0; s < 16; ++s) v[s] = Kc[(kk * TS + 4 * s) * ldi + k1 * TS + cq + lo];
#pragma unroll
      for (int s = 0; s < 16; ++s) Bs[4 * s * FS + cq + llo] = v[s];
    };
    if (cw >= 0) preload(0);
#ifndef GPRX_L9_BORDER
#define GPRX_L9_BORDER 1
#endif
#ifndef GPRX_L9_PK
#define GPRX_L9_PK 1
#endif
    // phase B (and the held inverse items): round-robin position.  BORDER 1: waves 4, 1, 2, 3 first
    // (wave 4 alone on its SIMD while wave 0 waits; waves 5-7 share SIMDs with the older waves 1-3,
    // which win issue arbitration: a younger wave's first item took 18-20 us against 10-11 us in the
    // leaf timeline), so the critical items land on the waves that run them fastest
    const int rw = GPRX_L9_BORDER ? (wave == 4 ? 0 : (wave <= 3 ? wave : wave - 1)) : l9_pos(wave, L9_HWB);
    int ncrit = 0;  // critical SYRK items of the steps so far (sy.crit's target)
    int nc4p = 0;   // critical items of the previous step's phase B (the held items' offset)
    for (int k = 0; k < n; ++k) {
      const int kk = o + k;
      const double* Kc = k > 0 ? S : K0;
      const double* dX = dXb + (k & 1) * TS * FS;
      // items of Y(k, j) held since the previous step: e = 4 j + c, phase-B item g = nc4p + e on
      // wave l9_wave_of(g); this wave's h-th one is g = g0 + 7 h (g0: its first g >= nc4p)
      const int nyp = 4 * k;  // Y(k, j), j < k
      const int g0p = nc4p + ((rw - nc4p) % L9_HWB + L9_HWB) % L9_HWB;
      lds_wait_gt(&sy.diag_done, k, db, slot);
      if (wave == 5) L9_TS(9 + 4 * k);
      // ---- phase A: the chain; the held inverse items of row k; the diagonal tile's stores; the
      //      other TRSMs of column k
      if (k < n - 1 && cw >= 0) {
        const int k1 = kk + 1;
        d4 cp[QM];  // -A(k1, k1) rows cq.. (blocks a <= cw): loaded under the first product
#pragma unroll
        for (int a = 0; a < QM; ++a)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            cp[a][q] = -Kc[(k1 * TS + 16 * a + 4 * q) * ldi + k1 * TS + cq + lo];  // upper blocks: masked below
        double bp[16];
        {
          const double* Bs = dXb + ((k + 1) & 1) * TS * FS;
#pragma unroll
          for (int s = 0; s < 16; ++s) bp[s] = Bs[4 * s * FS + cq + llo];
        }
        d4 u[QM];
        acc_zero4(u);
        lmma_tri(u, dX, bp);  // L(k1, kk) rows cq.. (transposed)
#pragma unroll
        for (int a = 0; a < QM; ++a)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            Lw[(kk * TS + 16 * a + 4 * q) * ldi + k1 * TS + cq + lo] = u[a][q];
            Tc[(16 * a + 4 * q) * FS + cq + llo] = u[a][q];
          }
        ctr_barrier(&sy.ch, cgen, 4, db, slot);
        // S(k1, k1) rows cq.. = A - L L^T: M = L from Tc, B operand = this wave's own rows of L
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          const double b = u[s >> 2][s & 3];
#pragma unroll
          for (int a = 0; a < QM; ++a)
            cp[a] = mfma(Tc[4 * s * FS + 16 * a + llo], b, cp[a]);
        }
#pragma unroll
        for (int a = 0; a < QM; ++a)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int x = 16 * a + lk + 4 * q;  // column; row cq + lr
            dT[(16 * a + 4 * q) * FS + cq + llo] = (cq + lr >= x) ? -cp[a][q] : 0.0;
          }
        ctr_barrier(&sy.ch, cgen, 4, db, slot);
        if (cw == 0) lds_publish(&sy.tile_ready, k + 2);
        if (wave == 4) L9_TS(10 + 4 * k);
      }
      // held items: X(k, j) = -Linv_kk Y(k, j), columns cq.. of tile (kk, o + j)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int e = g0p + L9_HWB * h - nc4p;
        if (rw >= 0 && e < nyp) {
          const int j = e >> 2, c = e & 3, tj = o + j, xq = 16 * c;
          double b[16];
#pragma unroll
          for (int s = 0; s < 16; ++s) b[s] = yh[h][s >> 2][s & 3];
          d4 x[QM];
          acc_zero4(x);
          lmma_tri(x, dX, b);
          const double yv = Y[tj * TS + xq + lr];
#pragma unroll
          for (int a = 0; a < QM; ++a) {
            double zt[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const double v = -x[a][q];  // Linv(kk, tj)[16a + lk + 4q][xq + lr]
              Li[(tj * TS + xq) * ldi + kk * TS + 16 * a + 4 * q + lo2] = v;
              Mt[(kk * TS + 16 * a + 4 * q) * ldi + tj * TS + xq + lo] = v;  // Mt(tj, kk)^T
              zt[q] = row_sum16(v * yv);
            }
            if (lr == 0) {
              const int kz = k * (k - 1) / 2 + j;
#pragma unroll
              for (int q = 0; q < 4; ++q) zq[kz][c][16 * a + lk + 4 * q] = zt[q];
            }
          }
        }
      }
      // general phase-A items after the held ones: e = nyp.. : the diagonal tile's stores (4
      // column quarters), then TRSM T(i, kk) rows (4 quarters per tile, i = kk + 2 ..)
      {
        const int nt1 = n - 2 - k > 0 ? n - 2 - k : 0;
        const int na = 4 + 4 * nt1;
        bool waited = false;
        for (int e = 0; e < na; ++e) {
          if ((e < 4 ? l9_store_wave(e) : l9_wave_of(nyp + e - 4)) != wave) continue;
          const int c = e & 3, xq = 16 * c;
          if (e >= 4 && !waited) {  // S(ti, kk): the previous step's critical items
            lds_wait_ge(&sy.crit, ncrit, db, slot);
            waited = true;
          }
          if (e < 4) {  // columns xq.. of the diagonal tile: Linv, Mt = Linv^T, z partial
            double* Lc = Li + (size_t)kk * TS * ld + kk * TS;
            double* Mc = Mt + (size_t)kk * TS * ld + kk * TS;
            const int r = l;
            double t = 0.0;
#pragma unroll 4
            for (int cc = xq; cc < xq + 16; ++cc) {
              const double xv = r >= cc ? dX[cc * FS + r] : 0.0;
              Lc[(size_t)cc * ld + r] = xv;
              Mc[(size_t)cc * ld + r] = (cc >= r) ? dX[r * FS + cc] : 0.0;
              t = fma(xv, Y[kk * TS + cc], t);
            }
            zqd[k][c][r] = t;
            if (c == 0) {  // the tile's log-determinant part from wave 0's copy of the diagonal
              const double lsum = wave_sum(log(ldiag[(k & 1) * TS + l]));
              if (l == 0) db.logdet_part[(size_t)slot * db.nt + kk] = lsum;
            }
          } else {  // T(ti, kk) rows xq..: L(ti, kk)[xq + lr][x] = sum_k A[xq + lr][k] Linv_kk[x][k]
            const int ti = kk + 2 + ((e - 4) >> 2);
            double b[16];
#pragma unroll
            for (int s = 0; s < 16; ++s) b[s] = Kc[(kk * TS + 4 * s) * ldi + ti * TS + xq + lo];
            d4 u[QM];
            acc_zero4(u);
            lmma_tri(u, dX, b);
#pragma unroll
            for (int a = 0; a < QM; ++a)
#pragma unroll
              for (int q = 0; q < 4; ++q) Lw[(kk * TS + 16 * a + 4 * q) * ldi + ti * TS + xq + lo] = u[a][q];
          }
        }
      }
      ctr_barrier(&sy.tk, gen, L9_TW, db, slot);
      if (wave == 5) {
        lds_publish(&sy.xfree, k + 1);  // every reader of dX[k & 1] in step k is past the barrier
        L9_TS(11 + 4 * k);
      }
      if (k == n - 1) break;
      // ---- phase B (round 5: no closing barrier): items in the order the next step needs them,
      //      g = 0.. on wave l9_wave_of(g):
      //        the critical SYRK rows (column kk+1 below the diagonal and tile (kk+2, kk+2): the next
      //        step's chain and TRSMs read them, after sy.crit counts them);
      //        Y(k+1, j), j <= k (held for the next phase A);
      //        the other SYRK rows (read only after the next phase A's barrier).
      //      The chain waves then wait for the critical count and stage the next chain operand.
      {
        const int k1 = kk + 1;
        const int ny = 4 * (k + 1);
        const int m = n - 1 - k;  // trailing tiles per edge
        const int nsy = m * (m + 1) / 2 - 1;
        const int nc4 = 4 * l9_crit_tiles(m);
        [[maybe_unused]] int nb = 0;
        W_TS(8 * k);
        // SYRK row item e (tile e / 4 of the enumeration, quarter e % 4)
        auto syrk_item = [&](int e) {
          const int c = e & 3, xq = 16 * c;
          int u = (e >> 2) + 1, cc = 0;  // lower trailing tile u (column-major), skipping (k1, k1)
          while (u >= m - cc) {
            u -= m - cc;
            ++cc;
          }
          const int tj = k1 + cc, ti = tj + u;
          // S(ti, tj) rows xq..: OUT[x][xq + lr] = S[xq + lr][x], M = L(tj, kk), N = L(ti, kk) rows xq..
          // (a diagonal tile's blocks above the diagonal are formed and stored too: no reader uses them)
          d4 acc[QM];
#if GPRX_L9_PK
          // row-packed core: block a holds OUT rows 32 (a / 2) + (a % 2) + 2 lk + 8 q
          const int lop = 2 * lk * ldi + lr;
#pragma unroll
          for (int a = 0; a < QM; ++a)
#pragma unroll
            for (int q = 0; q < 4; ++q)
              acc[a][q] = -Kc[(tj * TS + 32 * (a >> 1) + (a & 1) + 8 * q) * ldi + ti * TS + xq + lop];
          mma_rd_pk(acc, Lw + (size_t)kk * TS * ld + tj * TS, ld, Lw + (size_t)kk * TS * ld + ti * TS + xq, ld, TS);
#pragma unroll
          for (int a = 0; a < QM; ++a)
#pragma unroll
            for (int q = 0; q < 4; ++q)
              S[(tj * TS + 32 * (a >> 1) + (a & 1) + 8 * q) * ldi + ti * TS + xq + lop] = -acc[a][q];
#else
#pragma unroll
          for (int a = 0; a < QM; ++a)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[a][q] = -Kc[(tj * TS + 16 * a + 4 * q) * ldi + ti * TS + xq + lo];
          mma_rd(acc, Lw + (size_t)kk * TS * ld + tj * TS, ld, Lw + (size_t)kk * TS * ld + ti * TS + xq, ld, TS);
#pragma unroll
          for (int a = 0; a < QM; ++a)
#pragma unroll
            for (int q = 0; q < 4; ++q) S[(tj * TS + 16 * a + 4 * q) * ldi + ti * TS + xq + lo] = -acc[a][q];
#endif
          W_TS(8 * k + 1 + (nb < 5 ? nb++ : 5));
        };
        for (int g = rw < 0 ? nc4 : rw; g < nc4; g += L9_HWB) {
          syrk_item(g);
          lds_count(&sy.crit);
        }
        const int g0 = nc4 + ((rw - nc4) % L9_HWB + L9_HWB) % L9_HWB;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int e = g0 + L9_HWB * h - nc4;
          if (rw >= 0 && e < ny) {
            const int j = e >> 2, c = e & 3, tj = o + j, xq = 16 * c;
            // Y(k1, tj)[:, xq..] = sum_{m=tj}^{kk} L(k1, m) Linv(m, tj): M = Lw row k1, N = Mt row tj
            // (Linv(m, tj)^T); Linv(tj, tj)'s columns xq.. are zero above row xq: K starts at xq
            acc_zero4(yh[h]);
            mma_rd(yh[h], Lw + (size_t)(tj * TS + xq) * ld + k1 * TS, ld, Mt + (size_t)(tj * TS + xq) * ld + tj * TS + xq, ld,
                   (k1 - tj) * TS - xq);
            W_TS(8 * k + 1 + (nb < 5 ? nb++ : 5));
          }
        }
        for (int g = rw < 0 ? 4 * nsy + ny : nc4 + ny + ((rw - nc4 - ny) % L9_HWB + L9_HWB) % L9_HWB; g < 4 * nsy + ny; g += L9_HWB)
          syrk_item(g - ny);
        W_TS(8 * k + 7);
        ncrit += nc4;
        nc4p = nc4;
      }
      if (wave == 5) L9_TS(12 + 4 * k);
      if (cw >= 0 && k + 1 < n - 1) {
        lds_wait_ge(&sy.crit, ncrit, db, slot);  // S(kk+2, kk+1) and S(kk+2, kk+2) for the chain
        preload(k + 1);
      }
    }
  }
  __syncthreads();
  if (wave == 0) L9_TS(25);
  // z partials: the diagonal tiles' and the off-diagonal tiles' quarters summed in quarter order
  for (int e = threadIdx.x; e < (n + 6) * TS; e += 2 * NTHR) {
    const int t = e >> 6, r = e & 63;
    int ti, tj;
    double v;
    if (t < n) {
      ti = tj = o + t;
      v = ((zqd[t][0][r] + zqd[t][1][r]) + zqd[t][2][r]) + zqd[t][3][r];
    } else {
      const int kz = t - n;
      int k = 1;
      while (k * (k + 1) / 2 <= kz) ++k;
      ti = o + k;
      tj = o + (kz - k * (k - 1) / 2);
      v = ((zq[kz][0][r] + zq[kz][1][r]) + zq[kz][2][r]) + zq[kz][3][r];
    }
    zp_row(db, slot, 2 * tj)[ti * TS + r] = v;
    zp_row(db, slot, 2 * tj + 1)[ti * TS + r] = 0.0;
  }
}
constexpr size_t leaf9_lds_bytes() {
  return (4 * TS * FS + 10 * 4 * TS + 2 * TS) * sizeof(double) + sizeof(Leaf9Sync);
}
// k_node8's LINV21 epilogue puts its eight waves' transpose buffers in the leaf's LDS
static_assert(leaf9_lds_bytes() >= 2 * linv21_lds_bytes(), "k_node8: LINV21 transpose buffers exceed the leaf's LDS");
__global__ __launch_bounds__(2 * NTHR) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_leaf9(DevBatch db, int o, int upd) {
  leaf9_body(db, o, upd);
}
// A whole 8-tile recursion node (512 x 512) in one launch, one 8-wave workgroup per slot, a
// workgroup barrier between the phases: the top leaf (leaf9_body), TRSM and SYRK + TT, the bottom
// leaf (tiles updated into S) and LINV21 (L^-1_21 = -L22^-1 T) -- five launches of the recursion
// with the same tile work.  The GEMM phases run the slot's units on the two halves of the
// workgroup (gemm_unit); LINV21's transposed Mt store uses the leaf's LDS, dead after its barrier.
// Round 5: the node's second half joined the first (it was a launch of its own, k_node9b), so each
// slot goes on to its bottom leaf when its own SYRK + TT is done instead of every slot waiting for
// the slowest one at the launch boundary: 2.84-2.89 -> 2.79-2.82 ms per step for the four nodes.
__global__ __launch_bounds__(2 * NTHR) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_node8(DevBatch db, int o, int upd) {
  const int slot = blockIdx.x;
  if (slot >= db.B || !slot_active(db, slot)) return;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), half = wave >> 2, w = wave & 3;
  const GemmGeom none{OP_NONE, 0, 0, 0};
  N_TS(0);
  N_TS(6);
  N_TS(7);
  leaf9_body(db, o, upd);
  __syncthreads();
  N_TS(1);
  gemm_unit<false, REV_B, false>(db, GemmGeom{OP_TRSM, o, 4, 8, upd}, none, slot, half, w, 2);
  __syncthreads();
  N_TS(2);
  gemm_unit<false, TRI_A_FIRST, false>(db, GemmGeom{OP_SYRK, o, 4, 8, upd}, GemmGeom{OP_TT, o, 4, 8, upd}, slot, half, w, 2);
  __syncthreads();
  N_TS(3);
  leaf9_body(db, o + 4, 1);
  __syncthreads();
  N_TS(4);
  gemm_unit<false, REV_A, false>(db, GemmGeom{OP_LINV21, o, 4, 8, upd}, none, slot, half, w, 2);
  N_TS(5);
}

// ============================================================================================
// k_node8h (round 6): the same 8-tile node on a 4-wave workgroup per slot in 68 KB of LDS, so two
// slots share a CU (one wave of each per SIMD, 256 VGPRs each, as k_node8's two waves per SIMD).
// k_node8 holds one slot per CU: its leaves are latency chains (the diagonal wave's factor, the
// chain products, the task items' operand round trips) that leave the CU's MFMA pipes mostly idle,
// and a launch of more slots than CUs (the CP batches, the sweeps' and searches' N = 512 .. 2048
// groups) runs them round after round.  With two slots per CU one slot's leaf latency overlaps the
// other's GEMM phases -- the plan; measured (scratch/node_timeline.py), a paired slot runs every
// phase, its leaves included, at about half its solo speed: the diagonal wave's fp64 VALU chain and
// the items' MFMAs share each SIMD's one fp64 pipe with the other slot's MFMAs, so the pair gains
// nothing ("Two slots per CU").  Kept as an option (GPRX_OPT_NODE_WAVES = 4), off by
// default.  Every product, sum and store is k_node8's, in the same order: the results
// are bit-identical (tests/test_gpu.py::test_node8_four_wave_form_bit_identical), so the launch
// form never changes a result and the batch-size rule of set_geometry stays the only geometry one.
// What changes against leaf9_body:
//   * LDS: the tile image dT and ONE inverse image dX (leaf9: two, plus the chain's image Tc).  The
//     chain writes L(k+1,k) into dT (tile k's image is dead once its inverse is in dX), reads it
//     into registers, and writes tile k+1 over it after one more barrier.  The diagonal wave keeps
//     the 16 x 16 block inverses Dinv_P in dT's unused strictly-upper blocks while it factors
//     (diag_w1s), and writes the inverse into dX only after the previous step's readers of dX are
//     done (xfree), so most of its tile still overlaps them.
//   * the z partial quarters go to the slot's S buffer, in its unused upper tile (o, o + 3) (no
//     kernel reads or writes S's strictly-upper off-diagonal tiles), and are summed in leaf9's
//     order;
//   * the chain takes its operands straight from L2 (no staging image), and its four quarters run
//     on all four waves (the diagonal wave is idle during the chain);
//   * the inverse items' Y(k, j) are parked in their own Linv destination instead of registers
//     (any of the three task waves finishes any item; a counter orders park and reuse).
// ============================================================================================
struct Leaf4Sync {
  int tk;         // task-wave barrier counter (3 per barrier)
  int ch;         // chain barrier counter (4 per barrier)
  int diag_done;  // diagonal tiles factored and inverted
  int xfree;      // steps whose readers of dX are done
  int crit;       // critical SYRK items done (monotonic)
  int ypark;      // Y items parked (monotonic)
};
constexpr int L4_TW = 3;
constexpr size_t leaf4_lds_bytes() { return (2 * TS * FS + 2 * TS) * sizeof(double) + sizeof(Leaf4Sync); }
static_assert(leaf4_lds_bytes() >= linv21_lds_bytes(), "k_node8h: LINV21 transpose buffers exceed the leaf's LDS");
static_assert(2 * leaf4_lds_bytes() <= 160 * 1024, "k_node8h: two workgroups per CU");
// staging block of Dinv_P in the tile image's strictly-upper blocks: (row block, column block)
__device__ __forceinline__ constexpr int l4_stage_r(int P) { return P == 3 ? 16 : 0; }
__device__ __forceinline__ constexpr int l4_stage_c(int P) { return P == 3 ? 32 : 16 * (P + 1); }
// w1_panel with Dinv_P read from its staging block (the same values as Xi's diagonal block)
template <int P>
__device__ __forceinline__ void w1_panel_s(double* T, int lr, int lk) {
  constexpr int NT = 3 - P;
  if constexpr (NT > 0) {
    constexpr int c0 = 16 * P, R0 = l4_stage_r(P), C0 = l4_stage_c(P);
    double bv[4], av[NT][4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bv[s] = T[(C0 + 4 * s + lk) * FS + R0 + lr];
#pragma unroll
      for (int i = 0; i < NT; ++i) av[i][s] = T[(c0 + 4 * s + lk) * FS + 16 * (P + 1 + i) + lr];
    }
    d4 acc[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) acc[i] = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < NT; ++i) acc[i] = mfma(av[i][s], bv[s], acc[i]);
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) T[(c0 + lr) * FS + 16 * (P + 1 + i) + lk + 4 * q] = acc[i][q];
    wave_sync();
    double pv[NT][4];
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int s = 0; s < 4; ++s) pv[i][s] = T[(c0 + 4 * s + lk) * FS + 16 * (P + 1 + i) + lr];
    constexpr int NB = NT * (NT + 1) / 2;
    d4 sacc[NB], old[NB];
#pragma unroll
    for (int b = 0, j = 0; j < NT; ++j)
#pragma unroll
      for (int i = j; i < NT; ++i, ++b) {
#pragma unroll
        for (int q = 0; q < 4; ++q) old[b][q] = T[(16 * (P + 1 + j) + lr) * FS + 16 * (P + 1 + i) + lk + 4 * q];
        sacc[b] = (d4){0.0, 0.0, 0.0, 0.0};
      }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int b = 0, j = 0; j < NT; ++j)
#pragma unroll
        for (int i = j; i < NT; ++i, ++b) sacc[b] = mfma(pv[i][s], pv[j][s], sacc[b]);
#pragma unroll
    for (int b = 0, j = 0; j < NT; ++j)
#pragma unroll
      for (int i = j; i < NT; ++i, ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) T[(16 * (P + 1 + j) + lr) * FS + 16 * (P + 1 + i) + lk + 4 * q] = old[b][q] - sacc[b][q];
    wave_sync();
  }
}
// diag_w1 with the block inverses staged in T; before_inverse() runs between the factor and the
// inverse (the wait for dX's readers), then the staged blocks go to Xi and the off-diagonal inverse
// blocks follow as in diag_w1
template <class F>
__device__ __forceinline__ void diag_w1s(const DevBatch& db, int slot, int jt, double* T, double* Xi, double* ldiag,
                                         F&& before_inverse) {
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  int fail = -1;
  for (int P = 0; P < 4; ++P) {
    const int c0 = 16 * P;
    double a[16], y[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      a[k] = T[(c0 + k) * FS + c0 + lr];
      y[k] = (k == lr) ? 1.0 : 0.0;
    }
    double d = T[(c0 + lr) * FS + c0 + lr], pv = 1.0;
    int fl = -1;
    fact_step<0>(a, y, d, pv, lr, fl);
    fl = __builtin_amdgcn_readfirstlane(fl);
    if (fail < 0 && fl >= 0) fail = c0 + fl;
    {
      double sl, rl;
      sqrt_rsqrt(pv, sl, rl);
      fact_scale<0>(a, y, rl, sl, lr);
    }
    if (l < 16) {
#pragma unroll
      for (int k = 0; k < 16; ++k) T[(c0 + k) * FS + c0 + l] = (k <= l) ? a[k] : 0.0;
      ldiag[c0 + l] = a[l];
    }
    __builtin_amdgcn_wave_barrier();
    if (l < 16) {
      const int R0 = P == 3 ? 16 : 0, C0 = P == 3 ? 32 : 16 * (P + 1);
#pragma unroll
      for (int r = 0; r < 16; ++r) T[(C0 + l) * FS + R0 + r] = y[r];
    }
    wave_sync();
    switch (P) {
      case 0: w1_panel_s<0>(T, lr, lk); break;
      case 1: w1_panel_s<1>(T, lr, lk); break;
      case 2: w1_panel_s<2>(T, lr, lk); break;
      default: break;
    }
  }
  before_inverse();
#pragma unroll
  for (int P = 0; P < 4; ++P) {
    const int R0 = P == 3 ? 16 : 0, C0 = P == 3 ? 32 : 16 * (P + 1);
#pragma unroll
    for (int e = l; e < 256; e += 64) {
      const int r = e & 15, c = e >> 4;
      Xi[(16 * P + c) * FS + 16 * P + r] = T[(C0 + c) * FS + R0 + r];
    }
  }
  wave_sync();
  w1_inverse<1>(T, Xi, lr, lk);
  w1_inverse<2>(T, Xi, lr, lk);
  w1_inverse<3>(T, Xi, lr, lk);
  if (fail >= 0 && l == 0 && db.status[slot] == 0) {
    db.status[slot] = 1;
    db.info[slot] = jt * TS + fail + 1;
  }
}
// rot: the wave roles rotate by rot (0 or 2): the diagonal wave, the VALU-bound routine, is wave
// rot, so that two workgroups sharing a CU can put their diagonal waves on different SIMDs
__device__ __forceinline__ void leaf4_body(const DevBatch& db, int o, int upd, int rot) {
  constexpr int n = 4;
  extern __shared__ __attribute__((aligned(16))) double l4a[];
  double* dT = l4a;                    // the tile image; the chain's L(k+1,k); Dinv staging
  double* dX = dT + TS * FS;           // the inverse image Linv_kk
  double* ldiag = dX + TS * FS;        // [2][64]: the diagonal of L_kk (log-determinant)
  Leaf4Sync& sy = *(Leaf4Sync*)(ldiag + 2 * TS);
  const int slot = blockIdx.x;
  const int wave = (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) + rot) & 3;  // this wave's role
  const int l = threadIdx.x & 63, lr = l & 15, lk = l >> 4;
  const size_t ld = db.ld, so = (size_t)slot * db.mat;
  const int ldi = (int)ld;
  const int lo = lk * ldi + lr, lo2 = lr * ldi + lk, llo = lk * FS + lr;
  double* S = db.S + so;
  const double* K0 = (upd ? db.S : db.K) + so;
  double* Lw = db.Lw + so;
  double* Li = db.Linv + so;
  double* Mt = db.Mt + so;
  const double* Y = db.Y + (size_t)slot * db.Npad;
  // z partial quarters in S's upper tile (o, o + 3): column 4 kz + c (off-diagonal tile kz), 24 +
  // 4 t + c (diagonal tile t), row r
  double* zg = S + (size_t)(o + 3) * TS * ld + o * TS;
  {  // tile o into the image
    const double* A = K0 + (size_t)o * TS * ld + o * TS;
    double v[TS * TS / NTHR];
#pragma unroll
    for (int k = 0; k < TS * TS / NTHR; ++k) {
      const int e = threadIdx.x + k * NTHR, r = e & 63, c = e >> 6;
      v[k] = (r >= c) ? A[(size_t)c * ld + r] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < TS * TS / NTHR; ++k) {
      const int e = threadIdx.x + k * NTHR, r = e & 63, c = e >> 6;
      dT[c * FS + r] = v[k];
    }
    if (threadIdx.x == 0) {
      sy.tk = 0;
      sy.ch = 0;
      sy.diag_done = 0;
      sy.xfree = 0;
      sy.crit = 0;
      sy.ypark = 0;
    }
  }
  __syncthreads();
  const int cq = 16 * wave;  // this wave's chain quarter
  int cgen = 0;
  // the chain of step k on all four waves: L(k1, kk) rows cq.. = A(k1, kk) Linv_kk^T, then tile
  // k1 = A(k1, k1) - L L^T into dT (leaf9_body's products, operands from L2)
  auto chain = [&](int k, int ncrit) {
    const double* Kc = k > 0 ? S : K0;
    const int kk = o + k, k1 = kk + 1;
    lds_wait_ge(&sy.crit, ncrit, db, slot);  // S(k1, kk), S(k1, k1) of the previous step
    d4 cp[QM];
#pragma unroll
    for (int a = 0; a < QM; ++a)
#pragma unroll
      for (int q = 0; q < 4; ++q) cp[a][q] = -Kc[(k1 * TS + 16 * a + 4 * q) * ldi + k1 * TS + cq + lo];
    double bp[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) bp[s] = Kc[(kk * TS + 4 * s) * ldi + k1 * TS + cq + lo];
    d4 u[QM];
    acc_zero4(u);
    lmma_tri(u, dX, bp);
#pragma unroll
    for (int a = 0; a < QM; ++a)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        Lw[(kk * TS + 16 * a + 4 * q) * ldi + k1 * TS + cq + lo] = u[a][q];
        dT[(16 * a + 4 * q) * FS + cq + llo] = u[a][q];
      }
    ctr_barrier(&sy.ch, cgen, 4, db, slot);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const double b = u[s >> 2][s & 3];
#pragma unroll
      for (int a = 0; a < QM; ++a) cp[a] = mfma(dT[4 * s * FS + 16 * a + llo], b, cp[a]);
    }
    ctr_barrier(&sy.ch, cgen, 4, db, slot);  // every quarter's reads of L(k1, kk) done
#pragma unroll
    for (int a = 0; a < QM; ++a)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int x = 16 * a + lk + 4 * q;
        dT[(16 * a + 4 * q) * FS + cq + llo] = (cq + lr >= x) ? -cp[a][q] : 0.0;
      }
    ctr_barrier(&sy.ch, cgen, 4, db, slot);  // tile k1 in dT
  };
  if (wave == 0) {  // ---- the diagonal tiles, and chain quarter 0
    int ncrit = 0;
    for (int k = 0; k < n; ++k) {
      diag_w1s(db, slot, o + k, dT, dX, ldiag + (k & 1) * TS, [&] { lds_wait_ge(&sy.xfree, k, db, slot); });
      lds_publish(&sy.diag_done, k + 1);
      if (k == n - 1) break;
      chain(k, ncrit);
      ncrit += 4 * l9_crit_tiles(n - 1 - k);
    }
  } else {  // ---- the task waves 1..3: chain quarters 1..3 and every tile item
    const int tw = wave - 1;
    int gen = 0, ncrit = 0;
    for (int k = 0; k < n; ++k) {
      const int kk = o + k;
      const double* Kc = k > 0 ? S : K0;
      lds_wait_gt(&sy.diag_done, k, db, slot);
      if (k < n - 1) chain(k, ncrit);
      // ---- phase A: X(k, j) = -Linv_kk Y(k, j) (Y parked in the item's Linv destination), the
      //      diagonal tile's stores (4 column quarters), the TRSM rows of column k
      {
        const int nx = 4 * k, nt1 = n - 2 - k > 0 ? n - 2 - k : 0, na = nx + 4 + 4 * nt1;
        bool waited_y = false, waited_c = false;
        for (int e = tw; e < na; e += L4_TW) {
          if (e < nx) {
            if (!waited_y) {  // Y(k, .) of the previous step's phase B
              lds_wait_ge(&sy.ypark, 2 * k * (k + 1), db, slot);
              waited_y = true;
            }
            const int j = e >> 2, c = e & 3, tj = o + j, xq = 16 * c;
            double b[16];
#pragma unroll
            for (int s = 0; s < 16; ++s) b[s] = Li[(tj * TS + xq) * ldi + kk * TS + 16 * (s >> 2) + 4 * (s & 3) + lo2];
            d4 x[QM];
            acc_zero4(x);
            lmma_tri(x, dX, b);
            const double yv = Y[tj * TS + xq + lr];
#pragma unroll
            for (int a = 0; a < QM; ++a) {
              double zt[4];
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const double v = -x[a][q];
                Li[(tj * TS + xq) * ldi + kk * TS + 16 * a + 4 * q + lo2] = v;
                Mt[(kk * TS + 16 * a + 4 * q) * ldi + tj * TS + xq + lo] = v;
                zt[q] = row_sum16(v * yv);
              }
              if (lr == 0) {
                const int kz = k * (k - 1) / 2 + j;
#pragma unroll
                for (int q = 0; q < 4; ++q) zg[(size_t)(4 * kz + c) * ld + 16 * a + lk + 4 * q] = zt[q];
              }
            }
          } else if (e < nx + 4) {  // columns xq.. of the diagonal tile: Linv, Mt = Linv^T, z partial
            const int c = e - nx, xq = 16 * c;
            double* Lc = Li + (size_t)kk * TS * ld + kk * TS;
            double* Mc = Mt + (size_t)kk * TS * ld + kk * TS;
            const int r = l;
            double t = 0.0;
#pragma unroll 4
            for (int cc = xq; cc < xq + 16; ++cc) {
              const double xv = r >= cc ? dX[cc * FS + r] : 0.0;
              Lc[(size_t)cc * ld + r] = xv;
              Mc[(size_t)cc * ld + r] = (cc >= r) ? dX[r * FS + cc] : 0.0;
              t = fma(xv, Y[kk * TS + cc], t);
            }
            zg[(size_t)(24 + 4 * k + c) * ld + r] = t;
            if (c == 0) {
              const double lsum = wave_sum(log(ldiag[(k & 1) * TS + l]));
              if (l == 0) db.logdet_part[(size_t)slot * db.nt + kk] = lsum;
            }
          } else {  // T(ti, kk) rows xq..
            if (!waited_c) {  // S(ti, kk): the previous step's critical items
              lds_wait_ge(&sy.crit, ncrit, db, slot);
              waited_c = true;
            }
            const int f = e - nx - 4, c = f & 3, xq = 16 * c, ti = kk + 2 + (f >> 2);
            double b[16];
#pragma unroll
            for (int s = 0; s < 16; ++s) b[s] = Kc[(kk * TS + 4 * s) * ldi + ti * TS + xq + lo];
            d4 u[QM];
            acc_zero4(u);
            lmma_tri(u, dX, b);
#pragma unroll
            for (int a = 0; a < QM; ++a)
#pragma unroll
              for (int q = 0; q < 4; ++q) Lw[(kk * TS + 16 * a + 4 * q) * ldi + ti * TS + xq + lo] = u[a][q];
          }
        }
      }
      ctr_barrier(&sy.tk, gen, L4_TW, db, slot);
      if (wave == 1) lds_publish(&sy.xfree, k + 1);  // every reader of dX in step k is past the barrier
      if (k == n - 1) break;
      // ---- phase B: the critical SYRK rows (counted), Y(k+1, j) (parked, counted), the other
      //      SYRK rows; round robin over the task waves in that order
      {
        const int k1 = kk + 1;
        const int ny = 4 * (k + 1);
        const int m = n - 1 - k;
        const int nsy = m * (m + 1) / 2 - 1;
        const int nc4 = 4 * l9_crit_tiles(m);
        for (int g = tw; g < ny + 4 * nsy; g += L4_TW) {
          if (g >= nc4 && g < nc4 + ny) {  // Y(k1, tj)[:, xq..], parked at Linv(k1, tj)[:, xq..]
            const int e = g - nc4, j = e >> 2, c = e & 3, tj = o + j, xq = 16 * c;
            d4 yh[QM];
            acc_zero4(yh);
            mma_rd(yh, Lw + (size_t)(tj * TS + xq) * ld + k1 * TS, ld, Mt + (size_t)(tj * TS + xq) * ld + tj * TS + xq, ld,
                   (k1 - tj) * TS - xq);
#pragma unroll
            for (int a = 0; a < QM; ++a)
#pragma unroll
              for (int q = 0; q < 4; ++q) Li[(tj * TS + xq) * ldi + k1 * TS + 16 * a + 4 * q + lo2] = yh[a][q];
            lds_count(&sy.ypark);
            continue;
          }
          const int e = g < nc4 ? g : g - ny;  // SYRK row item e
          const int c = e & 3, xq = 16 * c;
          int u = (e >> 2) + 1, cc = 0;
          while (u >= m - cc) {
            u -= m - cc;
            ++cc;
          }
          const int tj = k1 + cc, ti = tj + u;
          d4 acc[QM];
#pragma unroll
          for (int a = 0; a < QM; ++a)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[a][q] = -Kc[(tj * TS + 16 * a + 4 * q) * ldi + ti * TS + xq + lo];
          mma_rd(acc, Lw + (size_t)kk * TS * ld + tj * TS, ld, Lw + (size_t)kk * TS * ld + ti * TS + xq, ld, TS);
#pragma unroll
          for (int a = 0; a < QM; ++a)
#pragma unroll
            for (int q = 0; q < 4; ++q) S[(tj * TS + 16 * a + 4 * q) * ldi + ti * TS + xq + lo] = -acc[a][q];
          if (g < nc4) lds_count(&sy.crit);
        }
        ncrit += nc4;
      }
    }
  }
  __syncthreads();
  // z partials: the quarters summed in quarter order (leaf9_body's sums)
  for (int e = threadIdx.x; e < (n + 6) * TS; e += NTHR) {
    const int t = e >> 6, r = e & 63;
    int ti, tj;
    double v;
    if (t < n) {
      ti = tj = o + t;
      const double* q0 = zg + (size_t)(24 + 4 * t) * ld + r;
      v = ((q0[0] + q0[ld]) + q0[2 * ld]) + q0[3 * ld];
    } else {
      const int kz = t - n;
      int k = 1;
      while (k * (k + 1) / 2 <= kz) ++k;
      ti = o + k;
      tj = o + (kz - k * (k - 1) / 2);
      const double* q0 = zg + (size_t)(4 * kz) * ld + r;
      v = ((q0[0] + q0[ld]) + q0[2 * ld]) + q0[3 * ld];
    }
    zp_row(db, slot, 2 * tj)[ti * TS + r] = v;
    zp_row(db, slot, 2 * tj + 1)[ti * TS + r] = 0.0;
  }
}
__global__ __launch_bounds__(NTHR) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_node8h(DevBatch db, int o, int upd) {
  const int slot = blockIdx.x;
  if (slot >= db.B || !slot_active(db, slot)) return;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const GemmGeom none{OP_NONE, 0, 0, 0};
#ifndef GPRX_N8H_ROT
#define GPRX_N8H_ROT 1
#endif
  // workgroups b and b + 256 tend to share a CU (256 CUs filled in block order)
  const int rot = GPRX_N8H_ROT == 1 ? ((blockIdx.x >> 8) & 1) * 2 : 0;
  N_TS(0);
  N_TS(6);
  N_TS(7);
  leaf4_body(db, o, upd, rot);
  __syncthreads();
  N_TS(1);
#pragma unroll 1
  for (int u = 0; u < 2; ++u) gemm_unit<false, REV_B, false>(db, GemmGeom{OP_TRSM, o, 4, 8, upd}, none, slot, u, wave, 2);
  __syncthreads();
  N_TS(2);
#pragma unroll 1
  for (int u = 0; u < 2; ++u)
    gemm_unit<false, TRI_A_FIRST, false>(db, GemmGeom{OP_SYRK, o, 4, 8, upd}, GemmGeom{OP_TT, o, 4, 8, upd}, slot, u, wave, 2);
  __syncthreads();
  N_TS(3);
  leaf4_body(db, o + 4, 1, rot);
  __syncthreads();
  N_TS(4);
#pragma unroll 1
  for (int u = 0; u < 2; ++u) gemm_unit<false, REV_A, false>(db, GemmGeom{OP_LINV21, o, 4, 8, upd}, none, slot, u, wave, 2);
  N_TS(5);
}



// ============================================================================================
// alpha = L^-T (L^-1 y).  phase 0: z = Linv y ; phase 1: alpha = Mt z.   grid = B * nt
// ============================================================================================
__global__ __launch_bounds__(NTHR) void k_alpha(DevBatch db, int phase) {
  __shared__ double part[4][TS];
  int slot, i;
  if (!map_slot(db, db.nt, slot, i)) return;
  const int r = threadIdx.x & 63, pt = threadIdx.x >> 6;
  if (phase == 0) {  // z = L^-1 y from the producers' partials: rows of tile i, halves h < 2(i+1)
    double acc = 0.0;
    for (int h = pt; h < 2 * (i + 1); h += 4) acc += zp_row(db, slot, h)[i * TS + r];
    part[pt][r] = acc;
    __syncthreads();
    if (pt == 0) db.z[(size_t)slot * db.Npad + i * TS + r] = ((part[0][r] + part[1][r]) + part[2][r]) + part[3][r];
    return;
  }
  const size_t ld = db.ld;
  // lane: rows 2 rp, 2 rp + 1 of the tile row (one 16-B load), columns of parity cp: one load
  // instruction reads two whole 512-B column segments.  The column range [k0, Npad) is split in 4
  // contiguous quarters of whole 16-column groups (wave-uniform, so z comes in by scalar loads).
  const int rp = r & 31, cp = r >> 5, w = __builtin_amdgcn_readfirstlane(pt);
  const double* A = db.Mt + (size_t)slot * db.mat + i * TS + 2 * rp + (size_t)cp * ld;
  const double* v = db.z + (size_t)slot * db.Npad;
  const int k0 = i * TS, k1 = db.Npad;
  const int ng = (k1 - k0) / 16, g0 = (ng * w) / 4, g1 = (ng * (w + 1)) / 4;
  typedef double d2 __attribute__((ext_vector_type(2)));
  d2 acc[4] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}};
  // group gq + 1's loads are issued before group gq's arithmetic (16 loads in flight per lane)
  d2 m[8];
  if (g0 < g1) {
#pragma unroll
    for (int u = 0; u < 8; ++u) m[u] = *(const d2*)(A + (size_t)(k0 + 16 * g0 + 2 * u) * ld);
  }
  for (int gq = g0; gq < g1; ++gq) {
    const int kk = k0 + 16 * gq;
    d2 mn[8];
    if (gq + 1 < g1) {
#pragma unroll
      for (int u = 0; u < 8; ++u) mn[u] = *(const d2*)(A + (size_t)(kk + 16 + 2 * u) * ld);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const double zv = cp ? v[kk + 2 * u + 1] : v[kk + 2 * u];
      acc[u & 3].x = fma(m[u].x, zv, acc[u & 3].x);
      acc[u & 3].y = fma(m[u].y, zv, acc[u & 3].y);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) m[u] = mn[u];
  }
  double s0 = (acc[0].x + acc[1].x) + (acc[2].x + acc[3].x), s1 = (acc[0].y + acc[1].y) + (acc[2].y + acc[3].y);
  s0 = sum_xor32(s0);  // the other column parity
  s1 = sum_xor32(s1);
  if (cp == 0) {
    part[pt][2 * rp] = s0;
    part[pt][2 * rp + 1] = s1;
  }
  __syncthreads();
  if (pt == 0) {
    const double s = ((part[0][r] + part[1][r]) + part[2][r]) + part[3][r];
    db.alpha[(size_t)slot * db.Npad + i * TS + r] = s;
  }
}

// ============================================================================================
// K^-1 lower tiles = Mt_i Mt_j^T (K range [i, nt)), fused with the gradient partial sums
//   G_rc = wt_rc * (alpha_r alpha_c - Kinv_rc) * Kf_rc    (wt = 1/2 on the diagonal, as
//                                                        dmll_kern! weights ααinvcKI[j,j]/2)
//   S_p = sum G_rc (x_pr - x_pc)^2,  S_f = sum G_rc,  T = sum_diag W_rr
// One gradient partial row per unit of 4 tiles.  Kf is K's lower tile (ti, tj) exactly as the Gram
// wrote it (the factorisation's SYRKs write S, never K), read once per output tile; only entries
// with gi > gj are used, so the noise on the diagonal is never seen: G_rr uses sf2 analytically.
//
// The distance sums are expanded per wave tile (rows r, columns c):
//   S_p = sum_r x_pr^2 R_r + sum_c x_pc^2 C_c - 2 sum_r x_pr Q_rp,   Q = G Xc  (64 x d)
// with R / C the row / column sums of G.  Q runs on the MFMA pipe with G straight from the
// accumulators as the B operand (the swapped-operand C layout of mma_64x32 is exactly a B
// fragment), so the epilogue costs ~2d MFMAs + a few dozen cross-lane sums per wave instead of
// 32 d distance evaluations and d wave reductions.  x is the centred copy Xc (per-dimension mean
// removed; S_p is translation invariant), which keeps the expansion's cancellation at the
// rounding level of the points' spread, as for the reference's own a^2 + b^2 - 2ab distances.
// LDS: the unit's point tiles as raw [point][xs] images (LDS-DMA, issued after the MFMA loop),
// per-wave partials and alpha of the image points.
// ============================================================================================
__device__ __forceinline__ void dma_tile(double* lds, const double* src, int ndbl) {
  // ndbl doubles (even) from src to lds, 16 B per lane, one wave-instruction per KiB;
  // the LDS destination of each instruction is wave-uniform (M0), lane i writes base + 16 i
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, nch = ndbl >> 1;
  for (int c0 = w * 64; c0 < nch; c0 += NTHR) {
    if (c0 + l < nch)
      __builtin_amdgcn_global_load_lds((const void*)(src + 2 * (c0 + l)),
                                       (__attribute__((address_space(3))) void*)(lds + 2 * c0), 16, 0, 0);
  }
}
constexpr int SPW = DMAX + 2;  // per-wave partial row: S_p (d), S_f, T
// LDS of a lauum workgroup: per-wave partials, alpha of the image points, then nimg point-tile
// images [64][xs] (16-B aligned: the small arrays hold an even count)
static_assert((4 * SPW + 5 * TS) % 2 == 0, "lauum LDS image base alignment");
__host__ __device__ inline size_t lauum_lds_dbl(int xs, int nimg) {
  return (size_t)4 * SPW + 5 * TS + (size_t)nimg * TS * xs;
}
// Unit = 4 output tiles of the lower triangle, one per wave, each with its own K range [ti, nt)
// (register-direct operands: the waves share no panel, only the unit's point-tile images for the
// epilogue).  Job table entry per unit (LU ints):
//   [0] unit id (-1: none)  [1] nimg  [2..6] image tiles  [7..10] ti per wave (-1: idle)
//   [11..14] tj  [15..18] image of ti  [19..22] image of tj
// The plan (lauum_plan) takes the lower tiles in row order, four consecutive tiles per unit: the
// waves' K ranges differ by at most one tile (99% of the wave time is MFMA work at nt = 32,
// against 92% for 2 x 2 units, whose diagonal units leave a wave idle and whose second tile row
// has 64 less K).  Such a unit needs up to 5 images (row tiles and column tiles); where 5 images
// would cost a workgroup per CU against 4 (d > 26 at two per CU, d > 63 at one), the plan falls
// back to 2 x 2 units.
__device__ __forceinline__ void lauum_unit(const DevBatch& db, int slot, const int* ju);
#ifndef GPRX_LAUUM_STAGGER
#define GPRX_LAUUM_STAGGER 0
#endif
__device__ __forceinline__ void lauum_body(const DevBatch& db) {
  int slot, job;
  if (!map_slot(db, db.nlj, slot, job)) return;
  const int* jb = db.lauum_order + (size_t)job * 2 * LU;
  GTS_L(0);
  const int nu = jb[LU] >= 0 ? 2 : 1;  // block-uniform: the folded short unit
  // stagger: half of the workgroups take their short unit first, so that the two workgroups on a
  // CU (one wave each per SIMD) reach their epilogues at different times
  const int sw = nu == 2 && (GPRX_LAUUM_STAGGER == 1 ? ((blockIdx.x >> 8) & 1)
                                                      : GPRX_LAUUM_STAGGER == 2 ? (__popc(blockIdx.x * 0x9E3779B1u) & 1) : 0);
  lauum_unit(db, slot, jb + (sw ? LU : 0));
  if (nu == 2) {
    __syncthreads();  // the first unit's LDS images and partials are consumed
    lauum_unit(db, slot, jb + (sw ? 0 : LU));
  }
}
__device__ __forceinline__ void lauum_unit(const DevBatch& db, int slot, const int* ju) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int d = db.d, tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int xs = db.xs, xt = TS * xs;  // point-tile image: [64][xs]
  const int nimg = ju[1];
  double* sp = sm;                      // [4][SPW]
  double* als = sp + 4 * SPW;           // [nimg][64] alpha of the image points
  double* img = als + 5 * TS;           // [nimg][64][xs]
  const int nt = db.nt;
  const double* X = db.Xc + (size_t)slot * db.Npad * xs;
  const double* al = db.alpha + (size_t)slot * db.Npad;
  const int ti = ju[7 + w], tj = ju[11 + w];
  const bool active = ti >= 0;
  const int l = tid & 63, lr = l & 15, lk = l >> 4;
  d4 acc[QM][QN];
  acc4_zero(acc);
  const size_t ld = db.ld, so = (size_t)slot * db.mat;
#ifdef GPRX_STAMPS
  const Stamp st0 = stamp_now();
#endif
  [[maybe_unused]] const int gu = (ju - db.lauum_order) % (2 * LU) == 0 ? 0 : 1;  // the job's first or second unit
  GTS_L(1 + 3 * gu);
  if (active) {  // wave-uniform: diagonal tiles form only their lower blocks
    const double* Ap = db.Mt + so + (size_t)ti * TS * ld + ti * TS;
    // global addressing here: the buffer-load form (k_gemm's) measured 0.15 ms slower in this kernel
    // (11.60 / 11.66 / 11.53 against 11.41 / 11.47 / 11.44 ms, same box, bit-identical output)
    if (ti == tj) mma_64x64_m<TRI_AB_FIRST, false>(acc, Ap, ld, Ap, ld, (nt - ti) * TS);
    else mma_64x64_m<TRI_A_FIRST, false>(acc, Ap, ld, db.Mt + so + (size_t)ti * TS * ld + tj * TS, ld, (nt - ti) * TS);
  }
  GTS_L(2 + 3 * gu);
#ifdef GPRX_STAMPS
  if (active && (ju - db.lauum_order) % (2 * LU) == 0) {  // the job's first (long) unit
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp_store(0, st0, stamp_now());
  }
#endif
  // the unit's point images by LDS-DMA after the main loop: issued before it, they sit ahead of
  // the first stage's loads in the wave's in-order load counter and delay the first MFMA
  for (int i = 0; i < nimg; ++i) dma_tile(img + i * xt, X + (size_t)ju[2 + i] * xt, xt);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA landed
  __syncthreads();                                   // ... and every other wave's
  GTS_D(gu, 4);
  double sf = 0.0, tr = 0.0;
  double* spw = sp + w * SPW;
  for (int e = l; e < SPW; e += 64) spw[e] = 0.0;
  const double* P = db.params + (size_t)slot * db.pst;
  for (int e = tid; e < nimg * TS; e += NTHR) als[e] = al[ju[2 + (e >> 6)] * TS + (e & 63)];
  __syncthreads();
  GTS_D(gu, 5);
  if (active) {
    const double sf2 = P[d];
    const int ir = ju[15 + w], ic = ju[19 + w];
    const double* xr = img + ir * xt;  // [r][xs]
    const double* xc = img + ic * xt;  // [c][xs]
    const double* ar = als + ir * TS;
    const double* ac = als + ic * TS;
    // G in place of acc, with Kf read from K's lower tile (ti, tj) as the Gram wrote it (the same
    // kernel values the factorisation used); only gi > gj is used: the diagonal (Kf + noise) is
    // never loaded, G_rr = W_rr sf2 / 2 analytically
    const double* Kf = db.K + so + (size_t)(tj * TS) * ld + ti * TS;
    const size_t ldk = ld;
#pragma unroll
    for (int a = 0; a < QM; ++a) {
      double kf[QN][4];
#pragma unroll
      for (int b = 0; b < QN; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) kf[b][q] = Kf[(size_t)(16 * b + lk + 4 * q) * ldk + 16 * a + lr];
#pragma unroll
      for (int b = 0; b < QN; ++b) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = 16 * a + lr, c = 16 * b + lk + 4 * q;
          const int gi = ti * TS + r, gj = tj * TS + c;
          double G = 0.0;
          if (gi < db.N && gj < db.N && gi >= gj) {
            const double W = ar[r] * ac[c] - acc[a][b][q];
            if (gi == gj) {
              G = 0.5 * (W * sf2);
              tr += W;
            } else {
              G = W * kf[b][q];
            }
            sf += G;
          }
          acc[a][b][q] = G;
        }
      }
    }
    GTS_D(gu, 6);
    // row sums R (row 16a + lr over the tile's 64 columns), column sums C (column 16b + lk + 4q
    // over the 64 rows)
    double R[QM], Cs[QN][4];
#pragma unroll
    for (int a = 0; a < QM; ++a) {
      double s = 0.0;
#pragma unroll
      for (int b = 0; b < QN; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) s += acc[a][b][q];
      s += __shfl_xor(s, 16);
      s += __shfl_xor(s, 32);
      R[a] = s;
    }
#pragma unroll
    for (int b = 0; b < QN; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        Cs[b][q] = row_sum16((acc[0][b][q] + acc[1][b][q]) + (acc[2][b][q] + acc[3][b][q]));
      }
    const int H = (d + 15) >> 4;
#pragma unroll 1
    for (int h = 0; h < H; ++h) {
      // A operand: x of column point c = 16b + 4q + lk, dimension pA = 16h + lr (clamped to a
      // finite image value for pA >= d: those Q columns and t2 lanes are never stored)
      const int pA = 16 * h + lr, pAc = pA < d ? pA : d - 1;
      double xa[QN][4];
      double t2 = 0.0;  // sum_c x_{pA,c}^2 C_c over this lane's 16 columns
#pragma unroll
      for (int b = 0; b < QN; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          xa[b][q] = xc[(16 * b + 4 * q + lk) * xs + pAc];
          t2 = fma(xa[b][q] * xa[b][q], Cs[b][q], t2);
        }
      double t13[4] = {0.0, 0.0, 0.0, 0.0};  // dims p = 16h + lk + 4q'
#pragma unroll
      for (int a = 0; a < QM; ++a) {
        d4 Q = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int b = 0; b < QN; ++b)
#pragma unroll
          for (int q = 0; q < 4; ++q) Q = mfma(xa[b][q], acc[a][b][q], Q);
        // lane: row r = 16a + lr; Q[q'] = Q[r][16h + lk + 4q']
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int p = 16 * h + lk + 4 * qq;
          const double x = xr[(16 * a + lr) * xs + (p < d ? p : d - 1)];
          t13[qq] = fma(x, fma(x, R[a], -2.0 * Q[qq]), t13[qq]);
        }
      }
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) t13[qq] = row_sum16(t13[qq]);
      t2 += __shfl_xor(t2, 16);
      t2 += __shfl_xor(t2, 32);
      if (lr == 0) {
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int p = 16 * h + lk + 4 * qq;
          if (p < d) spw[p] = t13[qq];
        }
      }
      __builtin_amdgcn_wave_barrier();
      if (lk == 0 && pA < d) spw[pA] += t2;
      __builtin_amdgcn_wave_barrier();
    }
  }
  GTS_D(gu, 7);
  sf = wave_sum(sf);
  tr = wave_sum(tr);
  if (l == 0) {
    spw[d] = sf;
    spw[d + 1] = tr;
  }
  __syncthreads();
  double* out = db.grad_part + ((size_t)slot * db.ngu + ju[0]) * db.gps;
  for (int e = tid; e < d + 2; e += NTHR)
    out[e] = ((sp[e] + sp[SPW + e]) + sp[2 * SPW + e]) + sp[3 * SPW + e];
  GTS_L(3 + 3 * gu);
}
__global__ __launch_bounds__(NTHR) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_lauum_grad(DevBatch db) {
  lauum_body(db);
}
// workgroups per CU that an LDS size allows (2 at most: the kernel's VGPRs)
static int lauum_wgs(size_t bytes) {
  const size_t cu = 160 * 1024;
  return bytes > cu ? 0 : (int)std::min<size_t>(2, cu / bytes);
}
int lauum_plan(int nt, int d, int* nunits, int* nimg, int* out) {
  const int xs = d | 1;
  const size_t b4 = lauum_lds_dbl(xs, 4) * sizeof(double), b5 = lauum_lds_dbl(xs, 5) * sizeof(double);
  const bool rows = lauum_wgs(b5) >= lauum_wgs(b4) && lauum_wgs(b5) > 0;
  // units in decreasing K order (K = nt - first row), each as its 4 (ti, tj) (ti = -1: idle wave)
  std::vector<std::array<int, 8>> us;
  if (rows) {
    std::vector<std::pair<int, int>> t;
    for (int i = 0; i < nt; ++i)
      for (int j = 0; j <= i; ++j) t.push_back({i, j});
    for (size_t k = 0; k < t.size(); k += 4) {
      std::array<int, 8> u;
      for (int w = 0; w < 4; ++w) {
        const bool in = k + w < t.size();
        u[w] = in ? t[k + w].first : -1;
        u[4 + w] = in ? t[k + w].second : -1;
      }
      us.push_back(u);
    }
  } else {
    for (int pr = 0; pr < nt; pr += 2)
      for (int pc = 0; pc <= pr; pc += 2) {
        std::array<int, 8> u;
        for (int w = 0; w < 4; ++w) {
          const int i = pr + (w >> 1), j = pc + (w & 1);
          const bool in = i < nt && j <= i;
          u[w] = in ? i : -1;
          u[4 + w] = in ? j : -1;
        }
        us.push_back(u);
      }
  }
  const int n = (int)us.size(), nj = (n + 1) / 2;
  *nunits = n;
  *nimg = 0;
  auto fill = [&](int* e, int id) {  // one LU-int entry of unit id (-1: none)
    for (int k = 0; k < LU; ++k) e[k] = -1;
    if (id < 0) return;
    const std::array<int, 8>& u = us[id];
    int img[8], ni = 0;
    auto slot_of = [&](int tile) {
      for (int k = 0; k < ni; ++k)
        if (img[k] == tile) return k;
      img[ni] = tile;
      return ni++;
    };
    e[0] = id;
    for (int w = 0; w < 4; ++w) {
      e[7 + w] = u[w];
      e[11 + w] = u[4 + w];
      if (u[w] >= 0) {
        e[15 + w] = slot_of(u[w]);
        e[19 + w] = slot_of(u[4 + w]);
      }
    }
    e[1] = ni;  // <= 5: at most 2 row tiles (2 x 2: 2 rows, 2 columns) and 4 column tiles
    for (int k = 0; k < ni && k < 5; ++k) e[2 + k] = img[k];
    if (ni > 5) e[1] = -1;  // not reached; lauum_plan returns -1
    *nimg = std::max(*nimg, ni);
  };
  std::vector<int> tmp(2 * LU);
  for (int j = 0; j < nj; ++j) {
    const int a = j, b = (n - 1 - j != j) ? n - 1 - j : -1;  // the j-th longest + the j-th shortest
    int* e = out ? out + (size_t)j * 2 * LU : tmp.data();
    fill(e, a);
    fill(e + LU, b);
    if (e[1] < 0 || (b >= 0 && e[LU + 1] < 0)) return -1;
  }
  return nj;
}

// ============================================================================================
// Per slot: mll = -(y.alpha + logdet + N log 2pi)/2 ; gradient (d+2) in GaussianProcesses order
// [log sn, log ell_1..d, log sf].  grid = B
// ============================================================================================
__global__ __launch_bounds__(NTHR) void k_finalize(DevBatch db, int want_grad) {
  __shared__ double red[4];
  const int slot = blockIdx.x, tid = threadIdx.x, d = db.d;
  if (!slot_active(db, slot)) return;
  const double* y = db.Y + (size_t)slot * db.Npad;
  const double* al = db.alpha + (size_t)slot * db.Npad;
  double s = 0.0;
  for (int k = tid; k < db.N; k += NTHR) s = fma(y[k], al[k], s);
  s = wave_sum(s);
  if ((tid & 63) == 0) red[tid >> 6] = s;
  __syncthreads();
  double* out = db.out + (size_t)slot * (d + 3);
  if (tid == 0) {
    const double ya = ((red[0] + red[1]) + red[2]) + red[3];
    double ldt = 0.0;
    for (int k = 0; k < db.nt; ++k) ldt += db.logdet_part[(size_t)slot * db.nt + k];
    const double log2pi = 1.8378770664093453;  // log(2pi), Julia's log2π
    out[0] = -((ya + 2.0 * ldt) + log2pi * db.N) / 2.0;
  }
  if (want_grad) {
    // deterministic parallel reduction over the lauum units: 4 waves x 64 lanes stride the units,
    // one parameter at a time
    __shared__ double pr[4];
    const double* P = db.params + (size_t)slot * db.pst;
    const double* gp = db.grad_part + (size_t)slot * db.ngu * db.gps;
    for (int q = 0; q < d + 2; ++q) {
      double tot = 0.0;
      for (int t = tid; t < db.ngu; t += NTHR) tot += gp[(size_t)t * db.gps + q];
      tot = wave_sum(tot);
      __syncthreads();
      if ((tid & 63) == 0) pr[tid >> 6] = tot;
      __syncthreads();
      if (tid == 0) {
        tot = ((pr[0] + pr[1]) + pr[2]) + pr[3];
        if (q < d) out[2 + q] = P[q] * tot;       // d mll / d log ell_q = il2_q * S_q
        else if (q == d) out[2 + d] = 2.0 * tot;  // d mll / d log sf     = 2 S_f
        else out[1] = P[d + 2] * tot;             // d mll / d log sn     = sn2 tr(W)
      }
    }
  }
}

// ============================================================================================
// Prediction.
//   pred_cross: K*^T tile (64 test x 64 train) + partial means over the train tile.
//               grid = B * nt * mt
//   (pred_var : OP_PREDVAR of k_gemm, V = Linv K*, column sums of V^2)
//   pred_final: mu = sum mu_part, var = max(sf2 - sum var_part, 0).       grid = B
// ============================================================================================
template <int MODE>
__global__ __launch_bounds__(NTHR) void k_pred_cross(DevBatch db) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  __shared__ __attribute__((aligned(16))) double tab[128];  // exp_sf's table, as k_gram
  const int d = db.d, tid = threadIdx.x;
  double* xt = sm;
  double* xs = sm + d * CS;
  double* pw = sm + 2 * d * CS;
  int slot, t;
  if (!map_slot(db, db.nt * db.mt, slot, t)) return;
  const int ch = t / db.mt, mtile = t - ch * db.mt;
  const double* X = db.X + (size_t)slot * db.Npad * d;
  const double* Xq = db.Xs + (size_t)slot * db.Mpad * d;
  const double* P = db.params + (size_t)slot * db.pst;
  double* sc = pw + DMAX + 4;  // as k_gram (sqrt(il2 / 2): the sums are r/2)
  if (MODE == 1) {
    for (int e = tid; e < d; e += NTHR) sc[e] = sqrt(0.5 * P[e]);
    __syncthreads();
  }
  {  // as k_gram: no per-element division, buffer loads
    const __amdgpu_buffer_rsrc_t xr = buffer_rsrc(X, db.Npad * d * (int)sizeof(double));
    const __amdgpu_buffer_rsrc_t qr = buffer_rsrc(Xq, db.Mpad * d * (int)sizeof(double));
    const int bi = ch * TS * d * (int)sizeof(double), bj = mtile * TS * d * (int)sizeof(double);
    const int os = 8 * d * (int)sizeof(double);
    for (int p = tid & 31; p < d; p += 32) {
      const double s = MODE == 1 ? sc[p] : 1.0;
      double vi[TS / 8], vj[TS / 8];
      const int o0 = ((tid >> 5) * d + p) * (int)sizeof(double);
#pragma unroll
      for (int m = 0; m < TS / 8; ++m) {
        vi[m] = buffer_load_f64(xr, o0, bi + m * os);
        vj[m] = buffer_load_f64(qr, o0, bj + m * os);
      }
#pragma unroll
      for (int m = 0; m < TS / 8; ++m) {
        const int r = (tid >> 5) + 8 * m;
        xt[p * CS + r] = vi[m] * s;
        xs[p * CS + r] = vj[m] * s;
      }
    }
  }
  for (int e = tid; e < d + 3; e += NTHR) pw[e] = P[e];
  if (tid < 64) {  // as k_gram
    const double s2 = P[d], h = g_exp2tab[2 * tid], lo = g_exp2tab[2 * tid + 1];
    const double th = s2 * h;
    tab[2 * tid] = th;
    tab[2 * tid + 1] = fma(s2, h, -th) + s2 * lo;
  }
  __syncthreads();
  const ExpK ek = g_expk;
  // thread: 4 test points (4mb..) x 4 train points (4rb..)
  const int mb = tid & 15, rb = tid >> 4;
  double rr[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) rr[a][b] = 0.0;
  for (int p = 0; p < d; ++p) {
    const double2 u0 = *(const double2*)(xt + p * CS + 4 * rb);
    const double2 u1 = *(const double2*)(xt + p * CS + 4 * rb + 2);
    const double2 v0 = *(const double2*)(xs + p * CS + 4 * mb);
    const double2 v1 = *(const double2*)(xs + p * CS + 4 * mb + 2);
    const double av[4] = {u0.x, u0.y, u1.x, u1.y};
    const double bv[4] = {v0.x, v0.y, v1.x, v1.y};
    const double wgt = pw[p];
    double a2[4], b2[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      a2[a] = av[a] * av[a];
      b2[a] = bv[a] * bv[a];
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        if (MODE == 0) {
          rr[a][b] = wacc<0>(rr[a][b], av[a], a2[a], bv[b], b2[b], wgt);
        } else {  // as k_gram
          const double t = av[a] - bv[b];
          rr[a][b] = __builtin_fma(t, t, rr[a][b]);
        }
      }
  }
  double* KsT = db.KsT + (size_t)slot * db.Npad * db.Mpad;
  const double* al = db.alpha + (size_t)slot * db.Npad;
  const bool inner = (ch + 1) * TS <= db.N && (mtile + 1) * TS <= db.M;  // block-uniform
  double mp[4] = {0.0, 0.0, 0.0, 0.0};  // this thread's share of the partial means
#pragma unroll
  for (int a = 0; a < 4; ++a) {  // train point gt
    const int gt = ch * TS + 4 * rb + a;
    const double alt = al[gt];
    double kv[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int gm = mtile * TS + 4 * mb + b;
      const double fv = exp_sf(MODE == 1 ? -rr[a][b] : -rr[a][b] * 0.5, ek, tab);  // padded points: finite, selected away
      kv[b] = (inner || (gt < db.N && gm < db.M)) ? fv : 0.0;
      mp[b] = fma(kv[b], alt, mp[b]);
    }
    double* o = KsT + (size_t)gt * db.Mpad + mtile * TS + 4 * mb;
    *(double2*)o = make_double2(kv[0], kv[1]);
    *(double2*)(o + 2) = make_double2(kv[2], kv[3]);
  }
  // the tile's partial means mu_part[ch][m] = sum_{t in tile ch} K*^T[t][m] alpha_t (k_pred_final adds
  // the tiles): the 4 train points of the thread, then the 4 row groups of the wave, then the waves
  double* mup = sc + DMAX;  // [4 waves][64 test points]
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    mp[b] = sum_xor32(sum_xor16(mp[b]));
  }
  if ((tid & 63) < 16) {
#pragma unroll
    for (int b = 0; b < 4; ++b) mup[(tid >> 6) * TS + 4 * mb + b] = mp[b];
  }
  __syncthreads();
  if (tid < TS)
    db.mu_part[((size_t)slot * db.nt + ch) * db.Mpad + mtile * TS + tid] = ((mup[tid] + mup[TS + tid]) + mup[2 * TS + tid]) + mup[3 * TS + tid];
}


__global__ __launch_bounds__(NTHR) void k_pred_final(DevBatch db) {
  const int slot = blockIdx.x;
  const double sf2 = db.params[(size_t)slot * db.pst + db.d];
  for (int m = threadIdx.x; m < db.Mpad; m += NTHR) {
    double mu = 0.0, s = 0.0;
    for (int k = 0; k < db.nt; ++k) {
      mu += db.mu_part[((size_t)slot * db.nt + k) * db.Mpad + m];
      if (db.want_var) s += db.var_part[((size_t)slot * db.nt + k) * db.Mpad + m];
    }
    const double v = sf2 - s;
    db.out_mu[(size_t)slot * db.Mpad + m] = mu;
    db.out_var[(size_t)slot * db.Mpad + m] = db.want_var ? (v > 0.0 ? v : 0.0) : 0.0;
  }
}


// ============================================================================================
// Rollout in minimal coordinates (examples/utils/predictdynamics.jl:30-102, predictdynamicsmin):
// per trajectory, `steps` rounds of  obs = f(q_old, qdot_old);  qdot_cur_g = mu_g(obs) for each of
// the nc GPs;  (q_old, qdot_old) = (q_cur, qdot_cur);  q_cur += qdot_cur dt.  One workgroup per
// trajectory runs the whole rollout (the step chain is serial, so it is latency-bound; one launch
// instead of steps x nc predict calls).  mu_g = sum_j sf2 exp(-r_j/2) alpha_j with r_j summed as
// distij does (il2-weighted; k_pred_cross sums coordinates pre-scaled by sqrt(il2/2) instead),
// so a rollout step reproduces gprx_batch_predict's mean up to rounding: the distance sums', the
// exp's (libm's here, k_pred_cross's table exp_sf) and the order of the final sum.  The state updates use
// explicit round-to-nearest mul/add (no fma contraction), as the reference's Julia arithmetic.
// ============================================================================================
__device__ __forceinline__ double pick3(const double (&e)[3], int i) {
  return i == 0 ? e[0] : (i == 1 ? e[1] : (i == 2 ? e[2] : 0.0));
}

template <int MODE, int NT>
__global__ __launch_bounds__(NT) void k_rollout(RolloutArgs a) {
  constexpr int NW = NT / 64, U = NT >= 1024 ? 2 : 4;  // training points per thread in flight
  __shared__ double red[2][NW][2];
  const int t = blockIdx.x, tid = threadIdx.x, nc = a.nc, d = a.d;
  const RolloutGP* gp = a.gps + (size_t)a.group[t] * nc;
  double qo[2], vo[2], qc[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    qo[c] = c < nc ? a.start[(size_t)t * 2 * nc + 2 * c] : 0.0;
    vo[c] = c < nc ? a.start[(size_t)t * 2 * nc + 2 * c + 1] : 0.0;
    qc[c] = __dadd_rn(qo[c], __dmul_rn(a.dt, vo[c]));
  }
  const bool s0 = a.usesin && a.ang0, s1 = a.usesin && a.ang1;
  const int w0 = s0 ? 3 : 2;
  for (int step = 0; step < a.steps; ++step) {
    double e0[3], e1[3];
    e0[0] = s0 ? sin(qo[0]) : qo[0];
    e0[1] = s0 ? cos(qo[0]) : vo[0];
    e0[2] = s0 ? vo[0] : 0.0;
    e1[0] = s1 ? sin(qo[1]) : qo[1];
    e1[1] = s1 ? cos(qo[1]) : vo[1];
    e1[2] = s1 ? vo[1] : 0.0;
    double ov[6], ov2[6];
#pragma unroll
    for (int p = 0; p < 6; ++p) {
      ov[p] = p < w0 ? pick3(e0, p) : pick3(e1, p - w0);
      ov2[p] = ov[p] * ov[p];
    }
    double acc[2] = {0.0, 0.0};
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      if (g >= nc) break;
      const RolloutGP G = gp[g];
      double il2[6];
#pragma unroll
      for (int p = 0; p < 6; ++p) il2[p] = p < d ? G.params[p] : 0.0;
      const double sf2 = G.params[d];
      double s = 0.0;
      // points j = tid + NT k in increasing k (the same order as a plain strided loop), U at a time
      for (int j0 = tid; j0 < G.N; j0 += U * NT) {
        double xv[U][6], al[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int j = j0 + u * NT;
          const bool ok = j < G.N;
          const double* x = G.X + (size_t)(ok ? j : 0) * d;
#pragma unroll
          for (int p = 0; p < 6; ++p) xv[u][p] = p < d ? x[p] : 0.0;
          al[u] = ok ? G.alpha[j] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          double r = 0.0;
#pragma unroll
          for (int p = 0; p < 6; ++p)
            if (p < d) r = wacc<MODE>(r, xv[u][p], xv[u][p] * xv[u][p], ov[p], ov2[p], il2[p]);
          if (j0 + u * NT < G.N) s = fma(sf2 * exp(-r * 0.5), al[u], s);
        }
      }
      acc[g] = wave_sum(s);
    }
    const int par = step & 1;
    if ((tid & 63) == 0) {
      red[par][tid >> 6][0] = acc[0];
      red[par][tid >> 6][1] = acc[1];
    }
    __syncthreads();  // red[par] is rewritten two steps later, after this step's reads
    double pred[2];
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      double v = red[par][0][g];
#pragma unroll
      for (int w = 1; w < NW; ++w) v += red[par][w][g];
      pred[g] = v;
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      qo[c] = qc[c];
      vo[c] = pred[c];
      qc[c] = __dadd_rn(qc[c], __dmul_rn(pred[c], a.dt));
    }
  }
  if (tid == 0)
    for (int c = 0; c < nc; ++c) {
      a.out[(size_t)t * 2 * nc + 2 * c] = qc[c];
      a.out[(size_t)t * 2 * nc + 2 * c + 1] = vo[c];
    }
}

// ---------------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------------
static size_t gram_lds(int d) { return (size_t)(2 * d * CS + DMAX + 4) * sizeof(double); }  // + k_gram's static table
static size_t lauum_lds(const DevBatch& b) { return lauum_lds_dbl(b.xs, b.nimg) * sizeof(double); }
static size_t cross_lds(int d) { return (size_t)(2 * d * CS + 2 * DMAX + 4 + 4 * TS) * sizeof(double); }  // + the static table

// Dynamic-LDS limits above the 64 KB default, for the current device.  Called once per device by
// gprx_ctx_create (std::call_once per device index) before any launch, so concurrent contexts on
// other threads never launch a kernel whose attribute is not yet set.
void set_kernel_attributes() {
  for (const void* f : {(const void*)k_gram<0>, (const void*)k_gram<1>})
    (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)gram_lds(DMAX));
  (void)hipFuncSetAttribute((const void*)k_lauum_grad, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (const void* f : {(const void*)k_pred_cross<0>, (const void*)k_pred_cross<1>})
    (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)cross_lds(DMAX));
  for (const void* f : {(const void*)k_leaf9, (const void*)k_node8})
    (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)leaf9_lds_bytes());
  (void)hipFuncSetAttribute((const void*)k_node8h, hipFuncAttributeMaxDynamicSharedMemorySize, (int)leaf4_lds_bytes());
  for (const void* f : {(const void*)k_gemm<REV_A>, (const void*)k_gemm<REV_B>, (const void*)k_gemm<TRI_A_FIRST>})
    (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)linv21_lds_bytes());
  set_lbfgs_attributes();
}

void launch_gram(const DevBatch& b, hipStream_t s) {
  if (b.dist_mode == 0) hipLaunchKernelGGL(k_gram<0>, dim3(grid_blocks(b.B, b.ntl)), dim3(NTHR), gram_lds(b.d), s, b);
  else hipLaunchKernelGGL(k_gram<1>, dim3(grid_blocks(b.B, b.ntl)), dim3(NTHR), gram_lds(b.d), s, b);
}
__global__ __launch_bounds__(64) void k_params(DevBatch b) {
  const int slot = blockIdx.x * 64 + threadIdx.x;
  if (slot < b.B) derive_params(b, slot);
}
void launch_params(const DevBatch& b, hipStream_t s) { hipLaunchKernelGGL(k_params, dim3((b.B + 63) / 64), dim3(64), 0, s, b); }
void launch_center(const DevBatch& b, hipStream_t s) { hipLaunchKernelGGL(k_center, dim3(b.B), dim3(NTHR), 0, s, b); }
void launch_diag(const DevBatch& b, int jt, int upd, hipStream_t s) {
  hipLaunchKernelGGL(k_diag_f, dim3(b.B), dim3(NTHR), 0, s, b, jt, upd);
}
void launch_leaf(const DevBatch& b, int o, int n, int upd, hipStream_t s) {
  if (n == 4) {
    hipLaunchKernelGGL(k_leaf9, dim3(b.B), dim3(2 * NTHR), leaf9_lds_bytes(), s, b, o, upd);
    return;
  }
  hipLaunchKernelGGL(k_leaf, dim3(b.B), dim3(NTHR), 0, s, b, o, n, upd);
}
void launch_node8(const DevBatch& b, int o, int upd, hipStream_t s, bool four) {
  if (four) hipLaunchKernelGGL(k_node8h, dim3(b.B), dim3(NTHR), leaf4_lds_bytes(), s, b, o, upd);
  else hipLaunchKernelGGL(k_node8, dim3(b.B), dim3(2 * NTHR), leaf9_lds_bytes(), s, b, o, upd);
}
void launch_gemm(const DevBatch& b, const GemmGeom& g, hipStream_t s, const GemmGeom& g2) {
  if (g.op != OP_PREDVAR && g.n <= b.small_n) {  // small node: pair units, 64 x 32 waves
    int T = pair_op_units(g, b.nt, b.mt);
    if (g2.op != OP_NONE) T += pair_op_units(g2, b.nt, b.mt);
    hipLaunchKernelGGL(k_gemm_p, dim3(grid_blocks(b.B, T)), dim3(NTHR), 0, s, b, g, g2);
    return;
  }
  int T = op_units(g, b.nt, b.mt);
  if (g2.op != OP_NONE) T += op_units(g2, b.nt, b.mt);
  if (n8_plan(g, g2)) T = 2;  // gemm_body's fixed plan
  const size_t lds = (g.op == OP_LINV21 || g2.op == OP_LINV21) ? linv21_lds_bytes() : 0;
  if (g.op == OP_PREDVAR) hipLaunchKernelGGL(k_gemm_pv, dim3(grid_blocks(b.B, T)), dim3(NTHR), lds, s, b, g, g2);
  else if (g.op == OP_TRSM) hipLaunchKernelGGL(k_gemm<REV_B>, dim3(grid_blocks(b.B, T)), dim3(NTHR), lds, s, b, g, g2);
  else if (g.op == OP_LINV21) hipLaunchKernelGGL(k_gemm<REV_A>, dim3(grid_blocks(b.B, T)), dim3(NTHR), lds, s, b, g, g2);
  else hipLaunchKernelGGL(k_gemm<TRI_A_FIRST>, dim3(grid_blocks(b.B, T)), dim3(NTHR), lds, s, b, g, g2);
}
void launch_alpha(const DevBatch& b, hipStream_t s, int phase) {
  hipLaunchKernelGGL(k_alpha, dim3(grid_blocks(b.B, b.nt)), dim3(NTHR), 0, s, b, phase);
}
void launch_lauum_grad(const DevBatch& b, hipStream_t s) {
  hipLaunchKernelGGL(k_lauum_grad, dim3(grid_blocks(b.B, b.nlj)), dim3(NTHR), lauum_lds(b), s, b);
}
void launch_finalize(const DevBatch& b, int want_grad, hipStream_t s) {
  hipLaunchKernelGGL(k_finalize, dim3(b.B), dim3(NTHR), 0, s, b, want_grad);
}
void launch_pred_cross(const DevBatch& b, hipStream_t s) {
  const dim3 grid(grid_blocks(b.B, b.nt * b.mt));
  if (b.dist_mode == 0) hipLaunchKernelGGL(k_pred_cross<0>, grid, dim3(NTHR), cross_lds(b.d), s, b);
  else hipLaunchKernelGGL(k_pred_cross<1>, grid, dim3(NTHR), cross_lds(b.d), s, b);
}
void launch_pred_final(const DevBatch& b, hipStream_t s) {
  hipLaunchKernelGGL(k_pred_final, dim3(b.B), dim3(NTHR), 0, s, b);
}
void launch_rollout(const RolloutArgs& a, int dist_mode, hipStream_t s) {
  // 256 threads per trajectory for every T (measured: 512 is 0.04 ms faster for 100 trajectories,
  // 256 is 1.4x faster for 3200; a fixed size keeps each trajectory's sums independent of T)
  if (a.T <= 0) return;
  if (dist_mode == 0) hipLaunchKernelGGL((k_rollout<0, 256>), dim3(a.T), dim3(256), 0, s, a);
  else hipLaunchKernelGGL((k_rollout<1, 256>), dim3(a.T), dim3(256), 0, s, a);
}

}  // namespace gprx

#ifdef GPRX_GSTAMPS
// diagnostic build only: copy (reset = 0) or clear (reset = 1) the GEMM tile timeline
extern "C" int gprx_dbg_gts(unsigned long long* out, long long n, int reset) {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(gprx::g_gts)) != hipSuccess) return 3;
  const size_t bytes = std::min<size_t>((size_t)n * 8, sizeof(gprx::g_gts));
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  if (reset) return hipMemset(p, 0, sizeof(gprx::g_gts)) == hipSuccess ? 0 : 3;
  return hipMemcpy(out, p, bytes, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 3;
}
#endif
#ifdef GPRX_STAMPS
// diagnostic build only: copy (reset = 0) or clear (reset = 1) stamp region `which`
extern "C" int gprx_dbg_stamps(int which, unsigned long long* out, long long n, int reset) {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(gprx::g_stamps)) != hipSuccess) return 3;
  char* base = (char*)p + (size_t)which * sizeof(gprx::g_stamps[0]);
  const size_t bytes = std::min<size_t>((size_t)n * 8, sizeof(gprx::g_stamps[0]));
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  if (reset) return hipMemset(base, 0, sizeof(gprx::g_stamps[0])) == hipSuccess ? 0 : 3;
  return hipMemcpy(out, base, bytes, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 3;
}
#endif

