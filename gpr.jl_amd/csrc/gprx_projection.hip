// gprx_projection.hip -- maximal-coordinate rollout physics on the device (gfx950, fp64).
//
// projectv! (src/projections/implicitProjection.jl:80-107): Newton iteration on the KKT system
//     F = [I + reg  G^T; G  reg I],  f(s) = [-s_u + s_v + G^T lambda ; g(x3(s), q3(s))],
//     s <- s - F \ f(s)   until |f| < eps and |ds| < eps (or newtonIter iterations),
// with the joint constraints g and their velocity Jacobians G = dg/d(v, w) of ConstrainedDynamics
// 0.7.4 [ext, restated in oracle/projection_oracle.py]:
//     x3 = xk + v dt,  q3 = qk * wbar(w) * dt / 2,  wbar(w) = (sqrt(4/dt^2 - w.w), w)
//     translational: g = C R(qa3)^T (xb3 + R(qb3) pb - xa3) - C pa
//     rotational:    g = C Im(qa3^-1 * qb3)
// One wave (projectv) or one workgroup (the rollout) runs one trajectory's solve with F in LDS
// (n = 6 nb + nd <= 48 rows); each sub-joint's rows and Jacobian blocks are built by one lane of
// wave 0; the LU is LAPACK dgetf2's
// right-looking partial pivoting (first maximal |pivot|, reciprocal scaling, rank-1 update) and
// dgetrs' unit-lower / upper substitutions, as Julia's F \ f.
//
// predictdynamics (examples/utils/predictdynamics.jl:7-22) for many trajectories: one 256-thread
// workgroup per trajectory runs every step on the device -- the G GPs' mean predictions at the
// current CState (the training points split over the workgroup), getvw, the projection (its LU
// update over the whole workgroup), the projection error and updatestate!.
#include "gprx_internal.h"

namespace gprx {

namespace {

struct Qd {
  double w, x, y, z;
};
__device__ __forceinline__ Qd qmul(const Qd& p, const Qd& q) {
  return Qd{p.w * q.w - (p.x * q.x + p.y * q.y + p.z * q.z), p.w * q.x + q.w * p.x + (p.y * q.z - p.z * q.y),
            p.w * q.y + q.w * p.y + (p.z * q.x - p.x * q.z), p.w * q.z + q.w * p.z + (p.x * q.y - p.y * q.x)};
}
__device__ __forceinline__ Qd qconj(const Qd& q) { return Qd{q.w, -q.x, -q.y, -q.z}; }
// R(q) p = (q0^2 - |qv|^2) p + 2 qv (qv.p) + 2 q0 qv x p
__device__ __forceinline__ void rot(const Qd& q, const double* p, double* o) {
  const double c = q.w * q.w - (q.x * q.x + q.y * q.y + q.z * q.z);
  const double d = q.x * p[0] + q.y * p[1] + q.z * p[2];
  const double cx = q.y * p[2] - q.z * p[1], cy = q.z * p[0] - q.x * p[2], cz = q.x * p[1] - q.y * p[0];
  o[0] = c * p[0] + 2.0 * q.x * d + 2.0 * q.w * cx;
  o[1] = c * p[1] + 2.0 * q.y * d + 2.0 * q.w * cy;
  o[2] = c * p[2] + 2.0 * q.z * d + 2.0 * q.w * cz;
}
// d (R(q) p) / dq, 3 x 4 (columns w, x, y, z)
__device__ __forceinline__ void drot(const Qd& q, const double* p, double (&J)[3][4]) {
  const double qv[3] = {q.x, q.y, q.z};
  const double cx = q.y * p[2] - q.z * p[1], cy = q.z * p[0] - q.x * p[2], cz = q.x * p[1] - q.y * p[0];
  const double cr[3] = {cx, cy, cz};
  const double d = q.x * p[0] + q.y * p[1] + q.z * p[2];
  // -2 q0 [p]x
  const double sk[3][3] = {{0.0, -p[2], p[1]}, {p[2], 0.0, -p[0]}, {-p[1], p[0], 0.0}};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    J[i][0] = 2.0 * q.w * p[i] + 2.0 * cr[i];
#pragma unroll
    for (int j = 0; j < 3; ++j)
      J[i][1 + j] = -2.0 * p[i] * qv[j] + (i == j ? 2.0 * d : 0.0) + 2.0 * qv[i] * p[j] - 2.0 * q.w * sk[i][j];
  }
}
// Lmat(p): p * q = Lmat(p) q ; Rmat(q): p * q = Rmat(q) p
__device__ __forceinline__ void lmat(const Qd& p, double (&M)[4][4]) {
  M[0][0] = p.w; M[0][1] = -p.x; M[0][2] = -p.y; M[0][3] = -p.z;
  M[1][0] = p.x; M[1][1] = p.w;  M[1][2] = -p.z; M[1][3] = p.y;
  M[2][0] = p.y; M[2][1] = p.z;  M[2][2] = p.w;  M[2][3] = -p.x;
  M[3][0] = p.z; M[3][1] = -p.y; M[3][2] = p.x;  M[3][3] = p.w;
}
__device__ __forceinline__ void rmat(const Qd& q, double (&M)[4][4]) {
  M[0][0] = q.w; M[0][1] = -q.x; M[0][2] = -q.y; M[0][3] = -q.z;
  M[1][0] = q.x; M[1][1] = q.w;  M[1][2] = q.z;  M[1][3] = -q.y;
  M[2][0] = q.y; M[2][1] = -q.z; M[2][2] = q.w;  M[2][3] = q.x;
  M[3][0] = q.z; M[3][1] = q.y;  M[3][2] = -q.x; M[3][3] = q.w;
}
// getq3: ((qk * wbar(w)) * dt) / 2
__device__ __forceinline__ Qd wbar_step(const Qd& qk, const double* w, double dt) {
  const Qd wb{sqrt(4.0 / (dt * dt) - (w[0] * w[0] + w[1] * w[1] + w[2] * w[2])), w[0], w[1], w[2]};
  const Qd r = qmul(qk, wb);
  return Qd{r.w * dt / 2.0, r.x * dt / 2.0, r.y * dt / 2.0, r.z * dt / 2.0};
}
// d q3 / d w (4 x 3) = Lmat(qk) [-w^T / s ; I] dt / 2
__device__ __forceinline__ void dq3(const Qd& qk, const double* w, double dt, double (&D)[4][3]) {
  const double s = sqrt(4.0 / (dt * dt) - (w[0] * w[0] + w[1] * w[1] + w[2] * w[2]));
  double L[4][4];
  lmat(qk, L);
  double Wp[4][3] = {{-w[0] / s, -w[1] / s, -w[2] / s}, {1.0, 0.0, 0.0}, {0.0, 1.0, 0.0}, {0.0, 0.0, 1.0}};
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      double t = 0.0;
#pragma unroll
      for (int k = 0; k < 4; ++k) t += L[i][k] * Wp[k][j];
      D[i][j] = t * (dt / 2.0);
    }
}

// Per-trajectory mechanism state and the KKT workspace in LDS.
struct PState {
  double xk[PJ_MAXB][3], qk[PJ_MAXB][4];  // discrete pose (x2, q2)
  double xc[PJ_MAXB][3], qc[PJ_MAXB][4], vc[PJ_MAXB][3], wc[PJ_MAXB][3];
  double s[PJ_MAXN], su[6 * PJ_MAXB], f[PJ_MAXN], ds[PJ_MAXN];
  int status, it;
};
// The Newton matrix F and the LU's working copy A live in dynamic LDS sized for the mechanism
// (2 n (n + 1) doubles, n = 6 nb + nd; row i at i (n + 1)), so a small mechanism's workgroups are
// not limited to the largest one's LDS footprint.
__device__ __forceinline__ double* pj_lds() {
  extern __shared__ __attribute__((aligned(16))) double pj_dyn[];
  return pj_dyn;
}
#define PJ_F (pj_lds())
#define PJ_A (pj_lds() + (size_t)(ldf - 1) * ldf)
__host__ __device__ inline size_t pj_lds_bytes(int nb, int nd) {
  const size_t n = 6 * (size_t)nb + nd;
  return 2 * n * (n + 1) * sizeof(double);
}
__device__ __forceinline__ Qd ldq(const double* q) { return Qd{q[0], q[1], q[2], q[3]}; }

// x3, q3 of body b (1-based; 0 = origin) at the current solution s
__device__ __forceinline__ void pose3(const PState& P, int b, double dt, double* x, Qd& q) {
  if (b == 0) {
    x[0] = x[1] = x[2] = 0.0;
    q = Qd{1.0, 0.0, 0.0, 0.0};
    return;
  }
  const double* v = P.s + 6 * (b - 1);
  const double* w = v + 3;
  for (int k = 0; k < 3; ++k) x[k] = P.xk[b - 1][k] + v[k] * dt;
  q = wbar_step(ldq(P.qk[b - 1]), w, dt);
}

// One sub-joint's constraint rows (into f[n6 + row0 ..] when want_g) and, when want_jac, its
// Jacobian blocks into F (G rows and the transposed G^T columns).  Called by one lane.
__device__ void subjoint(PState& P, const SubJoint& J, int n6, int ldf, double dt, bool want_g, bool want_jac,
                         bool sym = true) {
  double xa[3], xb[3];
  Qd qa, qb;
  pose3(P, J.a, dt, xa, qa);
  pose3(P, J.b, dt, xb, qb);
  const Qd qac = qconj(qa);
  const int R = J.rows;
  double gm[3];  // the 3-vector before C
  double Gv_b[3][3], Gw_b[3][3], Gv_a[3][3], Gw_a[3][3];
  const double* wb = P.s + 6 * (J.b - 1) + 3;
  double Db[4][3];
  dq3(ldq(P.qk[J.b - 1]), wb, dt, Db);
  double Da[4][3];
  if (J.a > 0) dq3(ldq(P.qk[J.a - 1]), P.s + 6 * (J.a - 1) + 3, dt, Da);
  if (J.kind == 0) {  // translational
    double rpb[3], y[3], e[3];
    rot(qb, J.pb, rpb);
    for (int k = 0; k < 3; ++k) y[k] = xb[k] + rpb[k] - xa[k];
    rot(qac, y, e);
    for (int k = 0; k < 3; ++k) gm[k] = e[k] - J.pa[k];
    if (want_jac) {
      double RaT[3][3];  // R(qa)^T: column j = R(qa^-1) e_j
      for (int j = 0; j < 3; ++j) {
        const double ej[3] = {j == 0 ? 1.0 : 0.0, j == 1 ? 1.0 : 0.0, j == 2 ? 1.0 : 0.0};
        double c[3];
        rot(qac, ej, c);
        for (int i = 0; i < 3; ++i) RaT[i][j] = c[i];
      }
      double Jb[3][4];
      drot(qb, J.pb, Jb);
      double M[3][3];  // RaT drot(qb, pb) Db
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
          double t = 0.0;
          for (int k = 0; k < 3; ++k) {
            double u = 0.0;
            for (int m = 0; m < 4; ++m) u += Jb[k][m] * Db[m][j];
            t += RaT[i][k] * u;
          }
          M[i][j] = t;
        }
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
          Gv_b[i][j] = RaT[i][j] * dt;
          Gw_b[i][j] = M[i][j];
          Gv_a[i][j] = -RaT[i][j] * dt;
        }
      if (J.a > 0) {
        double Ja[3][4];
        drot(qac, y, Ja);
        for (int i = 0; i < 3; ++i)
          for (int j = 0; j < 3; ++j) {
            double t = 0.0;
            for (int m = 0; m < 4; ++m) t += Ja[i][m] * (m == 0 ? 1.0 : -1.0) * Da[m][j];
            Gw_a[i][j] = t;
          }
      }
    }
  } else {  // rotational
    const Qd r = qmul(qac, qb);
    gm[0] = r.x;
    gm[1] = r.y;
    gm[2] = r.z;
    if (want_jac) {
      double L[4][4];
      lmat(qac, L);
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
          double t = 0.0;
          for (int m = 0; m < 4; ++m) t += L[1 + i][m] * Db[m][j];
          Gw_b[i][j] = t;
          Gv_b[i][j] = 0.0;
          Gv_a[i][j] = 0.0;
        }
      if (J.a > 0) {
        double Rq[4][4];
        rmat(qb, Rq);
        for (int i = 0; i < 3; ++i)
          for (int j = 0; j < 3; ++j) {
            double t = 0.0;
            for (int m = 0; m < 4; ++m) t += Rq[1 + i][m] * (m == 0 ? 1.0 : -1.0) * Da[m][j];
            Gw_a[i][j] = t;
          }
      }
    }
  }
  for (int r = 0; r < R; ++r) {
    const int row = n6 + J.row0 + r;
    if (want_g) {
      double t = 0.0;
      for (int k = 0; k < 3; ++k) t += J.C[r][k] * gm[k];
      P.f[row] = t;
    }
    if (want_jac) {
      for (int side = 0; side < 2; ++side) {
        const int body = side ? J.a : J.b;
        if (body == 0) continue;
        const int c0 = 6 * (body - 1);
        for (int j = 0; j < 3; ++j) {
          double tv = 0.0, tw = 0.0;
          for (int k = 0; k < 3; ++k) {
            tv += J.C[r][k] * (side ? Gv_a[k][j] : Gv_b[k][j]);
            tw += J.C[r][k] * (side ? Gw_a[k][j] : Gw_b[k][j]);
          }
          PJ_F[row * ldf + c0 + j] = tv;
          PJ_F[row * ldf + c0 + 3 + j] = tw;
          if (sym) {
            PJ_F[(c0 + j) * ldf + row] = tv;
            PJ_F[(c0 + 3 + j) * ldf + row] = tw;
          }
        }
      }
    }
  }
}

__device__ __forceinline__ double readlane_dbl(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double wsum(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// f(s) upper part: -su + s_v + G^T lambda (G read from F's lower-left block), lanes over columns
__device__ __forceinline__ void residual_upper(PState& P, int n6, int nd, int ldf, int l) {
  if (l < n6) {
    double t = 0.0;
    for (int r = 0; r < nd; ++r) t += PJ_F[(n6 + r) * ldf + l] * P.s[n6 + r];
    P.f[l] = (-P.su[l] + P.s[l]) + t;
  }
}

template <int NW>
__device__ __forceinline__ void pj_sync() {
  if constexpr (NW == 1) {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  } else {
    __syncthreads();
  }
}

// A x = b by LAPACK dgetf2's right-looking LU with partial pivoting (first maximal |pivot|,
// reciprocal scaling, rank-1 update spread over the NW waves, one element per thread) and dgetrs'
// unit-lower / upper substitutions, as Julia's F \ f.  A (n x n, row stride ldf) in LDS is
// overwritten; b: lane l < n holds b_l on entry and x_l on exit (the same on every wave).  Returns
// true for an exactly singular pivot (b is then undefined).  All NW * 64 threads call.
template <int NW>
__device__ bool lu_solve(double* A, int n, int ldf, double& b) {
  constexpr int NT = 64 * NW;
  const int tid = threadIdx.x & (NT - 1), l = tid & 63;
  const bool w0 = tid < 64;
  bool singular = false;
  for (int k = 0; k < n; ++k) {
    // pivot: first row of maximal |a_ik|, i >= k (idamax)
    double v = (l >= k && l < n) ? fabs(A[l * ldf + k]) : -1.0;
    int idx = l;
    for (int o = 1; o < 64; o <<= 1) {
      const double v2 = __shfl_xor(v, o);
      const int i2 = __shfl_xor(idx, o);
      if (v2 > v || (v2 == v && i2 < idx)) {
        v = v2;
        idx = i2;
      }
    }
    const int p = idx;
    if (p != k) {  // swap rows k and p of A and of the right-hand side
      if (NW > 1) pj_sync<NW>();  // every wave has read column k
      for (int j = tid; j < n; j += NT) {
        const double t = A[k * ldf + j];
        A[k * ldf + j] = A[p * ldf + j];
        A[p * ldf + j] = t;
      }
      const double bk = readlane_dbl(b, k), bp = readlane_dbl(b, p);
      if (l == k) b = bp;
      if (l == p) b = bk;
    }
    pj_sync<NW>();
    const double akk = A[k * ldf + k];
    if (akk == 0.0) singular = true;
    const int m = n - 1 - k;
    if (akk != 0.0 && m > 0) {
      if (w0 && l > k && l < n)
        A[l * ldf + k] = fabs(akk) >= DBL_MIN ? A[l * ldf + k] * (1.0 / akk) : A[l * ldf + k] / akk;
      pj_sync<NW>();
      // trailing update A[i][j] -= l_i A[k][j], i, j in (k, n): element e = (i - k - 1) m + (j - k - 1)
      const int si = NT / m, sj = NT - si * m;
      int i = tid / m, j = tid - i * m;
      for (int e = tid; e < m * m; e += NT) {
        const int gi = k + 1 + i, gj = k + 1 + j;
        A[gi * ldf + gj] = A[gi * ldf + gj] - A[gi * ldf + k] * A[k * ldf + gj];
        i += si;
        j += sj;
        if (j >= m) {
          j -= m;
          ++i;
        }
      }
    }
    pj_sync<NW>();
  }
  if (singular) return true;
  // forward substitution (unit lower), then backward (upper), as dgetrs / dtrsm
  for (int k = 0; k < n; ++k) {
    const double bk = readlane_dbl(b, k);
    if (bk != 0.0 && l > k && l < n) b = b - bk * A[l * ldf + k];
  }
  for (int k = n - 1; k >= 0; --k) {
    const double ukk = A[k * ldf + k];
    double bk = readlane_dbl(b, k);
    if (bk != 0.0) {
      bk = bk / ukk;
      if (l == k) b = bk;
      if (l < k) b = b - bk * A[l * ldf + k];
    }
  }
  return false;
}

// projectv! on NW waves (all NW * 64 threads call).  P.s holds the predicted (v, w) per body on
// entry (lambda = 0 appended); leaves the projected (v, w) in P.s[0 .. 6nb).  P.xk / P.qk set.
// Wave 0 builds the constraints, Jacobians and residuals (one lane per sub-joint / row); the LU's
// trailing update is spread over every thread, one element each; pivot search, the right-hand
// side and the substitutions run redundantly on every wave (the same values), so no broadcast is
// needed.  Each element sees the same operations in the same order for any NW.
template <int NW>
__device__ void project(PState& P, const MechDev& M, double dt, double reg, double eps, int iters) {
  constexpr int NT = 64 * NW;
  const int tid = threadIdx.x & (NT - 1), l = tid & 63;
  const bool w0 = tid < 64;
  const int nb = M.nb, nd = M.nd, n6 = 6 * nb, n = n6 + nd, ldf = n + 1;
  for (int i = tid; i < n * ldf; i += NT) PJ_F[i] = 0.0;
  pj_sync<NW>();
  if (w0) {
    if (l < n6) P.su[l] = P.s[l];
    if (l >= n6 && l < n) P.s[l] = 0.0;
  }
  pj_sync<NW>();
  if (w0 && l < M.nsub) subjoint(P, M.sub[l], n6, ldf, dt, false, true);  // updateF!
  pj_sync<NW>();
  if (w0 && l < n) PJ_F[l * ldf + l] = (l < n6 ? 1.0 : 0.0) + reg;        // F += I * regularizer
  if (tid == 0) {
    P.status = 0;
    P.it = 0;
  }
  pj_sync<NW>();
  for (int it = 1; it <= iters; ++it) {
    if (w0 && l < M.nsub) subjoint(P, M.sub[l], n6, ldf, dt, true, true);  // updateF! + g(mechanism)
    pj_sync<NW>();
    if (w0) residual_upper(P, n6, nd, ldf, l);
    pj_sync<NW>();
    // ---- ds = F \ f: LU with partial pivoting of a working copy A (F keeps the Newton matrix;
    // its G blocks are rebuilt by the next updateF!)
    for (int i = tid; i < n * ldf; i += NT) PJ_A[i] = PJ_F[i];
    double b = l < n ? P.f[l] : 0.0;
    pj_sync<NW>();
    if (lu_solve<NW>(PJ_A, n, ldf, b)) {  // Julia's F \ f throws SingularException: the trajectory stops
      if (tid == 0) P.status = 1;
      pj_sync<NW>();
      return;
    }
    // s -= ds, updateMechanism!
    if (w0 && l < n) {
      P.ds[l] = b;
      P.s[l] = P.s[l] - b;
    }
    pj_sync<NW>();
    // convergence: |f(s_new)| (with the iteration's G) and |ds|
    if (w0 && l < M.nsub) subjoint(P, M.sub[l], n6, ldf, dt, true, false);
    pj_sync<NW>();
    if (w0) residual_upper(P, n6, nd, ldf, l);
    pj_sync<NW>();
    const double fv = l < n ? P.f[l] : 0.0, dv = l < n ? P.ds[l] : 0.0;
    const double nf = sqrt(wsum(fv * fv)), nds = sqrt(wsum(dv * dv));
    if (tid == 0) P.it = it;
    pj_sync<NW>();
    if (nf < eps && nds < eps) break;
  }
}

// setstates! (+ discretizestate!, setsolution!) from a CState
__device__ void set_states(PState& P, const double* cs, int nb, double dt, int l) {
  if (l < nb) {
    const double* c = cs + 13 * l;
    for (int k = 0; k < 3; ++k) {
      P.xc[l][k] = c[k];
      P.vc[l][k] = c[7 + k];
      P.wc[l][k] = c[10 + k];
      P.xk[l][k] = c[k] + c[7 + k] * dt;
    }
    for (int k = 0; k < 4; ++k) P.qc[l][k] = c[3 + k];
    const Qd q = wbar_step(ldq(P.qc[l]), P.wc[l], dt);
    P.qk[l][0] = q.w;
    P.qk[l][1] = q.x;
    P.qk[l][2] = q.y;
    P.qk[l][3] = q.z;
  }
}
// updatestate! with the solution (v, w) in P.s
__device__ void update_state(PState& P, int nb, double dt, int l) {
  if (l < nb) {
    const double* v = P.s + 6 * l;
    const double* w = v + 3;
    for (int k = 0; k < 3; ++k) {
      P.xc[l][k] = P.xk[l][k];
      P.vc[l][k] = v[k];
      P.wc[l][k] = w[k];
      P.xk[l][k] = P.xk[l][k] + v[k] * dt;
    }
    for (int k = 0; k < 4; ++k) P.qc[l][k] = P.qk[l][k];
    const Qd q = wbar_step(ldq(P.qk[l]), w, dt);
    P.qk[l][0] = q.w;
    P.qk[l][1] = q.x;
    P.qk[l][2] = q.y;
    P.qk[l][3] = q.z;
  }
}
__device__ __forceinline__ double cstate_at(const PState& P, int i) {
  const int b = i / 13, k = i - 13 * b;
  if (k < 3) return P.xc[b][k];
  if (k < 7) return P.qc[b][k - 3];
  if (k < 10) return P.vc[b][k - 7];
  return P.wc[b][k - 10];
}

// ---- one variational-integrator step: ConstrainedDynamics 0.7.4 newton! (restated in gprx/vi.py,
// which documents the equations): per body, with the current state (x1, q1, v1, w1) and the discrete
// pose x2 = x1 + v1 dt, q2 = q1 wbar(w1) dt/2, Newton on s = (v2, w2 per body, lambda) for
//     m ((v2 - v1)/dt + g e_z) - Gpos_x^T lambda = 0
//     sq2 J w2 + w2 x J w2 - (sq1 J w1 - w1 x J w1) - Gpos_phi^T lambda = 0,  sq = sqrt(4/dt^2 - w.w)
//     g(x3, q3) = 0,  x3 = x2 + v2 dt,  q3 = q2 wbar(w2) dt/2
// Gpos = dg/d(x, phi) at pose 2 (phi: q -> q (1, phi)), fixed during the solve; the constraint rows'
// velocity Jacobian is the projection's (subjoint).  One wave per state; the Newton matrix is
// rebuilt in LDS every iteration and factored in place (lu_solve).
// R(q) as gprx/vi.py rotmat (unit quaternions)
__device__ __forceinline__ void rotm(const Qd& q, double (&R)[3][3]) {
  const double w = q.w, x = q.x, y = q.y, z = q.z;
  R[0][0] = w * w + x * x - y * y - z * z;
  R[0][1] = 2.0 * (x * y - w * z);
  R[0][2] = 2.0 * (x * z + w * y);
  R[1][0] = 2.0 * (x * y + w * z);
  R[1][1] = w * w - x * x + y * y - z * z;
  R[1][2] = 2.0 * (y * z - w * x);
  R[2][0] = 2.0 * (x * z - w * y);
  R[2][1] = 2.0 * (y * z + w * x);
  R[2][2] = w * w - x * x - y * y + z * z;
}
__device__ __forceinline__ void pose2(const PState& P, int b, double* x, Qd& q) {
  if (b == 0) {
    x[0] = x[1] = x[2] = 0.0;
    q = Qd{1.0, 0.0, 0.0, 0.0};
    return;
  }
  for (int k = 0; k < 3; ++k) x[k] = P.xk[b - 1][k];
  q = ldq(P.qk[b - 1]);
}
// one sub-joint's rows of Gpos = dg/d(x_1, phi_1, ..., x_nb, phi_nb) at pose 2 (gprx/vi.py jac_phi)
// into G (row-major, nd x n6); called by one lane
__device__ void subjoint_pose_jac(const PState& P, const SubJoint& J, int n6, double* G) {
  double xa[3], xb[3];
  Qd qa, qb;
  pose2(P, J.a, xa, qa);
  pose2(P, J.b, xb, qb);
  double Bx_b[3][3], Bp_b[3][3], Bx_a[3][3], Bp_a[3][3];  // the 3 x 3 blocks before C
  if (J.kind == 0) {  // translational: g = C (R(qa)^T (xb + R(qb) pb - xa) - pa)
    double Ra[3][3], Rb[3][3];
    rotm(qa, Ra);
    rotm(qb, Rb);
    double y[3], u[3];
    for (int i = 0; i < 3; ++i) y[i] = xb[i] + (Rb[i][0] * J.pb[0] + Rb[i][1] * J.pb[1] + Rb[i][2] * J.pb[2]) - xa[i];
    for (int i = 0; i < 3; ++i) u[i] = Ra[0][i] * y[0] + Ra[1][i] * y[1] + Ra[2][i] * y[2];
    const double spb[3][3] = {{0.0, -J.pb[2], J.pb[1]}, {J.pb[2], 0.0, -J.pb[0]}, {-J.pb[1], J.pb[0], 0.0}};
    const double su[3][3] = {{0.0, -u[2], u[1]}, {u[2], 0.0, -u[0]}, {-u[1], u[0], 0.0}};
    double RbS[3][3];  // R(qb) (-2 [pb]x)
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) RbS[i][j] = -2.0 * (Rb[i][0] * spb[0][j] + Rb[i][1] * spb[1][j] + Rb[i][2] * spb[2][j]);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        Bx_b[i][j] = Ra[j][i];
        Bp_b[i][j] = Ra[0][i] * RbS[0][j] + Ra[1][i] * RbS[1][j] + Ra[2][i] * RbS[2][j];
        Bx_a[i][j] = -Ra[j][i];
        Bp_a[i][j] = 2.0 * su[i][j];
      }
  } else {  // rotational: g = C Im(qa^-1 qb); d/dphi_b = Lmat(rq)[1:,1:], d/dphi_a = -Rmat(rq)[1:,1:]
    const Qd r = qmul(qconj(qa), qb);
    const double rv[3] = {r.x, r.y, r.z};
    const double sr[3][3] = {{0.0, -rv[2], rv[1]}, {rv[2], 0.0, -rv[0]}, {-rv[1], rv[0], 0.0}};
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        Bx_b[i][j] = 0.0;
        Bx_a[i][j] = 0.0;
        Bp_b[i][j] = (i == j ? r.w : 0.0) + sr[i][j];
        Bp_a[i][j] = -((i == j ? r.w : 0.0) - sr[i][j]);
      }
  }
  for (int rr = 0; rr < J.rows; ++rr) {
    double* g = G + (size_t)(J.row0 + rr) * n6;
    for (int side = 0; side < 2; ++side) {
      const int body = side ? J.a : J.b;
      if (body == 0) continue;
      const int c0 = 6 * (body - 1);
      for (int j = 0; j < 3; ++j) {
        double tx = 0.0, tp = 0.0;
        for (int k = 0; k < 3; ++k) {
          tx += J.C[rr][k] * (side ? Bx_a[k][j] : Bx_b[k][j]);
          tp += J.C[rr][k] * (side ? Bp_a[k][j] : Bp_b[k][j]);
        }
        g[c0 + j] = tx;
        g[c0 + 3 + j] = tp;
      }
    }
  }
}
// the dynamics rows of the residual, lane j < n6: body b = j / 6
__device__ __forceinline__ double vi_dyn_row(const PState& P, const MechDev& M, const double (*mom1)[3], const double* G,
                                             int n6, int nd, double dt, double grav, int j) {
  const int b = j / 6, c = j - 6 * b;
  const double* v2 = P.s + 6 * b;
  const double* w2 = v2 + 3;
  double d;
  if (c < 3) {
    d = M.m[b] * ((v2[c] - P.vc[b][c]) / dt + (c == 2 ? grav : 0.0));
  } else {
    const int k = c - 3;
    double Jw[3];
    for (int i = 0; i < 3; ++i) Jw[i] = M.J[b][i][0] * w2[0] + M.J[b][i][1] * w2[1] + M.J[b][i][2] * w2[2];
    const double sq2 = sqrt(4.0 / (dt * dt) - (w2[0] * w2[0] + w2[1] * w2[1] + w2[2] * w2[2]));
    const double cr = k == 0 ? w2[1] * Jw[2] - w2[2] * Jw[1] : (k == 1 ? w2[2] * Jw[0] - w2[0] * Jw[2] : w2[0] * Jw[1] - w2[1] * Jw[0]);
    d = (sq2 * Jw[k] + cr) - mom1[b][k];
  }
  double t = 0.0;
  for (int r = 0; r < nd; ++r) t += G[(size_t)r * n6 + j] * P.s[n6 + r];
  return d - t;
}

}  // namespace

// ---- projectv! for T independent mechanism states: one wave each ------------------------------
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_project(ProjArgs a) {
  __shared__ PState P;
  const int t = blockIdx.x, l = threadIdx.x;
  const int nb = a.mech.nb, n6 = 6 * nb;
  set_states(P, a.cs + (size_t)t * 13 * nb, nb, a.dt, l);
  if (l < n6) P.s[l] = a.vw[(size_t)t * n6 + l];
  __builtin_amdgcn_wave_barrier();
  project<1>(P, a.mech, a.dt, a.reg, a.eps, a.iters);
  __builtin_amdgcn_wave_barrier();
  if (l < n6) a.out[(size_t)t * n6 + l] = P.status ? NAN : P.s[l];
  if (l == 0) {
    a.iters_out[t] = P.it;
    a.status[t] = P.status;
  }
}

// ---- one variational-integrator step for T independent states: one wave each --------------------
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_vi_step(ViArgs a) {
  __shared__ PState P;
  __shared__ double mom1[PJ_MAXB][3];
  const int t = blockIdx.x, l = threadIdx.x;
  const MechDev& M = a.mech;
  const int nb = M.nb, nd = M.nd, n6 = 6 * nb, n = n6 + nd, ldf = n + 1;
  const double dt = a.dt;
  double* A = PJ_F;                         // the Newton matrix, rebuilt and factored each iteration
  double* G = PJ_F + (size_t)n * ldf;       // Gpos (nd x n6), fixed
  set_states(P, a.cs + (size_t)t * 13 * nb, nb, dt, l);
  if (l < nb) {  // (sq1 I - [w1 x]) J w1; setsolution!: (v2, w2) start at the current velocities
    const double* w1 = P.wc[l];
    double Jw[3];
    for (int i = 0; i < 3; ++i) Jw[i] = M.J[l][i][0] * w1[0] + M.J[l][i][1] * w1[1] + M.J[l][i][2] * w1[2];
    const double sq1 = sqrt(4.0 / (dt * dt) - (w1[0] * w1[0] + w1[1] * w1[1] + w1[2] * w1[2]));
    const double cr[3] = {w1[1] * Jw[2] - w1[2] * Jw[1], w1[2] * Jw[0] - w1[0] * Jw[2], w1[0] * Jw[1] - w1[1] * Jw[0]};
    for (int i = 0; i < 3; ++i) {
      mom1[l][i] = sq1 * Jw[i] - cr[i];
      P.s[6 * l + i] = P.vc[l][i];
      P.s[6 * l + 3 + i] = w1[i];
    }
  }
  if (l >= n6 && l < n) P.s[l] = 0.0;
  for (int i = l; i < nd * n6; i += 64) G[i] = 0.0;
  __builtin_amdgcn_wave_barrier();
  if (l < M.nsub) subjoint_pose_jac(P, M.sub[l], n6, G);
  __builtin_amdgcn_wave_barrier();
  int status = 1, it = 0;
  for (int k = 1; k <= a.iters; ++k) {
    // ---- the Newton matrix and the residual at the current solution
    for (int i = l; i < n * ldf; i += 64) A[i] = 0.0;
    __builtin_amdgcn_wave_barrier();
    if (l < M.nsub) {
      subjoint(P, M.sub[l], n6, ldf, dt, true, true, false);  // g(x3, q3) and dg/d(v2, w2)
    } else if (l < M.nsub + 9 * nb) {  // d/dw2 [(sq2 I + [w2 x]) J w2] (gprx/vi.py)
      const int e = l - M.nsub, b = e / 9, i = (e - 9 * b) / 3, kk = e - 9 * b - 3 * i;
      const double* w2 = P.s + 6 * b + 3;
      double Jw[3];
      for (int q = 0; q < 3; ++q) Jw[q] = M.J[b][q][0] * w2[0] + M.J[b][q][1] * w2[1] + M.J[b][q][2] * w2[2];
      const double sq2 = sqrt(4.0 / (dt * dt) - (w2[0] * w2[0] + w2[1] * w2[1] + w2[2] * w2[2]));
      const double sw[3][3] = {{0.0, -w2[2], w2[1]}, {w2[2], 0.0, -w2[0]}, {-w2[1], w2[0], 0.0}};
      const double sj[3][3] = {{0.0, -Jw[2], Jw[1]}, {Jw[2], 0.0, -Jw[0]}, {-Jw[1], Jw[0], 0.0}};
      const double swJ = sw[i][0] * M.J[b][0][kk] + sw[i][1] * M.J[b][1][kk] + sw[i][2] * M.J[b][2][kk];
      A[(6 * b + 3 + i) * ldf + 6 * b + 3 + kk] = ((sq2 * M.J[b][i][kk] + swJ) - sj[i][kk]) - Jw[i] * w2[kk] / sq2;
    } else if (l < M.nsub + 12 * nb) {
      const int e = l - M.nsub - 9 * nb, b = e / 3, c = e - 3 * b;
      A[(6 * b + c) * ldf + 6 * b + c] = M.m[b] / dt;
    }
    for (int e = l; e < n6 * nd; e += 64) {  // -Gpos^T (upper right), -reg I (lower right)
      const int j = e / nd, r = e - j * nd;
      A[j * ldf + n6 + r] = -G[(size_t)r * n6 + j];
    }
    if (l < nd && a.reg != 0.0) A[(n6 + l) * ldf + n6 + l] = -a.reg;
    __builtin_amdgcn_wave_barrier();
    if (l < n6) P.f[l] = vi_dyn_row(P, M, mom1, G, n6, nd, dt, a.grav, l);
    __builtin_amdgcn_wave_barrier();
    // a system that is not finite (|w| beyond 2/dt: the reference's sqrt throws a DomainError) or is
    // singular (SingularException) fails the state: its row is NaN
    bool fin = l < n ? isfinite(P.f[l]) : true;
    for (int i = l; i < n * ldf; i += 64) fin = fin && isfinite(A[i]);
    if (__any(!fin)) {
      status = 2;
      break;
    }
    double bvec = l < n ? P.f[l] : 0.0;
    if (lu_solve<1>(A, n, ldf, bvec) || __any(l < n && !isfinite(bvec))) {
      status = 2;
      break;
    }
    if (l < n) {
      P.ds[l] = bvec;
      P.s[l] = P.s[l] - bvec;
    }
    it = k;
    __builtin_amdgcn_wave_barrier();
    // ---- convergence: |f(s_new)| and |ds|
    if (l < M.nsub) subjoint(P, M.sub[l], n6, ldf, dt, true, false, false);
    __builtin_amdgcn_wave_barrier();
    if (l < n6) P.f[l] = vi_dyn_row(P, M, mom1, G, n6, nd, dt, a.grav, l);
    __builtin_amdgcn_wave_barrier();
    const double fv = l < n ? P.f[l] : 0.0, dv = l < n ? P.ds[l] : 0.0;
    const double nf = sqrt(wsum(fv * fv)), nds = sqrt(wsum(dv * dv));
    if (nf < a.eps && nds < a.eps) {
      status = 0;
      break;
    }
  }
  double* o = a.out + (size_t)t * 13 * nb;
  for (int i = l; i < 13 * nb; i += 64) {
    const int b = i / 13, k = i - 13 * b;
    double v;
    if (k < 3) v = P.xk[b][k];
    else if (k < 7) v = P.qk[b][k - 3];
    else v = P.s[6 * b + (k - 7)];  // v2 (7..9), w2 (10..12)
    o[i] = status == 2 ? NAN : v;
  }
  if (l == 0) {
    a.iters_out[t] = it;
    a.status[t] = status;
  }
}

// ---- predictdynamics: one workgroup per trajectory, every step on the device --------------------
template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_rollout_max(RolloutMaxArgs a) {
  constexpr int NT = 256, NW = NT / 64;
  __shared__ PState P;
  __shared__ double obs[13 * PJ_MAXB];
  __shared__ double red[NW][PJ_MAXG];
  __shared__ double perr_s;
  const int t = blockIdx.x, tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int nb = a.mech.nb, n6 = 6 * nb, d = a.d, G = a.G;
  const RolloutGP* gp = a.gps + (size_t)a.group[t] * G;
  const double* st0 = a.start + (size_t)t * d;
  if (w == 0) set_states(P, st0, nb, a.dt, l);
  for (int i = tid; i < d; i += NT) obs[i] = st0[i];
  if (tid == 0) {
    perr_s = 0.0;
    P.status = 0;
  }
  __syncthreads();
  for (int step = 0; step < a.steps && P.status == 0; ++step) {
    // ---- mu_g = sum_j sf2 exp(-r_j / 2) alpha_j at the current CState (predict_y means)
    for (int g = 0; g < G; ++g) {
      const RolloutGP Gp = gp[g];
      const double sf2 = Gp.params[d];
      double sacc = 0.0;
      for (int j = tid; j < Gp.N; j += NT) {
        const double* x = Gp.X + (size_t)j * d;
        double r = 0.0;
        for (int p = 0; p < d; ++p) {
          const double o = obs[p];
          if (MODE == 0) {
            const double v = fma(-2.0, x[p] * o, x[p] * x[p] + o * o);
            r = r + (v > 0.0 ? v : 0.0) * Gp.params[p];
          } else {
            const double df = x[p] - o;
            r = __builtin_fma(df * df, Gp.params[p], r);
          }
        }
        sacc = fma(sf2 * exp(-r * 0.5), Gp.alpha[j], sacc);
      }
      sacc = wsum(sacc);
      if (l == 0) red[w][g] = sacc;
    }
    __syncthreads();
    if (w == 0) {
      // getvw: mu_g at CState position vw[g], zero elsewhere; (v, w) per body into P.s
      if (l < n6) P.s[l] = 0.0;
      __builtin_amdgcn_wave_barrier();
      if (l < G) {
        double mu = red[0][l];
        for (int q = 1; q < NW; ++q) mu += red[q][l];
        const int pos = a.vw[l], b = pos / 13, k = pos - 13 * b;  // k in 7..12
        P.s[6 * b + (k - 7)] = mu;
      }
    }
    __syncthreads();
    project<NW>(P, a.mech, a.dt, a.reg, a.eps, a.iters);  // the whole workgroup
    if (w == 0) {
      // projection error |(v, w)_const - (v, w)_pred| (predictdynamics.jl:16), then updatestate!
      const double dv = l < n6 ? P.s[l] - P.su[l] : 0.0;
      const double e = sqrt(wsum(dv * dv));
      if (l == 0) perr_s += e;
      update_state(P, nb, a.dt, l);
      __builtin_amdgcn_wave_barrier();
      for (int i = l; i < d; i += 64) obs[i] = cstate_at(P, i);
    }
    __syncthreads();
  }
  if (w == 0) {
    update_state(P, nb, a.dt, l);  // the closing updatestate! (predictdynamics.jl:20)
    __builtin_amdgcn_wave_barrier();
    for (int i = l; i < d; i += 64) a.out[(size_t)t * d + i] = P.status ? NAN : cstate_at(P, i);
    if (l == 0) {
      a.perr[t] = P.status ? NAN : perr_s / (a.steps > 0 ? a.steps : 1);
      a.status[t] = P.status;
    }
  }
}

void launch_project(const ProjArgs& a, hipStream_t s) {
  if (a.T > 0) hipLaunchKernelGGL(k_project, dim3(a.T), dim3(64), pj_lds_bytes(a.mech.nb, a.mech.nd), s, a);
}
void launch_vi_step(const ViArgs& a, hipStream_t s) {
  if (a.T <= 0) return;
  const size_t n = 6 * (size_t)a.mech.nb + a.mech.nd;
  const size_t lds = (n * (n + 1) + (size_t)a.mech.nd * 6 * a.mech.nb) * sizeof(double);
  hipLaunchKernelGGL(k_vi_step, dim3(a.T), dim3(64), lds, s, a);
}
void launch_rollout_max(const RolloutMaxArgs& a, int dist_mode, hipStream_t s) {
  if (a.T <= 0) return;
  const size_t lds = pj_lds_bytes(a.mech.nb, a.mech.nd);
  if (dist_mode == 0) hipLaunchKernelGGL(k_rollout_max<0>, dim3(a.T), dim3(256), lds, s, a);
  else hipLaunchKernelGGL(k_rollout_max<1>, dim3(a.T), dim3(256), lds, s, a);
}

}  // namespace gprx
