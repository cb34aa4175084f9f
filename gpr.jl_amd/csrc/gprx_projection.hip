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
__device__ void subjoint(PState& P, const SubJoint& J, int n6, int ldf, double dt, bool want_g, bool want_jac) {
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
          PJ_F[(c0 + j) * ldf + row] = tv;
          PJ_F[(c0 + 3 + j) * ldf + row] = tw;
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
    bool singular = false;
    for (int k = 0; k < n; ++k) {
      // pivot: first row of maximal |a_ik|, i >= k (idamax)
      double v = (l >= k && l < n) ? fabs(PJ_A[l * ldf + k]) : -1.0;
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
          const double t = PJ_A[k * ldf + j];
          PJ_A[k * ldf + j] = PJ_A[p * ldf + j];
          PJ_A[p * ldf + j] = t;
        }
        const double bk = readlane_dbl(b, k), bp = readlane_dbl(b, p);
        if (l == k) b = bp;
        if (l == p) b = bk;
      }
      pj_sync<NW>();
      const double akk = PJ_A[k * ldf + k];
      if (akk == 0.0) singular = true;
      const int m = n - 1 - k;
      if (akk != 0.0 && m > 0) {
        if (w0 && l > k && l < n)
          PJ_A[l * ldf + k] = fabs(akk) >= DBL_MIN ? PJ_A[l * ldf + k] * (1.0 / akk) : PJ_A[l * ldf + k] / akk;
        pj_sync<NW>();
        // trailing update A[i][j] -= l_i A[k][j], i, j in (k, n): element e = (i - k - 1) m + (j - k - 1)
        const int si = NT / m, sj = NT - si * m;
        int i = tid / m, j = tid - i * m;
        for (int e = tid; e < m * m; e += NT) {
          const int gi = k + 1 + i, gj = k + 1 + j;
          PJ_A[gi * ldf + gj] = PJ_A[gi * ldf + gj] - PJ_A[gi * ldf + k] * PJ_A[k * ldf + gj];
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
    if (singular) {  // Julia's F \ f throws SingularException: the trajectory stops
      if (tid == 0) P.status = 1;
      pj_sync<NW>();
      return;
    }
    // forward substitution (unit lower), then backward (upper), as dgetrs / dtrsm
    for (int k = 0; k < n; ++k) {
      const double bk = readlane_dbl(b, k);
      if (bk != 0.0 && l > k && l < n) b = b - bk * PJ_A[l * ldf + k];
    }
    for (int k = n - 1; k >= 0; --k) {
      const double ukk = PJ_A[k * ldf + k];
      double bk = readlane_dbl(b, k);
      if (bk != 0.0) {
        bk = bk / ukk;
        if (l == k) b = bk;
        if (l < k) b = b - bk * PJ_A[l * ldf + k];
      }
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
void launch_rollout_max(const RolloutMaxArgs& a, int dist_mode, hipStream_t s) {
  if (a.T <= 0) return;
  const size_t lds = pj_lds_bytes(a.mech.nb, a.mech.nd);
  if (dist_mode == 0) hipLaunchKernelGGL(k_rollout_max<0>, dim3(a.T), dim3(256), lds, s, a);
  else hipLaunchKernelGGL(k_rollout_max<1>, dim3(a.T), dim3(256), lds, s, a);
}

}  // namespace gprx
