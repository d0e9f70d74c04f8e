// vg_la.h — fixed-size fp64 linear algebra for the product, usable from host
// C++ and HIP device code (no Eigen in this image). Row-major storage.
// Expression trees of every product follow the canonical order
//   s = a0*b0; s += a1*b1; s += a2*b2 ...
// and the library is built with -ffp-contract=off, so world points
// R*p + t (and therefore voxel keys) are reproducible bit-for-bit.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>

#if defined(__HIPCC__) || defined(__HIP__)
#define VG_HD __host__ __device__ __forceinline__
#else
#define VG_HD inline
#endif

namespace vg {

template <int R, int C>
struct M {
  double a[R * C];
  VG_HD double& operator()(int i, int j) { return a[i * C + j]; }
  VG_HD const double& operator()(int i, int j) const { return a[i * C + j]; }
  VG_HD double& operator[](int i) { return a[i]; }
  VG_HD const double& operator[](int i) const { return a[i]; }
  VG_HD void zero() {
    for (int i = 0; i < R * C; i++) a[i] = 0.0;
  }
  VG_HD static M Z() {
    M m;
    m.zero();
    return m;
  }
  VG_HD static M I() {
    M m;
    m.zero();
    for (int i = 0; i < (R < C ? R : C); i++) m(i, i) = 1.0;
    return m;
  }
};
using V3 = M<3, 1>;
using M3 = M<3, 3>;
using M6 = M<6, 6>;
using V6 = M<6, 1>;
using M15 = M<15, 15>;
using V15 = M<15, 1>;

template <int R, int C, int K>
VG_HD M<R, K> mul(const M<R, C>& x, const M<C, K>& y) {
  M<R, K> o;
  for (int i = 0; i < R; i++)
    for (int j = 0; j < K; j++) {
      double s = x(i, 0) * y(0, j);
      for (int k = 1; k < C; k++) s += x(i, k) * y(k, j);
      o(i, j) = s;
    }
  return o;
}
template <int R, int C>
VG_HD M<C, R> tr(const M<R, C>& x) {
  M<C, R> o;
  for (int i = 0; i < R; i++)
    for (int j = 0; j < C; j++) o(j, i) = x(i, j);
  return o;
}
template <int R, int C>
VG_HD M<R, C> add(const M<R, C>& x, const M<R, C>& y) {
  M<R, C> o;
  for (int i = 0; i < R * C; i++) o[i] = x[i] + y[i];
  return o;
}
template <int R, int C>
VG_HD M<R, C> sub(const M<R, C>& x, const M<R, C>& y) {
  M<R, C> o;
  for (int i = 0; i < R * C; i++) o[i] = x[i] - y[i];
  return o;
}
template <int R, int C>
VG_HD M<R, C> scl(const M<R, C>& x, double s) {
  M<R, C> o;
  for (int i = 0; i < R * C; i++) o[i] = x[i] * s;
  return o;
}
VG_HD V3 v3(double x, double y, double z) {
  V3 v;
  v[0] = x;
  v[1] = y;
  v[2] = z;
  return v;
}
VG_HD double dot3(const V3& a, const V3& b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
VG_HD double norm3(const V3& a) { return sqrt(dot3(a, a)); }
VG_HD V3 cross3(const V3& a, const V3& b) {
  return v3(a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]);
}
VG_HD M3 outer3(const V3& a, const V3& b) {
  M3 m;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) m(i, j) = a[i] * b[j];
  return m;
}
VG_HD M3 hat(const V3& v) {
  M3 m;
  m.zero();
  m(0, 1) = -v[2];
  m(0, 2) = v[1];
  m(1, 0) = v[2];
  m(1, 2) = -v[0];
  m(2, 0) = -v[1];
  m(2, 1) = v[0];
  return m;
}
// R*p + t with the canonical tree ((r0*x + r1*y) + r2*z) + t — the key contract.
VG_HD V3 rigid(const M3& R, const V3& p, const V3& t) {
  V3 o;
  for (int i = 0; i < 3; i++) {
    double s = R(i, 0) * p[0];
    s += R(i, 1) * p[1];
    s += R(i, 2) * p[2];
    o[i] = s + t[i];
  }
  return o;
}
VG_HD V3 mv3(const M3& R, const V3& p) { return mul(R, p); }

// so(3) exponential / logarithm / right Jacobians (math.hpp:12-88 semantics)
VG_HD M3 Exp(const V3& ang) {
  double n = norm3(ang);
  if (n >= 1e-9) {
    V3 r = scl(ang, 1.0 / n);
    for (int i = 0; i < 3; i++) r[i] = ang[i] / n;
    M3 K = hat(r);
    return add(add(M3::I(), scl(K, sin(n))), scl(mul(K, K), 1.0 - cos(n)));
  }
  return M3::I();
}
VG_HD M3 Exp(const V3& w, double dt) {
  double n = norm3(w);
  if (n > 1e-7) {
    V3 r;
    for (int i = 0; i < 3; i++) r[i] = w[i] / n;
    M3 K = hat(r);
    double a = n * dt;
    return add(add(M3::I(), scl(K, sin(a))), scl(mul(K, K), 1.0 - cos(a)));
  }
  return M3::I();
}
VG_HD V3 Log(const M3& R) {
  double tr_ = R(0, 0) + R(1, 1) + R(2, 2);
  double theta = (tr_ > 3.0 - 1e-6) ? 0.0 : acos(0.5 * (tr_ - 1));
  V3 K = v3(R(2, 1) - R(1, 2), R(0, 2) - R(2, 0), R(1, 0) - R(0, 1));
  return (fabs(theta) < 0.001) ? scl(K, 0.5) : scl(K, 0.5 * theta / sin(theta));
}
VG_HD M3 jr(V3 vec) {
  double ang = norm3(vec);
  if (ang < 1e-9) return M3::I();
  for (int i = 0; i < 3; i++) vec[i] /= ang;
  double ra = sin(ang) / ang;
  return sub(add(scl(M3::I(), ra), scl(outer3(vec, vec), 1 - ra)), scl(hat(vec), (1 - cos(ang)) / ang));
}
// angle-axis of a rotation matrix via the quaternion (Eigen::AngleAxisd(Matrix3d))
VG_HD void angle_axis(const M3& m, double& angle, V3& axis) {
  double q[4];
  double t = m(0, 0) + m(1, 1) + m(2, 2);
  if (t > 0) {
    t = sqrt(t + 1.0);
    q[3] = 0.5 * t;
    t = 0.5 / t;
    q[0] = (m(2, 1) - m(1, 2)) * t;
    q[1] = (m(0, 2) - m(2, 0)) * t;
    q[2] = (m(1, 0) - m(0, 1)) * t;
  } else {
    int i = 0;
    if (m(1, 1) > m(0, 0)) i = 1;
    if (m(2, 2) > m(i, i)) i = 2;
    int j = (i + 1) % 3, k = (j + 1) % 3;
    t = sqrt(m(i, i) - m(j, j) - m(k, k) + 1.0);
    q[i] = 0.5 * t;
    t = 0.5 / t;
    q[3] = (m(k, j) - m(j, k)) * t;
    q[j] = (m(j, i) + m(i, j)) * t;
    q[k] = (m(k, i) + m(i, k)) * t;
  }
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]);
  if (n != 0.0) {
    angle = 2.0 * atan2(n, fabs(q[3]));
    if (q[3] < 0) n = -n;
    axis = v3(q[0] / n, q[1] / n, q[2] / n);
  } else {
    angle = 0.0;
    axis = v3(1, 0, 0);
  }
}
VG_HD M3 jr_inv(const M3& R) {
  double ang;
  V3 ax;
  angle_axis(R, ang, ax);
  if (ang < 1e-9) return M3::I();
  double ctt = ang / 2 / tan(ang / 2);
  return add(add(scl(M3::I(), ctt), scl(outer3(ax, ax), 1 - ctt)), scl(hat(ax), ang / 2));
}

// Symmetric 3x3 eigen-decomposition, cyclic Jacobi, ascending eigenvalues,
// eigenvectors in columns (SelfAdjointEigenSolver<Matrix3d> semantics).
// Stops once the off-diagonal mass is below 1e-18 of the diagonal's: the
// eigenvalue error is then second order in it (far below one ulp) and the
// eigenvector error ~1e-18 |A| / gap; 3-4 sweeps instead of the 5-6 an
// exact-zero stop takes (a ~35 % shorter dependency chain on the GPU, where
// one decomposition per thread is pure latency).
VG_HD void eig3(const M3& Ain, V3& w, M3& V) {
  double a[3][3];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) a[i][j] = 0.5 * (Ain(i, j) + Ain(j, i));
  double v[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
  for (int sweep = 0; sweep < 60; sweep++) {
    double off = fabs(a[0][1]) + fabs(a[0][2]) + fabs(a[1][2]);
    if (off == 0.0 || off <= 1e-18 * (fabs(a[0][0]) + fabs(a[1][1]) + fabs(a[2][2]))) break;
    for (int p = 0; p < 2; p++)
      for (int q = p + 1; q < 3; q++) {
        double apq = a[p][q];
        if (apq == 0.0) continue;
        double theta = (a[q][q] - a[p][p]) / (2.0 * apq);
        double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        if (__builtin_isinf(theta)) t = 0.0;
        double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < 3; k++) {
          double akp = a[k][p], akq = a[k][q];
          a[k][p] = c * akp - s * akq;
          a[k][q] = s * akp + c * akq;
        }
        for (int k = 0; k < 3; k++) {
          double apk = a[p][k], aqk = a[q][k];
          a[p][k] = c * apk - s * aqk;
          a[q][k] = s * apk + c * aqk;
        }
        a[p][q] = a[q][p] = 0.0;
        for (int k = 0; k < 3; k++) {
          double vkp = v[k][p], vkq = v[k][q];
          v[k][p] = c * vkp - s * vkq;
          v[k][q] = s * vkp + c * vkq;
        }
      }
  }
  int idx[3] = {0, 1, 2};
  double ev[3] = {a[0][0], a[1][1], a[2][2]};
  for (int i = 0; i < 3; i++)
    for (int j = i + 1; j < 3; j++)
      if (ev[idx[j]] < ev[idx[i]]) {
        int tmp = idx[i];
        idx[i] = idx[j];
        idx[j] = tmp;
      }
  for (int j = 0; j < 3; j++) {
    w[j] = ev[idx[j]];
    for (int k = 0; k < 3; k++) V(k, j) = v[k][idx[j]];
  }
}

// Symmetric packed storage helpers (upper triangle, row-major).
VG_HD constexpr int sym_n(int n) { return n * (n + 1) / 2; }
VG_HD int sym_idx(int n, int i, int j) {
  if (i > j) {
    int t = i;
    i = j;
    j = t;
  }
  return i * n - i * (i - 1) / 2 + (j - i);
}

// Point cluster (types.hpp:115-175): P as packed sym 3x3 (xx,xy,xz,yy,yz,zz), v, N.
struct Clu {
  double P[6];
  double v[3];
  int N;
  int pad;
};
VG_HD void clu_zero(Clu& c) {
  for (int i = 0; i < 6; i++) c.P[i] = 0;
  for (int i = 0; i < 3; i++) c.v[i] = 0;
  c.N = 0;
  c.pad = 0;
}
VG_HD void clu_push(Clu& c, const V3& p) {
  c.N++;
  c.P[0] += p[0] * p[0];
  c.P[1] += p[0] * p[1];
  c.P[2] += p[0] * p[2];
  c.P[3] += p[1] * p[1];
  c.P[4] += p[1] * p[2];
  c.P[5] += p[2] * p[2];
  c.v[0] += p[0];
  c.v[1] += p[1];
  c.v[2] += p[2];
}
VG_HD void clu_add(Clu& c, const Clu& d) {
  for (int i = 0; i < 6; i++) c.P[i] += d.P[i];
  for (int i = 0; i < 3; i++) c.v[i] += d.v[i];
  c.N += d.N;
}
VG_HD void clu_sub(Clu& c, const Clu& d) {
  for (int i = 0; i < 6; i++) c.P[i] -= d.P[i];
  for (int i = 0; i < 3; i++) c.v[i] -= d.v[i];
  c.N -= d.N;
}
VG_HD M3 clu_Pm(const Clu& c) {
  M3 m;
  m(0, 0) = c.P[0];
  m(0, 1) = m(1, 0) = c.P[1];
  m(0, 2) = m(2, 0) = c.P[2];
  m(1, 1) = c.P[3];
  m(1, 2) = m(2, 1) = c.P[4];
  m(2, 2) = c.P[5];
  return m;
}
VG_HD V3 clu_v(const Clu& c) { return v3(c.v[0], c.v[1], c.v[2]); }
// PointCluster::cov — P/N - c c^T
VG_HD M3 clu_cov(const Clu& c) {
  V3 ce = v3(c.v[0] / c.N, c.v[1] / c.N, c.v[2] / c.N);
  M3 P = clu_Pm(c);
  M3 o;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) o(i, j) = P(i, j) / c.N - ce[i] * ce[j];
  return o;
}
// PointCluster::transform — v = R v + N t; P = R P R^T + R v t^T + t (R v)^T + N t t^T
VG_HD Clu clu_transform(const Clu& s, const M3& R, const V3& t) {
  Clu o;
  o.N = s.N;
  o.pad = 0;
  V3 Rv = mul(R, clu_v(s));
  double n = (double)s.N;
  for (int i = 0; i < 3; i++) o.v[i] = Rv[i] + t[i] * n;
  M3 P = mul(mul(R, clu_Pm(s)), tr(R));
  M3 rp = outer3(Rv, t);
  for (int i = 0; i < 3; i++)
    for (int j = i; j < 3; j++) {
      double val = P(i, j) + rp(i, j) + rp(j, i) + t[i] * t[j] * n;
      o.P[sym_idx(3, i, j)] = val;
    }
  return o;
}

}  // namespace vg

namespace vg {
// Dense inverse with partial pivoting (Gauss-Jordan) — stands in for Eigen's
// fixed-size .inverse() (odometry.cpp:82,194; imu_preintegration.cpp:126).
template <int N>
VG_HD M<N, N> inverse(const M<N, N>& Ain) {
  double a[N][2 * N];
  for (int i = 0; i < N; i++)
    for (int j = 0; j < N; j++) {
      a[i][j] = Ain(i, j);
      a[i][N + j] = (i == j) ? 1.0 : 0.0;
    }
  for (int c = 0; c < N; c++) {
    int p = c;
    double best = fabs(a[c][c]);
    for (int r = c + 1; r < N; r++)
      if (fabs(a[r][c]) > best) {
        best = fabs(a[r][c]);
        p = r;
      }
    if (p != c)
      for (int j = 0; j < 2 * N; j++) {
        double t = a[c][j];
        a[c][j] = a[p][j];
        a[p][j] = t;
      }
    double inv = 1.0 / a[c][c];
    for (int j = 0; j < 2 * N; j++) a[c][j] *= inv;
    for (int r = 0; r < N; r++) {
      if (r == c) continue;
      double f = a[r][c];
      if (f == 0.0) continue;
      for (int j = 0; j < 2 * N; j++) a[r][j] -= f * a[c][j];
    }
  }
  M<N, N> o;
  for (int i = 0; i < N; i++)
    for (int j = 0; j < N; j++) o(i, j) = a[i][N + j];
  return o;
}
}  // namespace vg

namespace vg {
// Eigen ColPivHouseholderQR(A).solve(b) for A m x 3 (m <= 8, row-major),
// restated from Eigen's algorithm (odometry.cpp:362): Householder
// QR with column pivoting on the largest remaining column norm (first on ties),
// the sqrt(eps) norm-downdate recompute rule, the rank cut of its
// nonzero-pivot count, Q^T b, back substitution, inverse column permutation.
// Reductions are sequential (Eigen vectorises them: rounding-level).
VG_HD void colpiv_qr_solve(const double* Ain, int m, const double* b, double* x) {
  const int n = 3, size = m < n ? m : n;
  double A[8 * 3];
  for (int i = 0; i < m * n; i++) A[i] = Ain[i];
  double tau[3], normU[3], normD[3];
  int trans[3];
  double maxnorm = 0.0;
  for (int j = 0; j < n; j++) {
    double s = 0.0;
    for (int r = 0; r < m; r++) s += A[r * 3 + j] * A[r * 3 + j];
    normD[j] = normU[j] = sqrt(s);
    if (normU[j] > maxnorm) maxnorm = normU[j];
  }
  const double eps = 2.220446049250313e-16;
  const double thr_helper = (maxnorm * eps) * (maxnorm * eps) / m;
  const double downdate_thr = sqrt(eps);
  int nonzero = size;
  for (int k = 0; k < size; k++) {
    int big = k;
    for (int j = k + 1; j < n; j++)
      if (normU[j] > normU[big]) big = j;
    const double big_sq = normU[big] * normU[big];
    if (nonzero == size && big_sq < thr_helper * (m - k)) nonzero = k;
    trans[k] = big;
    if (k != big) {
      for (int r = 0; r < m; r++) {
        const double t = A[r * 3 + k];
        A[r * 3 + k] = A[r * 3 + big];
        A[r * 3 + big] = t;
      }
      double t = normU[k];
      normU[k] = normU[big];
      normU[big] = t;
      t = normD[k];
      normD[k] = normD[big];
      normD[big] = t;
    }
    double tail = 0.0;
    for (int r = k + 1; r < m; r++) tail += A[r * 3 + k] * A[r * 3 + k];
    const double c0 = A[k * 3 + k];
    double beta;
    if (tail <= 2.2250738585072014e-308) {
      tau[k] = 0.0;
      beta = c0;
      for (int r = k + 1; r < m; r++) A[r * 3 + k] = 0.0;
    } else {
      beta = sqrt(c0 * c0 + tail);
      if (c0 >= 0.0) beta = -beta;
      for (int r = k + 1; r < m; r++) A[r * 3 + k] = A[r * 3 + k] / (c0 - beta);
      tau[k] = (beta - c0) / beta;
    }
    A[k * 3 + k] = beta;
    for (int j = k + 1; j < n; j++) {
      if (m - k == 1) {
        A[k * 3 + j] *= (1.0 - tau[k]);
      } else if (tau[k] != 0.0) {
        double t = 0.0;
        for (int r = k + 1; r < m; r++) t += A[r * 3 + k] * A[r * 3 + j];
        t += A[k * 3 + j];
        A[k * 3 + j] -= tau[k] * t;
        for (int r = k + 1; r < m; r++) A[r * 3 + j] -= tau[k] * A[r * 3 + k] * t;
      }
    }
    for (int j = k + 1; j < n; j++) {
      if (normU[j] != 0.0) {
        double t = fabs(A[k * 3 + j]) / normU[j];
        t = (1.0 + t) * (1.0 - t);
        if (t < 0.0) t = 0.0;
        const double q = normU[j] / normD[j];
        const double t2 = t * q * q;
        if (t2 <= downdate_thr) {
          double s = 0.0;
          for (int r = k + 1; r < m; r++) s += A[r * 3 + j] * A[r * 3 + j];
          normD[j] = sqrt(s);
          normU[j] = normD[j];
        } else {
          normU[j] *= sqrt(t);
        }
      }
    }
  }
  double c[8];
  for (int r = 0; r < m; r++) c[r] = b[r];
  for (int k = 0; k < nonzero; k++) {
    if (m - k == 1) {
      c[k] *= (1.0 - tau[k]);
    } else if (tau[k] != 0.0) {
      double t = 0.0;
      for (int r = k + 1; r < m; r++) t += A[r * 3 + k] * c[r];
      t += c[k];
      c[k] -= tau[k] * t;
      for (int r = k + 1; r < m; r++) c[r] -= tau[k] * A[r * 3 + k] * t;
    }
  }
  double y[3] = {0.0, 0.0, 0.0};
  for (int i = nonzero - 1; i >= 0; i--) {
    double s = c[i];
    for (int j = i + 1; j < nonzero; j++) s -= A[i * 3 + j] * y[j];
    y[i] = s / A[i * 3 + i];
  }
  int perm[3] = {0, 1, 2};
  for (int k = 0; k < size; k++) {
    const int t = perm[k];
    perm[k] = perm[trans[k]];
    perm[trans[k]] = t;
  }
  for (int i = 0; i < n; i++) x[perm[i]] = y[i];
}
}  // namespace vg
