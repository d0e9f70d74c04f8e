// ORACLE — test infrastructure only. Never linked into the product library.
//
// Tiny dependency-free fixed-size linear algebra for the CPU restatement of the
// VINA-SLAM per-scan hot path. Eigen3 is absent in this image, so every product
// below is a plain triple loop with the canonical accumulation order
//     s = a(i,0)*b(0,j); s += a(i,1)*b(1,j); ...
// The restatement is compiled with -ffp-contract=off so that the voxel-key
// arithmetic (world point -> key) follows one fixed expression tree that the
// HIP kernels reproduce exactly (the "key contract").
//
// Replaces: Eigen::Matrix<double,R,C> fixed-size arithmetic used throughout
// include/vina_slam/core/{types,math}.hpp, SelfAdjointEigenSolver<Matrix3d>
// (octree.cpp:362,435; factors.cpp:148; odometry.cpp:244), Matrix<15,15>::inverse
// (odometry.cpp:82,194; imu_preintegration.cpp:126) and MatrixXd::ldlt
// (optimizers.cpp:466).
#pragma once
#include <cmath>
#include <cstring>
#include <vector>
#include <algorithm>
#include <limits>

namespace orc {

template <int R, int C>
struct Mat {
  double d[R * C];
  Mat() { std::memset(d, 0, sizeof(d)); }
  double& operator()(int i, int j) { return d[i * C + j]; }
  const double& operator()(int i, int j) const { return d[i * C + j]; }
  double& operator[](int i) { return d[i]; }
  const double& operator[](int i) const { return d[i]; }
  static Mat Zero() { return Mat(); }
  static Mat Identity() {
    Mat m;
    for (int i = 0; i < (R < C ? R : C); i++) m(i, i) = 1.0;
    return m;
  }
  void setZero() { std::memset(d, 0, sizeof(d)); }
  void setIdentity() { *this = Identity(); }
  Mat<C, R> T() const {
    Mat<C, R> t;
    for (int i = 0; i < R; i++)
      for (int j = 0; j < C; j++) t(j, i) = (*this)(i, j);
    return t;
  }
  template <int K>
  Mat<R, K> operator*(const Mat<C, K>& b) const {
    Mat<R, K> o;
    for (int i = 0; i < R; i++)
      for (int j = 0; j < K; j++) {
        double s = (*this)(i, 0) * b(0, j);
        for (int k = 1; k < C; k++) s += (*this)(i, k) * b(k, j);
        o(i, j) = s;
      }
    return o;
  }
  Mat operator+(const Mat& b) const { Mat o; for (int i = 0; i < R * C; i++) o.d[i] = d[i] + b.d[i]; return o; }
  Mat operator-(const Mat& b) const { Mat o; for (int i = 0; i < R * C; i++) o.d[i] = d[i] - b.d[i]; return o; }
  Mat operator-() const { Mat o; for (int i = 0; i < R * C; i++) o.d[i] = -d[i]; return o; }
  Mat operator*(double s) const { Mat o; for (int i = 0; i < R * C; i++) o.d[i] = d[i] * s; return o; }
  Mat operator/(double s) const { Mat o; for (int i = 0; i < R * C; i++) o.d[i] = d[i] / s; return o; }
  Mat& operator+=(const Mat& b) { for (int i = 0; i < R * C; i++) d[i] += b.d[i]; return *this; }
  Mat& operator-=(const Mat& b) { for (int i = 0; i < R * C; i++) d[i] -= b.d[i]; return *this; }
  Mat& operator*=(double s) { for (int i = 0; i < R * C; i++) d[i] *= s; return *this; }
  Mat& operator/=(double s) { for (int i = 0; i < R * C; i++) d[i] /= s; return *this; }
  template <int r, int c>
  Mat<r, c> block(int i0, int j0) const {
    Mat<r, c> o;
    for (int i = 0; i < r; i++)
      for (int j = 0; j < c; j++) o(i, j) = (*this)(i0 + i, j0 + j);
    return o;
  }
  template <int r, int c>
  void setBlock(int i0, int j0, const Mat<r, c>& b) {
    for (int i = 0; i < r; i++)
      for (int j = 0; j < c; j++) (*this)(i0 + i, j0 + j) = b(i, j);
  }
  template <int r, int c>
  void addBlock(int i0, int j0, const Mat<r, c>& b) {
    for (int i = 0; i < r; i++)
      for (int j = 0; j < c; j++) (*this)(i0 + i, j0 + j) += b(i, j);
  }
  double trace() const { double s = 0; for (int i = 0; i < R; i++) s += (*this)(i, i); return s; }
};
template <int R, int C>
inline Mat<R, C> operator*(double s, const Mat<R, C>& m) { return m * s; }

using V3 = Mat<3, 1>;
using M3 = Mat<3, 3>;
using M6 = Mat<6, 6>;
using V6 = Mat<6, 1>;
using M9 = Mat<9, 9>;
using M15 = Mat<15, 15>;
using V15 = Mat<15, 1>;

inline V3 v3(double x, double y, double z) { V3 v; v[0] = x; v[1] = y; v[2] = z; return v; }
template <int N>
inline double dot(const Mat<N, 1>& a, const Mat<N, 1>& b) {
  double s = a[0] * b[0];
  for (int i = 1; i < N; i++) s += a[i] * b[i];
  return s;
}
template <int N>
inline double squaredNorm(const Mat<N, 1>& a) { return dot(a, a); }
template <int N>
inline double norm(const Mat<N, 1>& a) { return std::sqrt(squaredNorm(a)); }
inline V3 cross(const V3& a, const V3& b) {
  return v3(a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]);
}
inline M3 outer(const V3& a, const V3& b) {
  M3 m;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) m(i, j) = a[i] * b[j];
  return m;
}
inline V3 col(const M3& m, int j) { return v3(m(0, j), m(1, j), m(2, j)); }

// ---- symmetric 3x3 eigen decomposition (cyclic Jacobi), ascending eigenvalues,
// eigenvectors as columns. Replaces Eigen::SelfAdjointEigenSolver<Matrix3d>.
inline void eig3(const M3& Ain, V3& w, M3& V) {
  double a[3][3];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) a[i][j] = 0.5 * (Ain(i, j) + Ain(j, i));
  double v[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
  for (int sweep = 0; sweep < 60; sweep++) {
    double off = std::fabs(a[0][1]) + std::fabs(a[0][2]) + std::fabs(a[1][2]);
    if (off == 0.0) break;
    for (int p = 0; p < 2; p++)
      for (int q = p + 1; q < 3; q++) {
        double apq = a[p][q];
        if (apq == 0.0) continue;
        double theta = (a[q][q] - a[p][p]) / (2.0 * apq);
        double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
        if (std::isinf(theta)) t = 0.0;
        double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < 3; k++) {  // A <- J^T A J
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
  // ascending, stable
  for (int i = 0; i < 3; i++)
    for (int j = i + 1; j < 3; j++)
      if (ev[idx[j]] < ev[idx[i]]) std::swap(idx[i], idx[j]);
  for (int j = 0; j < 3; j++) {
    w[j] = ev[idx[j]];
    for (int k = 0; k < 3; k++) V(k, j) = v[k][idx[j]];
  }
}

// ---- dense inverse with partial pivoting (Gauss-Jordan). Replaces Eigen's
// fixed-size .inverse() (partial-pivot LU) on 15x15.
template <int N>
inline Mat<N, N> inverse(const Mat<N, N>& Ain) {
  double a[N][2 * N];
  for (int i = 0; i < N; i++)
    for (int j = 0; j < N; j++) {
      a[i][j] = Ain(i, j);
      a[i][N + j] = (i == j) ? 1.0 : 0.0;
    }
  for (int c = 0; c < N; c++) {
    int p = c;
    double best = std::fabs(a[c][c]);
    for (int r = c + 1; r < N; r++)
      if (std::fabs(a[r][c]) > best) { best = std::fabs(a[r][c]); p = r; }
    if (p != c)
      for (int j = 0; j < 2 * N; j++) std::swap(a[c][j], a[p][j]);
    double inv = 1.0 / a[c][c];
    for (int j = 0; j < 2 * N; j++) a[c][j] *= inv;
    for (int r = 0; r < N; r++) {
      if (r == c) continue;
      double f = a[r][c];
      if (f == 0.0) continue;
      for (int j = 0; j < 2 * N; j++) a[r][j] -= f * a[c][j];
    }
  }
  Mat<N, N> o;
  for (int i = 0; i < N; i++)
    for (int j = 0; j < N; j++) o(i, j) = a[i][N + j];
  return o;
}

// ---- dynamic dense matrix (row-major) for the 15W x 15W LM system.
struct MatX {
  int n = 0, m = 0;
  std::vector<double> d;
  MatX() {}
  MatX(int n_, int m_) : n(n_), m(m_), d((size_t)n_ * m_, 0.0) {}
  void resize(int n_, int m_) { n = n_; m = m_; d.assign((size_t)n_ * m_, 0.0); }
  double& operator()(int i, int j) { return d[(size_t)i * m + j]; }
  const double& operator()(int i, int j) const { return d[(size_t)i * m + j]; }
  void setZero() { std::fill(d.begin(), d.end(), 0.0); }
};

// Eigen::LDLT<MatrixXd, Lower>::compute + solve restated (Eigen 3.x,
// Cholesky/LDLT.h: ldlt_inplace<Lower>::unblocked and LDLT::_solve_impl);
// replaces (Hess + u*D).ldlt().solve(-JacT) at optimizers.cpp:466.
// The factorization is LEFT-looking: at step k only A(k,k) and column k below
// it are brought up to date, so the pivot (largest |A(i,i)|, i >= k, first on
// ties) is chosen among the *original* diagonal entries of the remaining rows,
// not the Schur-complement diagonal. Only the lower triangle is read (the
// LiDAR Hessian's diagonal 6x6 blocks are not exactly symmetric,
// factors.cpp:90-91).
inline std::vector<double> ldlt_solve(const MatX& Ain, const std::vector<double>& b) {
  const int n = Ain.n;
  MatX A = Ain;
  std::vector<int> tr(n);
  std::vector<double> temp(n);
  for (int k = 0; k < n; k++) {
    int p = k;
    double best = std::fabs(A(k, k));
    for (int i = k + 1; i < n; i++)
      if (std::fabs(A(i, i)) > best) { best = std::fabs(A(i, i)); p = i; }
    tr[k] = p;
    if (p != k) {  // transposition on the lower triangle only
      for (int j = 0; j < k; j++) std::swap(A(k, j), A(p, j));
      for (int i = p + 1; i < n; i++) std::swap(A(i, k), A(i, p));
      std::swap(A(k, k), A(p, p));
      for (int i = k + 1; i < p; i++) std::swap(A(i, k), A(p, i));
    }
    if (k > 0) {
      for (int j = 0; j < k; j++) temp[j] = A(j, j) * A(k, j);
      double s = 0.0;
      for (int j = 0; j < k; j++) s += A(k, j) * temp[j];
      A(k, k) -= s;
      for (int i = k + 1; i < n; i++) {
        double t = 0.0;
        for (int j = 0; j < k; j++) t += A(i, j) * temp[j];
        A(i, k) -= t;
      }
    }
    const double akk = A(k, k);
    if (k == 0 && akk == 0.0) {  // all-zero diagonal: Eigen stops, identity transpositions
      for (int j = 0; j < n; j++) tr[j] = j;
      break;
    }
    if (akk != 0.0)
      for (int i = k + 1; i < n; i++) A(i, k) /= akk;
  }
  std::vector<double> x(b);
  for (int k = 0; k < n; k++) std::swap(x[k], x[tr[k]]);  // P b
  for (int i = 0; i < n; i++) {                          // L^-1
    double s = 0.0;
    for (int j = 0; j < i; j++) s += A(i, j) * x[j];
    x[i] -= s;
  }
  for (int i = 0; i < n; i++)  // pseudo-inverse of D (Eigen bug 241)
    x[i] = (std::fabs(A(i, i)) > std::numeric_limits<double>::min()) ? x[i] / A(i, i) : 0.0;
  for (int i = n - 1; i >= 0; i--) {  // L^-T
    double s = 0.0;
    for (int j = i + 1; j < n; j++) s += A(j, i) * x[j];
    x[i] -= s;
  }
  for (int k = n - 1; k >= 0; k--) std::swap(x[k], x[tr[k]]);  // P^T
  return x;
}

}  // namespace orc
