// kdlio.hpp — TEST INFRASTRUCTURE (oracle). CPU restatement of the
// initialisation-phase LIO, VINA_SLAM::lio_state_estimation_kdtree
// (src/pipeline/odometry.cpp:267-439), for the parity
// tests of the device path. Only tests/ and bench.py's cpu_baseline load it.
//
// Third-party arithmetic restated (absent here):
//  * pcl::KdTreeFLANN::nearestKSearch (FLANN single kd-tree, exact search):
//    the k = 5 nearest map points by float squared distance, ascending; here a
//    brute-force scan, ties by map index.
//  * Eigen ColPivHouseholderQR::solve (A 5x3, b = -1): Householder QR with
//    column pivoting by the largest remaining column norm (first on ties),
//    norm downdating with the sqrt(eps) recompute rule, rank cut at
//    |pivot|^2 < (eps * max column norm)^2 / rows * (rows - k), Q^T b, upper
//    triangular back substitution, inverse column permutation. Eigen's
//    vectorised reductions are summed sequentially here (rounding-level).
#pragma once
#include <cfloat>
#include <cmath>
#include <vector>

#include "core.hpp"

namespace orc {

constexpr int kNMatch = 5;  // NMATCH, include/vina_slam/core/constants.hpp

// float squared distance in FLANN's L2_Simple order
inline float kd_sqdist(const PointType& p, float x, float y, float z) {
  const float dx = p.x - x, dy = p.y - y, dz = p.z - z;
  return (dx * dx + dy * dy) + dz * dz;
}

// k nearest (ascending distance, ties by index)
inline int knn_brute(const std::vector<PointType>& pts, float x, float y, float z, int k, int* idx, float* sq) {
  int cnt = 0;
  for (int i = 0; i < (int)pts.size(); i++) {
    const float d = kd_sqdist(pts[i], x, y, z);
    if (cnt == k && !(d < sq[k - 1])) continue;
    int pos = cnt < k ? cnt++ : k - 1;
    while (pos > 0 && sq[pos - 1] > d) {
      sq[pos] = sq[pos - 1];
      idx[pos] = idx[pos - 1];
      pos--;
    }
    sq[pos] = d;
    idx[pos] = i;
  }
  return cnt;
}

// ColPivHouseholderQR(A).solve(b), A m x 3 (m <= 8), column-major scratch
inline void colpiv_qr_solve(const double* Ain, int m, const double* b, double* x) {
  const int n = 3, size = m < n ? m : n;
  double A[8 * 3];  // A[r * 3 + c]
  for (int i = 0; i < m * n; i++) A[i] = Ain[i];
  double tau[3], normU[3], normD[3];
  int trans[3];
  double maxnorm = 0.0;
  for (int j = 0; j < n; j++) {
    double s = 0.0;
    for (int r = 0; r < m; r++) s += A[r * 3 + j] * A[r * 3 + j];
    normD[j] = normU[j] = std::sqrt(s);
    if (normU[j] > maxnorm) maxnorm = normU[j];
  }
  const double eps = DBL_EPSILON;
  const double thr_helper = (maxnorm * eps) * (maxnorm * eps) / m;
  const double downdate_thr = std::sqrt(eps);
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
    // makeHouseholderInPlace on A[k:, k]
    double tail = 0.0;
    for (int r = k + 1; r < m; r++) tail += A[r * 3 + k] * A[r * 3 + k];
    const double c0 = A[k * 3 + k];
    double beta;
    if (tail <= DBL_MIN) {
      tau[k] = 0.0;
      beta = c0;
      for (int r = k + 1; r < m; r++) A[r * 3 + k] = 0.0;
    } else {
      beta = std::sqrt(c0 * c0 + tail);
      if (c0 >= 0.0) beta = -beta;
      for (int r = k + 1; r < m; r++) A[r * 3 + k] = A[r * 3 + k] / (c0 - beta);
      tau[k] = (beta - c0) / beta;
    }
    A[k * 3 + k] = beta;
    // applyHouseholderOnTheLeft to A[k:, k+1:]
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
    // column norm downdate
    for (int j = k + 1; j < n; j++) {
      if (normU[j] != 0.0) {
        double t = std::fabs(A[k * 3 + j]) / normU[j];
        t = (1.0 + t) * (1.0 - t);
        if (t < 0.0) t = 0.0;
        const double q = normU[j] / normD[j];
        const double t2 = t * q * q;
        if (t2 <= downdate_thr) {
          double s = 0.0;
          for (int r = k + 1; r < m; r++) s += A[r * 3 + j] * A[r * 3 + j];
          normD[j] = std::sqrt(s);
          normU[j] = normD[j];
        } else {
          normU[j] *= std::sqrt(t);
        }
      }
    }
  }
  // solve: c = Q^T b over the nonzero pivots, back substitution, permutation
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

}  // namespace orc
