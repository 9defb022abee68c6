// ORACLE — TEST INFRASTRUCTURE ONLY.
// Eigen::LDLT (lower storage, diagonal pivoting: the pivot at step k is the largest |diagonal| of the
// not yet factored part, first index on ties) + solve, restated for the solves of
// EnergyFunctional::solveSystemF (Src/EnergyFunctional.cpp:799-801) and
// CoarseTracker::trackNewestCoarse (Src/CoarseTracker.cpp:561-563).  Eigen is not vendored by the
// reference (version unpinned): the solve is parity unpinned and compared with a tolerance.
#pragma once
#include <cmath>
#include <limits>
#include <utility>
#include <vector>

namespace hso {

// Eigen::LDLT<MatrixXd> (lower, diagonal pivoting) + solve, in place on a copy.
inline void ldlt_solve(std::vector<double> A, int n, const std::vector<double>& b, std::vector<double>& x) {
  std::vector<int> transp(n);
  std::vector<double> temp(n);
  auto at = [&](int i, int j) -> double& { return A[i * n + j]; };
  for (int k = 0; k < n; k++) {
    int idx = k;
    double best = std::fabs(at(k, k));
    for (int i = k + 1; i < n; i++)
      if (std::fabs(at(i, i)) > best) { best = std::fabs(at(i, i)); idx = i; }
    transp[k] = idx;
    if (k != idx) {
      // symmetric swap of rows/cols k and idx (lower triangle semantics; we keep full matrix)
      for (int j = 0; j < n; j++) std::swap(at(k, j), at(idx, j));
      for (int i = 0; i < n; i++) std::swap(at(i, k), at(i, idx));
    }
    const int rs = n - k - 1;
    if (k > 0) {
      for (int j = 0; j < k; j++) temp[j] = at(j, j) * at(k, j);
      double s = 0;
      for (int j = 0; j < k; j++) s += at(k, j) * temp[j];
      at(k, k) -= s;
      for (int i = k + 1; i < n; i++) {
        double t = 0;
        for (int j = 0; j < k; j++) t += at(i, j) * temp[j];
        at(i, k) -= t;
      }
    }
    double akk = at(k, k);
    bool valid = std::fabs(akk) > std::numeric_limits<double>::min();
    if (rs > 0 && valid)
      for (int i = k + 1; i < n; i++) at(i, k) /= akk;
    // keep the upper triangle consistent with the lower (we swap full rows/cols)
    for (int i = k + 1; i < n; i++) at(k, i) = at(i, k);
  }
  // solve: x = P b ; L y = x ; y /= D ; L^T z = y ; P^T z
  x = b;
  for (int k = 0; k < n; k++)
    if (transp[k] != k) std::swap(x[k], x[transp[k]]);
  for (int i = 0; i < n; i++)
    for (int j = 0; j < i; j++) x[i] -= at(i, j) * x[j];
  for (int i = 0; i < n; i++) {
    if (std::fabs(at(i, i)) > std::numeric_limits<double>::min()) x[i] /= at(i, i);
    else x[i] = 0;
  }
  for (int i = n - 1; i >= 0; i--)
    for (int j = i + 1; j < n; j++) x[i] -= at(j, i) * x[j];
  for (int k = n - 1; k >= 0; k--)
    if (transp[k] != k) std::swap(x[k], x[transp[k]]);
}

}  // namespace hso
