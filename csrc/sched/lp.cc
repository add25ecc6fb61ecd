#include "sched/lp.h"

#include <algorithm>
#include <cmath>
#include <limits>

namespace dissem {

namespace {

constexpr double kEps = 1e-10;    // pivot / reduced-cost tolerance
constexpr double kFeas = 1e-8;    // phase-1 residual counted as feasible

struct Tableau {
  int m = 0, W = 0;                // rows (constraints), row stride (columns + rhs)
  std::vector<double> t;           // (m + 1) x W, last row = reduced costs, last column = rhs
  std::vector<int> basis;          // basic column of each row
  double& at(int i, int j) { return t[size_t(i) * size_t(W) + size_t(j)]; }
  double* row(int i) { return &t[size_t(i) * size_t(W)]; }

  void pivot(int r, int c) {
    double* pr = row(r);
    const double inv = 1.0 / pr[c];
    for (int j = 0; j < W; ++j) pr[j] *= inv;
    pr[c] = 1.0;
    for (int i = 0; i <= m; ++i) {
      if (i == r) continue;
      double* pi = row(i);
      const double f = pi[c];
      if (f == 0.0) continue;
      for (int j = 0; j < W; ++j) pi[j] -= f * pr[j];
      pi[c] = 0.0;
    }
    basis[size_t(r)] = c;
  }

  // Minimize the objective in the last row over the columns `allowed` lets in.
  // Returns "optimal", "unbounded" or "iteration limit".
  template <class Allowed>
  const char* run(Allowed allowed, int ncols, int& pivots, int max_pivots, bool always_bland = false) {
    int degenerate = 0;
    for (;;) {
      if (pivots >= max_pivots) return "iteration limit";
      double* obj = row(m);
      int c = -1;
      const bool bland = always_bland || degenerate > 50;
      double best = -kEps;
      for (int j = 0; j < ncols; ++j) {
        if (!allowed(j) || obj[j] >= -kEps) continue;
        if (bland) {
          c = j;
          break;
        }
        if (obj[j] < best) {
          best = obj[j];
          c = j;
        }
      }
      if (c < 0) return "optimal";
      int r = -1;
      double ratio = std::numeric_limits<double>::infinity();
      for (int i = 0; i < m; ++i) {
        const double a = at(i, c);
        if (a <= kEps) continue;
        const double q = std::max(0.0, at(i, W - 1)) / a;
        if (q < ratio - 1e-14 || (q <= ratio + 1e-14 && r >= 0 && basis[size_t(i)] < basis[size_t(r)])) {
          ratio = q;
          r = i;
        }
      }
      if (r < 0) return "unbounded";
      degenerate = ratio <= 1e-14 ? degenerate + 1 : 0;
      pivot(r, c);
      ++pivots;
    }
  }
};

}  // namespace

namespace {
LpResult solve_once(const LpProblem& p, int max_pivots, bool bland);
}

LpResult solve_lp(const LpProblem& p, int max_pivots) {
  // Dantzig's rule first (fast); an instance it loses to round-off on long
  // degenerate stretches (a spurious "unbounded"/"infeasible", seen with
  // measured link rates next to planning constants) is solved again with
  // Bland's rule from the start, which never cycles, and then with every row
  // equilibrated (divided by its largest coefficient: the same feasible set,
  // pivots of one magnitude).
  LpResult r = solve_once(p, max_pivots, false);
  if (r.ok) return r;
  LpResult b = solve_once(p, max_pivots, true);
  b.pivots += r.pivots;
  if (b.ok) return b;
  LpProblem q = p;
  for (auto* rows : {&q.eq, &q.le})
    for (auto& row : *rows) {
      double mx = 0;
      for (auto& e : row.a) mx = std::max(mx, std::fabs(e.second));
      if (mx <= 0) continue;
      for (auto& e : row.a) e.second /= mx;
      row.b /= mx;
    }
  LpResult e = solve_once(q, max_pivots, true);
  e.pivots += b.pivots;
  if (!e.ok) e.status = r.status + " / bland: " + b.status + " / equilibrated: " + e.status;
  return e;
}

namespace {
LpResult solve_once(const LpProblem& p, int max_pivots, bool bland) {
  LpResult res;
  const int n = p.n, neq = int(p.eq.size()), nle = int(p.le.size());
  const int m = neq + nle;
  const int slack0 = n, art0 = n + nle, ncols = n + nle + neq;
  Tableau T;
  T.m = m;
  T.W = ncols + 1;
  T.t.assign(size_t(m + 1) * size_t(T.W), 0.0);
  T.basis.assign(size_t(m), -1);
  for (int i = 0; i < neq; ++i) {
    const LpRow& r = p.eq[size_t(i)];
    for (auto& e : r.a) T.at(i, e.first) += e.second;
    const double sgn = r.b < 0 ? -1.0 : 1.0;  // keep every rhs >= 0
    if (sgn < 0)
      for (int j = 0; j < n; ++j) T.at(i, j) = -T.at(i, j);
    T.at(i, T.W - 1) = sgn * r.b;
    T.at(i, art0 + i) = 1.0;
    T.basis[size_t(i)] = art0 + i;
  }
  for (int k = 0; k < nle; ++k) {
    const int i = neq + k;
    const LpRow& r = p.le[size_t(k)];
    if (r.b < 0) {
      res.status = "negative rhs on a <= row";
      return res;
    }
    for (auto& e : r.a) T.at(i, e.first) += e.second;
    T.at(i, slack0 + k) = 1.0;
    T.at(i, T.W - 1) = r.b;
    T.basis[size_t(i)] = slack0 + k;
  }
  // Phase 1: minimize the sum of the artificials (reduced costs = -column sums of the eq rows).
  {
    double* obj = T.row(m);
    for (int i = 0; i < neq; ++i) {
      const double* ri = T.row(i);
      for (int j = 0; j < art0; ++j) obj[j] -= ri[j];
      obj[T.W - 1] -= ri[T.W - 1];
    }
    const char* st = T.run([&](int j) { return j < art0; }, ncols, res.pivots, max_pivots, bland);
    if (std::string(st) != "optimal") {
      res.status = st;
      return res;
    }
    if (-T.at(m, T.W - 1) > kFeas) {
      res.status = "infeasible";
      return res;
    }
    // Drive artificials still basic (at 0) out of the basis where a real column can replace them.
    for (int i = 0; i < m; ++i) {
      if (T.basis[size_t(i)] < art0) continue;
      for (int j = 0; j < art0; ++j)
        if (std::fabs(T.at(i, j)) > 1e-9) {
          T.pivot(i, j);
          ++res.pivots;
          break;
        }
    }
  }
  // Phase 2: reduced costs of the real objective for the current basis.
  {
    double* obj = T.row(m);
    std::fill(obj, obj + T.W, 0.0);
    for (int j = 0; j < n; ++j) obj[j] = p.c[size_t(j)];
    for (int i = 0; i < m; ++i) {
      const int b = T.basis[size_t(i)];
      const double cb = b < n ? p.c[size_t(b)] : 0.0;
      if (cb == 0.0) continue;
      const double* ri = T.row(i);
      for (int j = 0; j < T.W; ++j) obj[j] -= cb * ri[j];
    }
    const char* st = T.run([&](int j) { return j < art0; }, ncols, res.pivots, max_pivots, bland);
    res.status = st;
    if (std::string(st) != "optimal") return res;
  }
  res.ok = true;
  res.x.assign(size_t(n), 0.0);
  for (int i = 0; i < m; ++i)
    if (T.basis[size_t(i)] < n) res.x[size_t(T.basis[size_t(i)])] = std::max(0.0, T.at(i, T.W - 1));
  res.obj = 0;
  for (int j = 0; j < n; ++j) res.obj += p.c[size_t(j)] * res.x[size_t(j)];
  return res;
}
}  // namespace

}  // namespace dissem
