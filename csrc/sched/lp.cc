#include "sched/lp.h"

#include <algorithm>
#include <cmath>
#include <limits>

namespace dissem {

namespace {

constexpr double kInfB = std::numeric_limits<double>::infinity();

// The working model: every row an equality (a slack per <= row, an
// artificial per = row), columns stored sparse, bounds per column.
struct Model {
  int m = 0, n = 0;                 // rows, columns (structural + slacks + artificials)
  int n_struct = 0, art0 = 0;       // first artificial column
  std::vector<int> cstart, ridx;    // column-major sparse matrix
  std::vector<double> val;
  std::vector<double> lo, up, cost, b;
  std::vector<double> rscale, cscale;  // a'_ij = rscale_i a_ij cscale_j
};

Model build(const LpProblem& p) {
  Model md;
  const int neq = int(p.eq.size()), nle = int(p.le.size());
  md.m = neq + nle;
  md.n_struct = p.n;
  md.art0 = p.n + nle;
  md.n = p.n + nle + neq;
  std::vector<std::vector<std::pair<int, double>>> cols(size_t(md.n));
  md.b.assign(size_t(md.m), 0.0);
  for (int i = 0; i < neq; ++i) {
    const LpRow& r = p.eq[size_t(i)];
    const double sgn = r.b < 0 ? -1.0 : 1.0;  // rhs >= 0: the artificial starts feasible
    for (auto& e : r.a) cols[size_t(e.first)].push_back({i, sgn * e.second});
    md.b[size_t(i)] = sgn * r.b;
    cols[size_t(md.art0 + i)].push_back({i, 1.0});
  }
  for (int k = 0; k < nle; ++k) {
    const int i = neq + k;
    const LpRow& r = p.le[size_t(k)];
    for (auto& e : r.a) cols[size_t(e.first)].push_back({i, e.second});
    md.b[size_t(i)] = r.b;
    cols[size_t(p.n + k)].push_back({i, 1.0});
  }
  // merge duplicate (row, col) entries
  md.cstart.push_back(0);
  for (auto& c : cols) {
    std::sort(c.begin(), c.end());
    for (size_t q = 0; q < c.size(); ++q) {
      if (!md.ridx.empty() && int(md.ridx.size()) > md.cstart.back() && md.ridx.back() == c[q].first) {
        md.val.back() += c[q].second;
        continue;
      }
      md.ridx.push_back(c[q].first);
      md.val.push_back(c[q].second);
    }
    md.cstart.push_back(int(md.ridx.size()));
  }
  md.lo.assign(size_t(md.n), 0.0);
  md.up.assign(size_t(md.n), kInfB);
  md.cost.assign(size_t(md.n), 0.0);
  for (int j = 0; j < p.n; ++j) md.cost[size_t(j)] = p.c[size_t(j)];
  md.rscale.assign(size_t(md.m), 1.0);
  md.cscale.assign(size_t(md.n), 1.0);
  return md;
}

// Geometric-mean scaling of rows and structural columns (a few passes), then
// every slack / artificial column rescaled back to a unit entry. Rates that
// span orders of magnitude (measured links next to planning constants, 1e6 to
// 5e10 B/s) become coefficients of one magnitude.
void scale(Model& md) {
  const int m = md.m;
  std::vector<double> rmin(static_cast<size_t>(m)), rmax(static_cast<size_t>(m));
  for (int pass = 0; pass < 6; ++pass) {
    std::fill(rmin.begin(), rmin.end(), kInfB);
    std::fill(rmax.begin(), rmax.end(), 0.0);
    for (int j = 0; j < md.n_struct; ++j)
      for (int q = md.cstart[size_t(j)]; q < md.cstart[size_t(j) + 1]; ++q) {
        const double a = std::fabs(md.val[size_t(q)] * md.rscale[size_t(md.ridx[size_t(q)])] * md.cscale[size_t(j)]);
        if (a == 0) continue;
        const int i = md.ridx[size_t(q)];
        rmin[size_t(i)] = std::min(rmin[size_t(i)], a);
        rmax[size_t(i)] = std::max(rmax[size_t(i)], a);
      }
    for (int i = 0; i < m; ++i)
      if (rmax[size_t(i)] > 0) md.rscale[size_t(i)] /= std::sqrt(rmin[size_t(i)] * rmax[size_t(i)]);
    for (int j = 0; j < md.n_struct; ++j) {
      double lo = kInfB, hi = 0;
      for (int q = md.cstart[size_t(j)]; q < md.cstart[size_t(j) + 1]; ++q) {
        const double a = std::fabs(md.val[size_t(q)] * md.rscale[size_t(md.ridx[size_t(q)])] * md.cscale[size_t(j)]);
        if (a == 0) continue;
        lo = std::min(lo, a);
        hi = std::max(hi, a);
      }
      if (hi > 0) md.cscale[size_t(j)] /= std::sqrt(lo * hi);
    }
  }
  // powers of two: scaling then changes no mantissa
  auto p2 = [](double s) { return std::ldexp(1.0, int(std::lround(std::log2(s)))); };
  for (auto& s : md.rscale) s = p2(s);
  for (int j = 0; j < md.n_struct; ++j) md.cscale[size_t(j)] = p2(md.cscale[size_t(j)]);
  for (int j = md.n_struct; j < md.n; ++j)  // slack / artificial: one entry, kept at 1
    md.cscale[size_t(j)] = 1.0 / md.rscale[size_t(md.ridx[size_t(md.cstart[size_t(j)])])];
  for (int j = 0; j < md.n; ++j) {
    for (int q = md.cstart[size_t(j)]; q < md.cstart[size_t(j) + 1]; ++q)
      md.val[size_t(q)] *= md.rscale[size_t(md.ridx[size_t(q)])] * md.cscale[size_t(j)];
    md.cost[size_t(j)] *= md.cscale[size_t(j)];
    md.lo[size_t(j)] /= md.cscale[size_t(j)];
    if (md.up[size_t(j)] < kInfB) md.up[size_t(j)] /= md.cscale[size_t(j)];
  }
  for (int i = 0; i < m; ++i) md.b[size_t(i)] *= md.rscale[size_t(i)];
}

enum class St : uint8_t { Basic, Lower, Upper };

// Bounded primal revised simplex on an explicit dense basis inverse:
// Dantzig pricing (Bland's rule on long degenerate stretches, which cannot
// cycle), Harris's two-pass ratio test (bound-flip aware), product-form
// updates of the inverse and a fresh inverse (LU with partial pivoting)
// every kReinvert pivots and before any verdict, so round-off cannot pile up.
class Simplex {
 public:
  Simplex(Model& md, int max_pivots) : md_(md), m_(md.m), n_(md.n), max_pivots_(max_pivots) {
    binv_.assign(size_t(m_) * size_t(m_), 0.0);
    basis_.assign(size_t(m_), -1);
    st_.assign(size_t(n_), St::Lower);
    x_.assign(size_t(n_), 0.0);
    // slack basis for <= rows, artificial basis for = rows
    const int neq = n_ - md_.art0;
    for (int i = 0; i < m_; ++i) {
      const int j = i < neq ? md_.art0 + i : md_.n_struct + (i - neq);
      basis_[size_t(i)] = j;
      st_[size_t(j)] = St::Basic;
    }
  }

  int pivots = 0;

  // phase 1: minimize the artificials; then phase 2 with them fixed at 0
  std::string solve() {
    const int neq = n_ - md_.art0;
    std::vector<double> c1(size_t(n_), 0.0);
    for (int j = md_.art0; j < n_; ++j) c1[size_t(j)] = 1.0;
    if (!reinvert()) return "singular basis";
    if (neq > 0) {
      std::string s = run(c1);
      if (s != "optimal") return s;
      double infeas = 0;
      for (int j = md_.art0; j < n_; ++j) infeas += std::fabs(x_[size_t(j)]);
      double bnorm = 1;
      for (double v : md_.b) bnorm = std::max(bnorm, std::fabs(v));
      if (infeas > 1e-7 * bnorm) return "infeasible";
    }
    for (int j = md_.art0; j < n_; ++j) {  // artificials: fixed at zero from now on
      md_.up[size_t(j)] = 0.0;
      if (st_[size_t(j)] != St::Basic) {
        st_[size_t(j)] = St::Lower;
        x_[size_t(j)] = 0.0;
      }
    }
    recompute_basic();  // phase 1 ended on a verified inverse
    return run(md_.cost);
  }

  const std::vector<double>& x() const { return x_; }

 private:
  static constexpr int kReinvert = 100;
  static constexpr int kTrustUpdates = 8;  // product-form updates a verdict may rest on without reinversion
  static constexpr double kPivTol = 1e-9;   // |alpha| below this never pivots
  static constexpr double kFeasTol = 1e-9;  // primal bound tolerance (Harris's slack)
  static constexpr double kDualTol = 1e-9;

  Model& md_;
  int m_, n_;
  int max_pivots_;
  std::vector<double> binv_;  // row-major m x m
  std::vector<int> basis_;
  std::vector<St> st_;
  std::vector<double> x_;
  int since_inv_ = 0;

  double& B(int i, int k) { return binv_[size_t(i) * size_t(m_) + size_t(k)]; }

  // B^-1 from scratch (Gauss-Jordan with partial pivoting on the basis
  // columns), then the basic values from the nonbasic ones.
  bool reinvert() {
    // A basis of unit columns (slacks / artificials: the starting basis) is its
    // own inverse up to the entries' reciprocals.
    bool unit = true;
    for (int k = 0; k < m_ && unit; ++k) {
      const int j = basis_[size_t(k)];
      unit = md_.cstart[size_t(j) + 1] - md_.cstart[size_t(j)] == 1 && md_.ridx[size_t(md_.cstart[size_t(j)])] == k;
    }
    if (unit) {
      std::fill(binv_.begin(), binv_.end(), 0.0);
      for (int k = 0; k < m_; ++k) B(k, k) = 1.0 / md_.val[size_t(md_.cstart[size_t(basis_[size_t(k)])])];
      recompute_basic();
      since_inv_ = 0;
      return true;
    }
    std::vector<double> a(size_t(m_) * size_t(m_), 0.0);
    for (int k = 0; k < m_; ++k) {
      const int j = basis_[size_t(k)];
      for (int q = md_.cstart[size_t(j)]; q < md_.cstart[size_t(j) + 1]; ++q)
        a[size_t(md_.ridx[size_t(q)]) * size_t(m_) + size_t(k)] = md_.val[size_t(q)];
    }
    std::fill(binv_.begin(), binv_.end(), 0.0);
    for (int i = 0; i < m_; ++i) B(i, i) = 1.0;
    for (int c = 0; c < m_; ++c) {
      int pr = c;
      double best = std::fabs(a[size_t(c) * size_t(m_) + size_t(c)]);
      for (int r = c + 1; r < m_; ++r) {
        const double v = std::fabs(a[size_t(r) * size_t(m_) + size_t(c)]);
        if (v > best) {
          best = v;
          pr = r;
        }
      }
      if (best < 1e-13) return false;
      if (pr != c) {
        for (int k = 0; k < m_; ++k) {
          std::swap(a[size_t(pr) * size_t(m_) + size_t(k)], a[size_t(c) * size_t(m_) + size_t(k)]);
          std::swap(B(pr, k), B(c, k));
        }
      }
      const double inv = 1.0 / a[size_t(c) * size_t(m_) + size_t(c)];
      for (int k = 0; k < m_; ++k) {
        a[size_t(c) * size_t(m_) + size_t(k)] *= inv;
        B(c, k) *= inv;
      }
      for (int r = 0; r < m_; ++r) {
        if (r == c) continue;
        const double f = a[size_t(r) * size_t(m_) + size_t(c)];
        if (f == 0.0) continue;
        for (int k = 0; k < m_; ++k) {
          a[size_t(r) * size_t(m_) + size_t(k)] -= f * a[size_t(c) * size_t(m_) + size_t(k)];
          B(r, k) -= f * B(c, k);
        }
      }
    }
    // row k of the inverse belongs to basis_[k] (the columns were placed in order)
    recompute_basic();
    since_inv_ = 0;
    return true;
  }

  void recompute_basic() {
    std::vector<double> r = md_.b;
    for (int j = 0; j < n_; ++j) {
      if (st_[size_t(j)] == St::Basic) continue;
      x_[size_t(j)] = st_[size_t(j)] == St::Upper ? md_.up[size_t(j)] : md_.lo[size_t(j)];
      const double v = x_[size_t(j)];
      if (v == 0.0) continue;
      for (int q = md_.cstart[size_t(j)]; q < md_.cstart[size_t(j) + 1]; ++q)
        r[size_t(md_.ridx[size_t(q)])] -= md_.val[size_t(q)] * v;
    }
    for (int i = 0; i < m_; ++i) {
      double s = 0;
      for (int k = 0; k < m_; ++k) s += B(i, k) * r[size_t(k)];
      x_[size_t(basis_[size_t(i)])] = s;
    }
  }

  std::string run(const std::vector<double>& c) {
    std::vector<double> y(static_cast<size_t>(m_)), alpha(static_cast<size_t>(m_));
    int degenerate = 0;
    bool verified = false;  // optimality confirmed on a fresh inverse
    for (;;) {
      if (pivots >= max_pivots_) return "iteration limit";
      if (since_inv_ >= kReinvert && !reinvert()) return "singular basis";
      // duals y = c_B B^-1
      std::fill(y.begin(), y.end(), 0.0);
      for (int i = 0; i < m_; ++i) {
        const double cb = c[size_t(basis_[size_t(i)])];
        if (cb == 0.0) continue;
        for (int k = 0; k < m_; ++k) y[size_t(k)] += cb * B(i, k);
      }
      // pricing
      const bool bland = degenerate > 30;
      int q = -1;
      double best = 0;
      for (int j = 0; j < n_; ++j) {
        if (st_[size_t(j)] == St::Basic) continue;
        if (md_.lo[size_t(j)] == md_.up[size_t(j)]) continue;  // fixed (artificials in phase 2)
        double d = c[size_t(j)];
        for (int p = md_.cstart[size_t(j)]; p < md_.cstart[size_t(j) + 1]; ++p)
          d -= y[size_t(md_.ridx[size_t(p)])] * md_.val[size_t(p)];
        const bool cand = (st_[size_t(j)] == St::Lower && d < -kDualTol) || (st_[size_t(j)] == St::Upper && d > kDualTol);
        if (!cand) continue;
        if (bland) {
          q = j;
          break;
        }
        if (std::fabs(d) > best) {
          best = std::fabs(d);
          q = j;
        }
      }
      if (q < 0) {
        // a verdict on an inverse that saw few updates stands; after many, it is
        // confirmed on a fresh one
        if (verified || since_inv_ <= kTrustUpdates) return "optimal";
        if (!reinvert()) return "singular basis";  // confirm on a fresh inverse
        verified = true;
        continue;
      }
      verified = false;
      const double dir = st_[size_t(q)] == St::Lower ? 1.0 : -1.0;
      // alpha = B^-1 a_q
      std::fill(alpha.begin(), alpha.end(), 0.0);
      for (int p = md_.cstart[size_t(q)]; p < md_.cstart[size_t(q) + 1]; ++p) {
        const int k = md_.ridx[size_t(p)];
        const double v = md_.val[size_t(p)];
        for (int i = 0; i < m_; ++i) alpha[size_t(i)] += B(i, k) * v;
      }
      // Harris pass 1: the largest step every basic variable allows with its
      // bound relaxed by the feasibility tolerance
      double tmax = kInfB;
      for (int i = 0; i < m_; ++i) {
        const double a = dir * alpha[size_t(i)];  // x_B(i) moves by -a * t
        const int j = basis_[size_t(i)];
        if (a > kPivTol) {
          if (md_.lo[size_t(j)] > -kInfB) tmax = std::min(tmax, (x_[size_t(j)] - md_.lo[size_t(j)] + kFeasTol) / a);
        } else if (a < -kPivTol) {
          if (md_.up[size_t(j)] < kInfB) tmax = std::min(tmax, (md_.up[size_t(j)] - x_[size_t(j)] + kFeasTol) / -a);
        }
      }
      const double span = md_.up[size_t(q)] - md_.lo[size_t(q)];
      if (tmax == kInfB && !(span < kInfB)) return "unbounded";
      // pass 2: among the rows whose exact ratio is within that step, the
      // largest pivot
      int r = -1;
      double rt = 0, pbest = 0;
      if (tmax < kInfB) {
        for (int i = 0; i < m_; ++i) {
          const double a = dir * alpha[size_t(i)];
          const int j = basis_[size_t(i)];
          double ratio;
          if (a > kPivTol && md_.lo[size_t(j)] > -kInfB) ratio = (x_[size_t(j)] - md_.lo[size_t(j)]) / a;
          else if (a < -kPivTol && md_.up[size_t(j)] < kInfB) ratio = (md_.up[size_t(j)] - x_[size_t(j)]) / -a;
          else continue;
          if (ratio <= tmax && std::fabs(a) > pbest) {
            pbest = std::fabs(a);
            r = i;
            rt = std::max(0.0, ratio);
          }
        }
      }
      if (span < kInfB && (r < 0 || span <= rt)) {
        // bound flip: the entering variable reaches its other bound first
        for (int i = 0; i < m_; ++i) x_[size_t(basis_[size_t(i)])] -= dir * span * alpha[size_t(i)];
        st_[size_t(q)] = st_[size_t(q)] == St::Lower ? St::Upper : St::Lower;
        x_[size_t(q)] = st_[size_t(q)] == St::Upper ? md_.up[size_t(q)] : md_.lo[size_t(q)];
        ++pivots;
        degenerate = 0;
        continue;
      }
      if (r < 0) return "unbounded";
      degenerate = rt <= 1e-12 ? degenerate + 1 : 0;
      // step
      for (int i = 0; i < m_; ++i) x_[size_t(basis_[size_t(i)])] -= dir * rt * alpha[size_t(i)];
      x_[size_t(q)] += dir * rt;
      const int leave = basis_[size_t(r)];
      const double a_r = dir * alpha[size_t(r)];
      // the leaving variable sits at the bound it reached
      if (a_r > 0) {
        st_[size_t(leave)] = St::Lower;
        x_[size_t(leave)] = md_.lo[size_t(leave)];
      } else {
        st_[size_t(leave)] = St::Upper;
        x_[size_t(leave)] = md_.up[size_t(leave)];
      }
      basis_[size_t(r)] = q;
      st_[size_t(q)] = St::Basic;
      // product-form update of the inverse: pivot on alpha_r
      const double inv = 1.0 / alpha[size_t(r)];
      double* br = &binv_[size_t(r) * size_t(m_)];
      for (int k = 0; k < m_; ++k) br[k] *= inv;
      for (int i = 0; i < m_; ++i) {
        if (i == r) continue;
        const double f = alpha[size_t(i)];
        if (f == 0.0) continue;
        double* bi = &binv_[size_t(i) * size_t(m_)];
        for (int k = 0; k < m_; ++k) bi[k] -= f * br[k];
      }
      ++pivots;
      ++since_inv_;
    }
  }
};

LpResult solve_scaled(const LpProblem& p, int max_pivots, bool do_scale) {
  LpResult res;
  for (auto& r : p.le)
    if (r.b < 0) {
      res.status = "negative rhs on a <= row";
      return res;
    }
  Model md = build(p);
  if (do_scale) scale(md);
  Simplex sx(md, max_pivots);
  res.status = sx.solve();
  res.pivots = sx.pivots;
  if (res.status != "optimal") return res;
  res.ok = true;
  res.x.assign(size_t(p.n), 0.0);
  for (int j = 0; j < p.n; ++j) res.x[size_t(j)] = std::max(0.0, sx.x()[size_t(j)] * md.cscale[size_t(j)]);
  res.obj = 0;
  for (int j = 0; j < p.n; ++j) res.obj += p.c[size_t(j)] * res.x[size_t(j)];
  return res;
}

}  // namespace

LpResult solve_lp(const LpProblem& p, int max_pivots) {
  LpResult r = solve_scaled(p, max_pivots, true);
  if (r.ok || r.status == "infeasible" || r.status == "negative rhs on a <= row") return r;
  // a scaled model the factorization found singular: once more unscaled
  LpResult u = solve_scaled(p, max_pivots, false);
  u.pivots += r.pivots;
  if (!u.ok) u.status = r.status + " / unscaled: " + u.status;
  return u;
}

}  // namespace dissem
