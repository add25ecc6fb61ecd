// Small dense linear programs for the mode-3 planner (sched/maxflow.cc).
//
//   minimize c.x  subject to  A_eq x = b_eq (b_eq >= 0),  A_le x <= b_le (b_le >= 0),  x >= 0
//
// Two-phase primal simplex on a dense tableau: phase 1 drives the equality
// rows' artificial variables out, phase 2 minimizes c.x. Dantzig pricing with
// a switch to Bland's rule after a run of degenerate pivots (no cycling).
// Sized for the planner's aggregated instances (hundreds of rows/columns);
// callers scale their data so coefficients are O(1).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace dissem {

struct LpRow {
  std::vector<std::pair<int, double>> a;  // (column, coefficient)
  double b = 0;
};

struct LpProblem {
  int n = 0;                 // columns
  std::vector<double> c;     // objective, size n
  std::vector<LpRow> eq, le;
};

struct LpResult {
  bool ok = false;           // optimal solution found
  std::string status;        // "optimal", "infeasible", "unbounded", "iteration limit"
  double obj = 0;
  std::vector<double> x;
  int pivots = 0;
};

LpResult solve_lp(const LpProblem& p, int max_pivots = 200000);

}  // namespace dissem
