// lsq.h — host-side small dense least squares of the CGMRES inner loop.
//
// The reference minimises ||beta e1 - H y||^2 with scipy SLSQP (solvers.py:211-235), with
// equality constraints term0 + term1.y + y.term2.y = 0 at constrained steps (:242-255), and
// FGMRES uses np.linalg.lstsq (:113).  Here:
//   * GivensQR keeps an incremental QR of the (j+2) x (j+1) Hessenberg matrix (one rotation
//     per column), so the unconstrained LS solution is a p x p back substitution;
//   * kkt_newton solves the constrained problem by Newton's method on the KKT system, using
//     the same R, g (||beta e1 - H y||^2 = ||g - R y||^2 + rho^2), warm-started at y0 like
//     SLSQP (:225-227).
// p <= a few hundred, so this is O(p^3) host work per constrained step, microseconds.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace spis {

class GivensQR {
 public:
  void reset(int kmax, double beta);
  // append column j: h[0..j+1] = H[0:j+2, j] (solvers.py:194-196)
  void add_column(int j, const double* h);
  // y[0..p) = argmin ||beta e1 - H[:p+1,:p] y|| (p = number of columns added)
  void solve(int p, double* y) const;
  int kmax() const { return kmax_; }
  // R (p x p, column-major, leading dim kmax_+1) and g (rotated beta e1)
  const double* R() const { return R_.data(); }
  const double* g() const { return g_.data(); }
  int ld() const { return kmax_ + 1; }

 private:
  int kmax_ = 0;
  std::vector<double> R_, c_, s_, g_;
};

struct QuadCon {  // term0 + term1.y + y.term2.y (term2 row-major p x p), solvers.py:42-47
  double term0 = 0.0;
  std::vector<double> term1, term2;
};

// value of one constraint at y, evaluated as the reference's constraint_func:
// (term0 + term1 @ y) + ((y @ term2) @ y)
double con_value(const QuadCon& c, int p, const double* y);

struct KKTResult {
  int message = 0;     // spis_ls_message
  int iterations = 0;
  bool finite = true;
};

// min ||g - R y||^2  s.t.  c_i(y) = 0, i < m ; y initialised with y0.  R upper triangular
// p x p column-major with leading dimension ld.  Mirrors SLSQP's observable outcomes:
// m > p -> y = y0, message "More equality constraints than independent variables".
// lam0 (tests): receives the first start's initial multipliers (least squares on the scaled
// constraint Jacobian at y0)
KKTResult kkt_newton(int p, const double* R, int ld, const double* g, int m, const QuadCon* cons,
                     const double* y0, double* y, int max_iter = 100, std::vector<double>* lam0 = nullptr);

// dense LU with partial pivoting; returns false if singular / non-finite
bool lu_solve(int n, std::vector<double>& A /* row-major n x n, destroyed */, double* b);

}  // namespace spis
