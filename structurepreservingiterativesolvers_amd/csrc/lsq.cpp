// lsq.cpp — host-side small dense least squares (see lsq.h).
#include "lsq.h"

#include <algorithm>
#include <cfloat>
#include <cmath>

#include "spis.h"

namespace spis {

void GivensQR::reset(int kmax, double beta) {
  kmax_ = kmax;
  R_.assign(static_cast<size_t>(kmax + 1) * (kmax > 0 ? kmax : 1), 0.0);
  c_.assign(kmax > 0 ? kmax : 1, 1.0);
  s_.assign(kmax > 0 ? kmax : 1, 0.0);
  g_.assign(kmax + 1, 0.0);
  g_[0] = beta;
}

void GivensQR::add_column(int j, const double* h) {
  const int ld = kmax_ + 1;
  double* col = R_.data() + static_cast<size_t>(j) * ld;
  for (int i = 0; i <= j + 1; ++i) col[i] = h[i];
  for (int i = 0; i < j; ++i) {
    const double a = col[i], b = col[i + 1];
    col[i] = c_[i] * a + s_[i] * b;
    col[i + 1] = -s_[i] * a + c_[i] * b;
  }
  const double a = col[j], b = col[j + 1];
  double c = 1.0, s = 0.0, r = a;
  if (b != 0.0) {
    r = std::hypot(a, b);
    c = a / r;
    s = b / r;
  }
  c_[j] = c;
  s_[j] = s;
  col[j] = r;
  col[j + 1] = 0.0;
  const double gj = g_[j];
  g_[j] = c * gj;
  g_[j + 1] = -s * gj;
}

void GivensQR::solve(int p, double* y) const {
  const int ld = kmax_ + 1;
  for (int i = p - 1; i >= 0; --i) {
    double t = g_[i];
    for (int k = i + 1; k < p; ++k) t -= R_[static_cast<size_t>(k) * ld + i] * y[k];
    const double d = R_[static_cast<size_t>(i) * ld + i];
    y[i] = d != 0.0 ? t / d : 0.0;  // exactly singular column (cgmres_p after a breakdown)
  }
}

double con_value(const QuadCon& c, int p, const double* y) {
  double lin = 0.0;
  for (int a = 0; a < p; ++a) lin += c.term1[a] * y[a];
  double quad = 0.0;
  for (int b = 0; b < p; ++b) {
    double u = 0.0;
    for (int a = 0; a < p; ++a) u += y[a] * c.term2[static_cast<size_t>(a) * p + b];
    quad += u * y[b];
  }
  return (c.term0 + lin) + quad;
}

// magnitude of the terms summed by con_value: the rounding scale of a computed value
static double con_scale(const QuadCon& c, int p, const double* y) {
  double s = std::fabs(c.term0);
  for (int a = 0; a < p; ++a) s += std::fabs(c.term1[a] * y[a]);
  for (int a = 0; a < p; ++a)
    for (int b = 0; b < p; ++b) s += std::fabs(y[a] * c.term2[static_cast<size_t>(a) * p + b] * y[b]);
  return s;
}

bool lu_solve(int n, std::vector<double>& A, double* b) {
  for (int k = 0; k < n; ++k) {
    int piv = k;
    double best = std::fabs(A[static_cast<size_t>(k) * n + k]);
    for (int i = k + 1; i < n; ++i) {
      const double v = std::fabs(A[static_cast<size_t>(i) * n + k]);
      if (v > best) { best = v; piv = i; }
    }
    if (!(best > 0.0) || !std::isfinite(best)) return false;
    if (piv != k) {
      for (int j = 0; j < n; ++j) std::swap(A[static_cast<size_t>(k) * n + j], A[static_cast<size_t>(piv) * n + j]);
      std::swap(b[k], b[piv]);
    }
    const double d = A[static_cast<size_t>(k) * n + k];
    for (int i = k + 1; i < n; ++i) {
      const double f = A[static_cast<size_t>(i) * n + k] / d;
      if (f == 0.0) continue;
      for (int j = k + 1; j < n; ++j) A[static_cast<size_t>(i) * n + j] -= f * A[static_cast<size_t>(k) * n + j];
      b[i] -= f * b[k];
    }
  }
  for (int i = n - 1; i >= 0; --i) {
    double t = b[i];
    for (int j = i + 1; j < n; ++j) t -= A[static_cast<size_t>(i) * n + j] * b[j];
    b[i] = t / A[static_cast<size_t>(i) * n + i];
    if (!std::isfinite(b[i])) return false;
  }
  return true;
}

namespace {

struct KKTState {
  int p, m;
  std::vector<double> B, b0;            // grad f = B y - b0, B = 2 R'R, b0 = 2 R' g
  std::vector<std::vector<double>> S;   // T + T'
  std::vector<double> tau;              // target offsets (c_i(y) = -tau_i)

  void residual(const QuadCon* cons, const double* y, const double* lam, double* F,
                std::vector<double>& J) const {
    // J (m x p row-major); F = [grad f + J' lam ; c + tau]
    for (int i = 0; i < m; ++i) {
      const std::vector<double>& Si = S[i];
      for (int a = 0; a < p; ++a) {
        double t = cons[i].term1[a];
        for (int b = 0; b < p; ++b) t += Si[static_cast<size_t>(a) * p + b] * y[b];
        J[static_cast<size_t>(i) * p + a] = t;
      }
    }
    for (int a = 0; a < p; ++a) {
      double t = -b0[a];
      for (int b = 0; b < p; ++b) t += B[static_cast<size_t>(a) * p + b] * y[b];
      for (int i = 0; i < m; ++i) t += J[static_cast<size_t>(i) * p + a] * lam[i];
      F[a] = t;
    }
    for (int i = 0; i < m; ++i) F[p + i] = con_value(cons[i], p, y) + tau[i];
  }
};

double norm2(const double* v, int n) {
  double s = 0.0;
  for (int i = 0; i < n; ++i) s += v[i] * v[i];
  return std::sqrt(s);
}

}  // namespace

KKTResult kkt_newton(int p, const double* R, int ld, const double* g, int m, const QuadCon* cons,
                     const double* y0, double* y, int max_iter) {
  KKTResult res;
  for (int a = 0; a < p; ++a) y[a] = y0[a];
  if (m > p) {  // SLSQP exit mode 2 leaves x at the initial guess
    res.message = SPIS_MSG_MORE_EQ;
    return res;
  }
  KKTState st;
  st.p = p;
  st.m = m;
  st.B.assign(static_cast<size_t>(p) * p, 0.0);
  st.b0.assign(p, 0.0);
  for (int a = 0; a < p; ++a) {
    for (int b = 0; b < p; ++b) {
      double t = 0.0;
      const int top = std::min(a, b);
      for (int k = 0; k <= top; ++k) t += R[static_cast<size_t>(a) * ld + k] * R[static_cast<size_t>(b) * ld + k];
      st.B[static_cast<size_t>(a) * p + b] = 2.0 * t;
    }
    double t = 0.0;
    for (int k = 0; k <= a; ++k) t += R[static_cast<size_t>(a) * ld + k] * g[k];
    st.b0[a] = 2.0 * t;
  }
  st.S.resize(m);
  for (int i = 0; i < m; ++i) {
    st.S[i].assign(static_cast<size_t>(p) * p, 0.0);
    for (int a = 0; a < p; ++a)
      for (int b = 0; b < p; ++b)
        st.S[i][static_cast<size_t>(a) * p + b] =
            cons[i].term2[static_cast<size_t>(a) * p + b] + cons[i].term2[static_cast<size_t>(b) * p + a];
  }
  st.tau.assign(m, 0.0);

  const int n = p + m;
  std::vector<double> lam(m, 0.0), J(static_cast<size_t>(m) * p), F(n), Fn(n), K, rhs(n), yn(p),
      ln(m);
  // least-squares multipliers at y0: (J J') lam = -J grad f
  st.residual(cons, y, lam.data(), F.data(), J);
  if (m > 0) {
    std::vector<double> JJ(static_cast<size_t>(m) * m);
    std::vector<double> r(m);
    for (int i = 0; i < m; ++i) {
      for (int k = 0; k < m; ++k) {
        double t = 0.0;
        for (int a = 0; a < p; ++a) t += J[static_cast<size_t>(i) * p + a] * J[static_cast<size_t>(k) * p + a];
        JJ[static_cast<size_t>(i) * m + k] = t;
      }
      double t = 0.0;
      for (int a = 0; a < p; ++a) t += J[static_cast<size_t>(i) * p + a] * F[a];
      r[i] = -t;
    }
    if (lu_solve(m, JJ, r.data()))
      for (int i = 0; i < m; ++i) lam[i] = r[i];
  }
  bool converged = false;
  int it = 0;
  for (; it < max_iter; ++it) {
    // offsets: a few ulps of each constraint's rounding scale, so that the COMPUTED value
    // lands <= 0 (the reference's checker is a signed max against ctol, solvers.py:14-18,267)
    for (int i = 0; i < m; ++i) st.tau[i] = 8.0 * DBL_EPSILON * con_scale(cons[i], p, y);
    st.residual(cons, y, lam.data(), F.data(), J);
    const double fn = norm2(F.data(), n);
    if (!std::isfinite(fn)) { res.finite = false; break; }
    {  // converged at the rounding floor: the gradient part of F within 64 ulps of its terms'
       // scale and every constraint at its target (c_i in [-2 tau_i, 0]).  Newton steps from
       // here are noise; the line search would backtrack ~30 times per step (~60 us at p = 30)
      double gs = 0.0, gn = 0.0;
      for (int a = 0; a < p; ++a) {
        double t = std::fabs(st.b0[a]);
        for (int b = 0; b < p; ++b) t += std::fabs(st.B[static_cast<size_t>(a) * p + b] * y[b]);
        for (int i = 0; i < m; ++i) t += std::fabs(J[static_cast<size_t>(i) * p + a] * lam[i]);
        gs = std::max(gs, t);
        gn = std::max(gn, std::fabs(F[a]));
      }
      bool cons_ok = true;
      for (int i = 0; i < m; ++i) cons_ok = cons_ok && std::fabs(F[p + i]) <= st.tau[i];
      if (cons_ok && gn <= 64.0 * DBL_EPSILON * gs) {
        converged = true;
        break;
      }
    }
    K.assign(static_cast<size_t>(n) * n, 0.0);
    for (int a = 0; a < p; ++a)
      for (int b = 0; b < p; ++b) {
        double w = st.B[static_cast<size_t>(a) * p + b];
        for (int i = 0; i < m; ++i) w += lam[i] * st.S[i][static_cast<size_t>(a) * p + b];
        K[static_cast<size_t>(a) * n + b] = w;
      }
    for (int i = 0; i < m; ++i)
      for (int a = 0; a < p; ++a) {
        K[static_cast<size_t>(a) * n + p + i] = J[static_cast<size_t>(i) * p + a];
        K[static_cast<size_t>(p + i) * n + a] = J[static_cast<size_t>(i) * p + a];
      }
    for (int r = 0; r < n; ++r) rhs[r] = -F[r];
    if (!lu_solve(n, K, rhs.data())) { res.message = SPIS_MSG_SINGULAR_C; break; }
    {  // a Newton step below the stopping size: take it unless it raises ||F||, and stop (no
       // backtracking: at roundoff level the sufficient-decrease test cannot pass and would cost
       // 40 residual evaluations)
      double step = 0.0, ymax = 0.0;
      for (int a = 0; a < p; ++a) {
        step = std::max(step, std::fabs(rhs[a]));
        ymax = std::max(ymax, std::fabs(y[a] + rhs[a]));
      }
      if (step <= 4.0 * DBL_EPSILON * (1.0 + ymax)) {
        for (int a = 0; a < p; ++a) yn[a] = y[a] + rhs[a];
        for (int i = 0; i < m; ++i) ln[i] = lam[i] + rhs[p + i];
        st.residual(cons, yn.data(), ln.data(), Fn.data(), J);
        const double fnew = norm2(Fn.data(), n);
        if (std::isfinite(fnew) && fnew <= fn)
          for (int a = 0; a < p; ++a) y[a] = yn[a];
        converged = true;
        ++it;
        break;
      }
    }
    double alpha = 1.0;
    double fnew = 0.0;
    // <= 10 halvings: once the Newton residual sits at its rounding floor (||grad f|| ~ eps ||B|| ||y||)
    // the direction is noise, and a step of alpha < 1e-3 only moves y by roundoff (40 halvings cost
    // ~60 us per constrained step at p = 30)
    for (int ls = 0; ls < 40; ++ls) {
      for (int a = 0; a < p; ++a) yn[a] = y[a] + alpha * rhs[a];
      for (int i = 0; i < m; ++i) ln[i] = lam[i] + alpha * rhs[p + i];
      st.residual(cons, yn.data(), ln.data(), Fn.data(), J);
      fnew = norm2(Fn.data(), n);
      if (std::isfinite(fnew) && fnew <= (1.0 - 1e-4 * alpha) * fn) break;
      alpha *= 0.5;
    }
    double step = 0.0, ymax = 0.0;
    for (int a = 0; a < p; ++a) {
      step = std::max(step, std::fabs(yn[a] - y[a]));
      ymax = std::max(ymax, std::fabs(yn[a]));
    }
    if (std::isfinite(fnew) && fnew <= fn) {
      for (int a = 0; a < p; ++a) y[a] = yn[a];
      for (int i = 0; i < m; ++i) lam[i] = ln[i];
    }
    if (step <= 4.0 * DBL_EPSILON * (1.0 + ymax) || !(fnew < fn)) {
      converged = true;
      ++it;
      break;
    }
  }
  res.iterations = it;
  for (int a = 0; a < p; ++a)
    if (!std::isfinite(y[a])) res.finite = false;
  if (res.message == 0 && !converged) res.message = SPIS_MSG_ITER_LIMIT;
  return res;
}

}  // namespace spis
