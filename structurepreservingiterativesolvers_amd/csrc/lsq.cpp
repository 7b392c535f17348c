// lsq.cpp — host-side small dense least squares (see lsq.h).
#include "lsq.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>

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

// Host-time note (round 5): the O(p^2) and O(p^3) sums below run with the loop over independent
// sums innermost (u[b] here, J[a] and F[a] in residual, ...): every sum keeps its own operand
// order, so results are bitwise those of the row-by-row loops, without one dependent add chain
// per entry (C3's KKT solve, p = 30, m = 2: the GPU waits on it).
double con_value(const QuadCon& c, int p, const double* y) {
  double lin = 0.0;
  for (int a = 0; a < p; ++a) lin += c.term1[a] * y[a];
  double ub[128];
  std::vector<double> uv;
  double* u = ub;
  if (p > 128) {
    uv.assign(p, 0.0);
    u = uv.data();
  }
  for (int b = 0; b < p; ++b) u[b] = 0.0;
  const double* T = c.term2.data();
  for (int a = 0; a < p; ++a) {  // u[b] = sum_a y[a] T[a][b], a ascending
    const double ya = y[a];
    const double* row = T + static_cast<size_t>(a) * p;
    for (int b = 0; b < p; ++b) u[b] += ya * row[b];
  }
  double quad = 0.0;
  for (int b = 0; b < p; ++b) quad += u[b] * y[b];
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
  // scaled constraints (kkt_newton): values are the unscaled constraint's, as the reference's
  // checker evaluates it, times 1 / scale, so their sign is exactly the checker's
  const QuadCon* orig = nullptr;
  std::vector<double> inv_s;
  const double* R = nullptr;  // upper triangular p x p, column-major, leading dimension ld
  const double* g = nullptr;
  int ld = 0;

  double cval(const QuadCon* cons, int i, const double* y) const {
    return orig ? con_value(orig[i], p, y) * inv_s[i] : con_value(cons[i], p, y);
  }

  // out[a] = init[a] + sum_b Sym[a][b] v[b], b ascending, for an exactly symmetric Sym (B, S_i:
  // entrywise sums of commuting products): summed down column a, the loop over a innermost
  void symv(const double* Sym, const double* init, const double* v, double* out) const {
    for (int a = 0; a < p; ++a) out[a] = init[a];
    for (int b = 0; b < p; ++b) {
      const double vb = v[b];
      const double* col = Sym + static_cast<size_t>(b) * p;
      for (int a = 0; a < p; ++a) out[a] += col[a] * vb;
    }
  }

  void residual(const QuadCon* cons, const double* y, const double* lam, double* F,
                std::vector<double>& J) const {
    // J (m x p row-major); F = [grad f + J' lam ; c + tau]
    for (int i = 0; i < m; ++i) symv(S[i].data(), cons[i].term1.data(), y, J.data() + static_cast<size_t>(i) * p);
    for (int a = 0; a < p; ++a) F[a] = -b0[a];
    for (int b = 0; b < p; ++b) {
      const double yb = y[b];
      const double* col = B.data() + static_cast<size_t>(b) * p;
      for (int a = 0; a < p; ++a) F[a] += col[a] * yb;
    }
    for (int i = 0; i < m; ++i) {
      const double li = lam[i];
      const double* Ji = J.data() + static_cast<size_t>(i) * p;
      for (int a = 0; a < p; ++a) F[a] += Ji[a] * li;
    }
    for (int i = 0; i < m; ++i) F[p + i] = cval(cons, i, y) + tau[i];
  }
};

double norm2(const double* v, int n) {
  double s = 0.0;
  for (int i = 0; i < n; ++i) s += v[i] * v[i];
  return std::sqrt(s);
}

}  // namespace

namespace {

// Outcome of one SQP run on the KKT system.
enum class Stop { kFloor, kSmallStep, kStall, kIterLimit, kSingular, kNonFinite };

struct Run {
  Stop stop = Stop::kIterLimit;
  int iterations = 0;
  double fn = 0.0;  // ||F|| at the returned point
};

// ||grad_y L|| and the magnitude of its terms at (y, lam); J must hold the Jacobian at y
void grad_scale(const KKTState& st, const double* y, const double* lam, const double* F,
                const std::vector<double>& J, double* gn, double* gs) {
  const int p = st.p, m = st.m;
  *gn = 0.0;
  *gs = 0.0;
  std::vector<double> t(p);
  for (int a = 0; a < p; ++a) t[a] = std::fabs(st.b0[a]);
  for (int b = 0; b < p; ++b) {  // B exactly symmetric: row a summed down column a
    const double yb = y[b];
    const double* col = st.B.data() + static_cast<size_t>(b) * p;
    for (int a = 0; a < p; ++a) t[a] += std::fabs(col[a] * yb);
  }
  for (int i = 0; i < m; ++i)
    for (int a = 0; a < p; ++a) t[a] += std::fabs(J[static_cast<size_t>(i) * p + a] * lam[i]);
  for (int a = 0; a < p; ++a) {
    *gs = std::max(*gs, t[a]);
    *gn = std::max(*gn, std::fabs(F[a]));
  }
}

// Positive definiteness of the reduced Hessian N'(W + delta I)N on the null space of the m x p
// Jacobian (Jt: p x m, column i = grad c_i; both copied, they are transformed in place): the
// Householder reflections of a QR of J' are applied to W from both sides (Q' W Q, 4 p^2 flops each;
// the explicit null-space basis and the products N'(W N) would cost 2 p^3), whose trailing
// (p - m) block is the reduced Hessian; Cholesky with a shift of shift_rel times its largest
// diagonal entry.
bool reduced_pd(const std::vector<double>& W_in, const std::vector<double>& Jt_in, int p, int m, double delta,
                double shift_rel) {
  if (m >= p) return true;
  // (scratch reused per thread; every sum below keeps the operand order of the row-by-row form)
  thread_local std::vector<double> W, Jt, v, u, tw, Lc, tr;
  W.assign(W_in.begin(), W_in.end());
  Jt.assign(Jt_in.begin(), Jt_in.end());
  v.assign(p, 0.0);
  u.assign(p, 0.0);
  tw.assign(p, 0.0);
  for (int a = 0; a < p; ++a) W[static_cast<size_t>(a) * p + a] += delta;
  for (int i = 0; i < m; ++i) {
    double* col = Jt.data() + static_cast<size_t>(i) * p;
    double nrm = 0.0;
    for (int a = i; a < p; ++a) nrm += col[a] * col[a];
    nrm = std::sqrt(nrm);
    if (nrm == 0.0) continue;
    const double alpha = col[i] > 0 ? -nrm : nrm;
    std::fill(v.begin(), v.end(), 0.0);
    for (int a = i; a < p; ++a) v[a] = col[a];
    v[i] -= alpha;
    double vv = 0.0;
    for (int a = i; a < p; ++a) vv += v[a] * v[a];
    if (vv == 0.0) continue;
    const double s2 = 2.0 / vv;
    for (int k = i; k < m; ++k) {  // the remaining columns of J'
      double* x = Jt.data() + static_cast<size_t>(k) * p;
      double t = 0.0;
      for (int a = i; a < p; ++a) t += v[a] * x[a];
      t *= s2;
      for (int a = i; a < p; ++a) x[a] -= t * v[a];
    }
    // W <- H W H with H = I - s2 v v' (W symmetric up to rounding: both sides explicitly)
    // W <- W H: row a -= s2 (W_a . v) v', each row's sum over b ascending (four rows side by side)
    int a = 0;
    for (; a + 3 < p; a += 4) {
      const double* r0 = W.data() + static_cast<size_t>(a) * p;
      const double* r1 = r0 + p;
      const double* r2 = r1 + p;
      const double* r3 = r2 + p;
      double t0 = 0.0, t1 = 0.0, t2 = 0.0, t3 = 0.0;
      for (int b = i; b < p; ++b) {
        const double vb = v[b];
        t0 += r0[b] * vb;
        t1 += r1[b] * vb;
        t2 += r2[b] * vb;
        t3 += r3[b] * vb;
      }
      tw[a] = t0;
      tw[a + 1] = t1;
      tw[a + 2] = t2;
      tw[a + 3] = t3;
    }
    for (; a < p; ++a) {
      const double* r0 = W.data() + static_cast<size_t>(a) * p;
      double t0 = 0.0;
      for (int b = i; b < p; ++b) t0 += r0[b] * v[b];
      tw[a] = t0;
    }
    for (int a2 = 0; a2 < p; ++a2) {
      double* row = W.data() + static_cast<size_t>(a2) * p;
      const double t = tw[a2] * s2;
      for (int b = i; b < p; ++b) row[b] -= t * v[b];
    }
    std::fill(u.begin(), u.end(), 0.0);  // W <- H W: W -= s2 v (v' W)
    for (int a2 = i; a2 < p; ++a2) {
      const double va = v[a2];
      const double* row = W.data() + static_cast<size_t>(a2) * p;
      for (int b = 0; b < p; ++b) u[b] += va * row[b];
    }
    for (int a2 = i; a2 < p; ++a2) {
      double* row = W.data() + static_cast<size_t>(a2) * p;
      const double f = s2 * v[a2];
      for (int b = 0; b < p; ++b) row[b] -= f * u[b];
    }
  }
  // Cholesky of the trailing (p - m) block with a shift of shift_rel times its largest diagonal
  // entry, in place, column-major (Lc[c][r] = entry (r, c)): each column's update runs down a
  // contiguous column, every entry's sum over k ascending as in the row-major form
  const int nz = p - m;
  Lc.resize(static_cast<size_t>(nz) * nz);
  tr.resize(nz);
  double dmax = 0.0;
  for (int c = 0; c < nz; ++c) {
    double* lc = Lc.data() + static_cast<size_t>(c) * nz;
    for (int r = 0; r < nz; ++r) lc[r] = W[static_cast<size_t>(m + r) * p + m + c];
    dmax = std::max(dmax, std::fabs(lc[c]));
  }
  const double shift = shift_rel * dmax;
  for (int c = 0; c < nz; ++c) {
    double* lc = Lc.data() + static_cast<size_t>(c) * nz;
    double d = lc[c] + shift;
    for (int k = 0; k < c; ++k) {
      const double ck = Lc[static_cast<size_t>(k) * nz + c];
      d -= ck * ck;
    }
    if (!(d > 0.0)) return false;
    d = std::sqrt(d);
    lc[c] = d;
    for (int r = c + 1; r < nz; ++r) tr[r] = lc[r];
    for (int k = 0; k < c; ++k) {
      const double* lk = Lc.data() + static_cast<size_t>(k) * nz;
      const double ck = lk[c];
      for (int r = c + 1; r < nz; ++r) tr[r] -= lk[r] * ck;
    }
    for (int r = c + 1; r < nz; ++r) lc[r] = tr[r] / d;
  }
  return true;
}

// Hessian of the Lagrangian B + sum lam_i S_i (p x p) and J' (p x m) at (y, lam); J (m x p) given
void lagrangian_hessian(const KKTState& st, const double* lam, const std::vector<double>& J, std::vector<double>& W,
                        std::vector<double>& Jt) {
  const int p = st.p, m = st.m;
  W.assign(st.B.begin(), st.B.end());  // each entry B + lam_0 S_0 + lam_1 S_1 ..., i ascending
  Jt.resize(static_cast<size_t>(p) * m);
  for (int i = 0; i < m; ++i) {
    const double li = lam[i];
    const double* Si = st.S[i].data();
    for (size_t ab = 0; ab < static_cast<size_t>(p) * p; ++ab) W[ab] += li * Si[ab];
  }
  for (int i = 0; i < m; ++i)
    for (int a = 0; a < p; ++a) Jt[static_cast<size_t>(i) * p + a] = J[static_cast<size_t>(i) * p + a];
}

// SQP on the KKT system from (y, lam), both updated in place.  Each iteration solves
//   [W + delta I  J'] [d    ]   [-grad f    ]
//   [J            0 ] [lam+ ] = [-(c + tau) ]
// with W the Lagrangian Hessian and delta >= 0 the smallest shift (0, then 1e-12 .. 1e2 of W's
// scale) that makes the reduced Hessian positive definite: with delta = 0 this is Newton's step
// on the KKT conditions (quadratic convergence at a constrained minimum); with delta > 0 the
// step descends the exact L1 merit f + mu sum |c_i + tau_i| (mu > max |lam+|, SLSQP's merit),
// so a run is not attracted by constrained saddles and maxima of the indefinite energy
// constraint, as Newton on ||F|| is (C5 restart cycle 8: ||F|| Newton from the warm start
// converged to a saddle at f = 2.3e-2 where SLSQP finds the minimum, f = 7.0e-3).  Steps are
// accepted on the merit, or, in the locally convex regime (delta = 0), on a decrease of ||F||
// (the merit can reject full Newton steps near a solution: Maratos).  The constraints are
// scaled to unit gradient at the start (kkt_newton), so mu is not set by a degenerate row.
Run sqp_run(KKTState& st, const QuadCon* cons, double* y, std::vector<double>& lam, int max_iter) {
  const int p = st.p, m = st.m, n = p + m;
  std::vector<double> J(static_cast<size_t>(m) * p), F(n), Fn(n), K, rhs(n), yn(p), ln(m), W, Jt, gf(p);
  Run run;
  double mu = 0.0;
  double bscale = 0.0;
  for (int a = 0; a < p; ++a) bscale = std::max(bscale, std::fabs(st.B[static_cast<size_t>(a) * p + a]));
  if (!(bscale > 0.0)) bscale = 1.0;
  // f - rho^2 = ||g - R v||^2 from the residual itself (1/2 v'Bv - b0'v cancels to roundoff of
  // |b0| |v| near a solution whose f is ~1e-21, so merit comparisons would be noise)
  std::vector<double> fr(p);
  auto fval = [&](const double* v) {  // r[a] = g[a] - sum_{b >= a} R[a][b] v[b], b ascending
    for (int a = 0; a < p; ++a) fr[a] = st.g[a];
    for (int b = 0; b < p; ++b) {
      const double vb = v[b];
      const double* col = st.R + static_cast<size_t>(b) * st.ld;
      for (int a = 0; a <= b; ++a) fr[a] -= col[a] * vb;
    }
    double t = 0.0;
    for (int a = 0; a < p; ++a) t += fr[a] * fr[a];
    return t;
  };
  int it = 0;
  for (; it < max_iter; ++it) {
    // offsets: a few ulps of each constraint's rounding scale, so that the COMPUTED value
    // lands <= 0 (the reference's checker is a signed max against ctol, solvers.py:14-18,267)
    for (int i = 0; i < m; ++i) st.tau[i] = 8.0 * DBL_EPSILON * con_scale(cons[i], p, y);
    st.residual(cons, y, lam.data(), F.data(), J);
    const double fn = norm2(F.data(), n);
    run.fn = fn;
    if (!std::isfinite(fn)) { run.stop = Stop::kNonFinite; break; }
    {  // converged at the rounding floor: the gradient part of F within 64 ulps of its terms'
       // scale and every constraint at its target (c_i in [-2 tau_i, 0]).  Steps from here are
       // noise; the line search would backtrack ~30 times per step (~60 us at p = 30)
      double gn, gs;
      grad_scale(st, y, lam.data(), F.data(), J, &gn, &gs);
      bool cons_ok = true;
      for (int i = 0; i < m; ++i) cons_ok = cons_ok && std::fabs(F[p + i]) <= st.tau[i];
      if (cons_ok && gn <= 64.0 * DBL_EPSILON * gs) { run.stop = Stop::kFloor; break; }
    }
    for (int a = 0; a < p; ++a) gf[a] = -st.b0[a];
    st.symv(st.B.data(), gf.data(), y, gf.data());
    lagrangian_hessian(st, lam.data(), J, W, Jt);
    double delta = 0.0;
    bool pd = reduced_pd(W, Jt, p, m, 0.0, 0.0);
    for (int e = -12; !pd && e <= 2; e += 2) {
      delta = bscale * std::pow(10.0, e);
      pd = reduced_pd(W, Jt, p, m, delta, 0.0);
    }
    if (!pd) { run.stop = Stop::kSingular; break; }
    K.assign(static_cast<size_t>(n) * n, 0.0);
    for (int a = 0; a < p; ++a) {
      for (int b = 0; b < p; ++b) K[static_cast<size_t>(a) * n + b] = W[static_cast<size_t>(a) * p + b];
      K[static_cast<size_t>(a) * n + a] += delta;
    }
    for (int i = 0; i < m; ++i)
      for (int a = 0; a < p; ++a) {
        K[static_cast<size_t>(a) * n + p + i] = J[static_cast<size_t>(i) * p + a];
        K[static_cast<size_t>(p + i) * n + a] = J[static_cast<size_t>(i) * p + a];
      }
    for (int a = 0; a < p; ++a) rhs[a] = -gf[a];
    for (int i = 0; i < m; ++i) rhs[p + i] = -F[p + i];
    if (!lu_solve(n, K, rhs.data())) { run.stop = Stop::kSingular; break; }
    const double* d = rhs.data();
    const double* lp = rhs.data() + p;
    {  // a step below the stopping size: take it unless it raises ||F||, and stop (no
       // backtracking: at roundoff level no sufficient-decrease test can pass)
      double step = 0.0, ymax = 0.0;
      for (int a = 0; a < p; ++a) {
        step = std::max(step, std::fabs(d[a]));
        ymax = std::max(ymax, std::fabs(y[a] + d[a]));
      }
      if (step <= 4.0 * DBL_EPSILON * (1.0 + ymax)) {
        for (int a = 0; a < p; ++a) yn[a] = y[a] + d[a];
        for (int i = 0; i < m; ++i) ln[i] = lp[i];
        st.residual(cons, yn.data(), ln.data(), Fn.data(), J);
        const double fnew = norm2(Fn.data(), n);
        if (std::isfinite(fnew) && fnew <= fn) {
          for (int a = 0; a < p; ++a) y[a] = yn[a];
          for (int i = 0; i < m; ++i) lam[i] = ln[i];
          run.fn = fnew;
        }
        run.stop = Stop::kSmallStep;
        ++it;
        break;
      }
    }
    double lmax = 0.0;
    for (int i = 0; i < m; ++i) lmax = std::max(lmax, std::fabs(lp[i]));
    mu = std::max(mu, 2.0 * lmax);
    double v0 = 0.0;  // viol(y): F holds c_i(y) + tau_i (the residual at y, the same tau)
    for (int i = 0; i < m; ++i) v0 += std::fabs(F[p + i]);
    const double phi0 = fval(y) + mu * v0;
    double dd = 0.0;  // directional derivative of the merit along d (J d = -(c + tau))
    for (int a = 0; a < p; ++a) dd += gf[a] * d[a];
    dd -= mu * v0;
    double alpha = 1.0, fnew = 0.0;
    bool ok = false;
    for (int ls = 0; ls < 40; ++ls) {
      for (int a = 0; a < p; ++a) yn[a] = y[a] + alpha * d[a];
      for (int i = 0; i < m; ++i) ln[i] = lam[i] + alpha * (lp[i] - lam[i]);
      st.residual(cons, yn.data(), ln.data(), Fn.data(), J);
      fnew = norm2(Fn.data(), n);
      if (std::isfinite(fnew)) {
        double vn = 0.0;  // viol(yn) from Fn (c_i(yn) + tau_i)
        for (int i = 0; i < m; ++i) vn += std::fabs(Fn[p + i]);
        const double phin = fval(yn.data()) + mu * vn;
        if ((dd < 0.0 && phin <= phi0 + 1e-4 * alpha * dd) || (delta == 0.0 && fnew <= (1.0 - 1e-4 * alpha) * fn)) {
          ok = true;
          break;
        }
      }
      alpha *= 0.5;
    }
    if (!ok) { run.stop = Stop::kStall; ++it; break; }
    double step = 0.0, ymax = 0.0;
    for (int a = 0; a < p; ++a) {
      step = std::max(step, std::fabs(yn[a] - y[a]));
      ymax = std::max(ymax, std::fabs(yn[a]));
      y[a] = yn[a];
    }
    for (int i = 0; i < m; ++i) lam[i] = ln[i];
    run.fn = fnew;
    if (step <= 4.0 * DBL_EPSILON * (1.0 + ymax)) { run.stop = Stop::kSmallStep; ++it; break; }
  }
  run.iterations = it;
#ifdef SPIS_KKT_DEBUG
  fprintf(stderr, "  sqp_run: stop=%d it=%d fn=%.3e mu=%.3e lam=", static_cast<int>(run.stop), it, run.fn, mu);
  for (int i = 0; i < m; ++i) fprintf(stderr, "%.3e ", lam[i]);
  fprintf(stderr, "\n");
#endif
  return run;
}

// First-order test at the returned point, looser than the rounding floor (a run that stops on
// a small step or a stalled line search has not necessarily converged): gradient of the
// Lagrangian within 1e-8 of its terms' scale and every constraint within 1e-10 of its own
// rounding scale.  The multipliers are refit by least squares first (the run's lam may lag).
bool first_order_ok(KKTState& st, const QuadCon* cons, const double* y, std::vector<double>& lam) {
  const int p = st.p, m = st.m;
  std::vector<double> J(static_cast<size_t>(m) * p), F(p + m), zero(m, 0.0);
  st.residual(cons, y, zero.data(), F.data(), J);
  if (m > 0) {
    std::vector<double> JJ(static_cast<size_t>(m) * m), r(m);
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
    // a rank-deficient J (a constraint whose gradient is roundoff, e.g. a conserved quantity the
    // Krylov space cannot change) keeps the run's multipliers
    if (lu_solve(m, JJ, r.data())) {
      std::vector<double> lam_fit(r.begin(), r.end());
      std::vector<double> Ft(p + m);
      st.residual(cons, y, lam_fit.data(), Ft.data(), J);
      std::vector<double> Fr(p + m);
      st.residual(cons, y, lam.data(), Fr.data(), J);
      if (norm2(Ft.data(), p) < norm2(Fr.data(), p)) lam = lam_fit;
    }
  }
  st.residual(cons, y, lam.data(), F.data(), J);
  double gn, gs;
  grad_scale(st, y, lam.data(), F.data(), J, &gn, &gs);
  if (!(gn <= 1e-8 * gs)) return false;
  for (int i = 0; i < m; ++i) {
    const double sc = con_scale(cons[i], p, y);
    if (!(std::fabs(F[p + i]) <= 1e-10 * sc + 1e-300)) return false;
  }
  return true;
}

// Second-order test: the Hessian of the Lagrangian, B + sum lam_i S_i, positive definite on the
// null space of J (a constrained minimum, not a saddle of the indefinite energy constraint);
// Cholesky with a shift of 1e-10 of its largest diagonal entry, so a semidefinite direction at
// roundoff passes.
bool second_order_ok(const KKTState& st, const QuadCon* cons, const double* y, const std::vector<double>& lam) {
  const int p = st.p, m = st.m;
  if (m >= p) return true;
  std::vector<double> J(static_cast<size_t>(m) * p), F(p + m), W, Jt;
  st.residual(cons, y, lam.data(), F.data(), J);
  lagrangian_hessian(st, lam.data(), J, W, Jt);
  return reduced_pd(W, Jt, p, m, 0.0, 1e-10);
}

}  // namespace

KKTResult kkt_newton(int p, const double* R, int ld, const double* g, int m, const QuadCon* cons,
                     const double* y0, double* y, int max_iter, std::vector<double>* lam0) {
  KKTResult res;
  for (int a = 0; a < p; ++a) y[a] = y0[a];
  if (m > p) {  // SLSQP exit mode 2 leaves x at the initial guess
    res.message = SPIS_MSG_MORE_EQ;
    return res;
  }
  KKTState st;
  st.p = p;
  st.m = m;
  st.R = R;
  st.g = g;
  st.ld = ld;
  // B[a][b] = 2 sum_{k <= min(a, b)} R[k][a] R[k][b], k ascending: rank-one updates by row k of
  // R (the same sums, formed side by side; R column-major: R[k][a] = R[a * ld + k])
  st.B.assign(static_cast<size_t>(p) * p, 0.0);
  st.b0.assign(p, 0.0);
  {
    std::vector<double> rk(p);
    for (int k = 0; k < p; ++k) {
      for (int b = k; b < p; ++b) rk[b] = R[static_cast<size_t>(b) * ld + k];
      for (int a = k; a < p; ++a) {
        const double ra = rk[a];
        double* row = st.B.data() + static_cast<size_t>(a) * p;
        for (int b = k; b < p; ++b) row[b] += ra * rk[b];
      }
    }
    for (double& t : st.B) t *= 2.0;
  }
  for (int a = 0; a < p; ++a) {
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

  // least-squares multipliers at a start point: (J J') lam = -J grad f, with the constraints the
  // SQP runs on (cc: scaled to unit gradient at y0, as st.S is by then)
  auto init_lam = [&](const QuadCon* cc, const double* ys, std::vector<double>& lam) {
    lam.assign(m, 0.0);
    if (m == 0) return;
    std::vector<double> J(static_cast<size_t>(m) * p), F(p + m), JJ(static_cast<size_t>(m) * m), r(m);
    st.residual(cc, ys, lam.data(), F.data(), J);
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
  };
  // 0) SLSQP's first LSQ subproblem (LSEI) triangularises the constraint Jacobian at y0 by
  //    Householder reflections and stops with "Singular matrix C in LSQ subproblem" (mode 6,
  //    x = y0) when a diagonal element falls below machine epsilon (absolute, unscaled).  A
  //    constraint whose gradient is pure roundoff (swe/lkdvRK mass with a massless Krylov space,
  //    |grad| ~ 1e-18) is infeasible for Newton as well: without this test both starts run to the
  //    iteration limit (C4: 13.6 ms host time, then the same fallback as the reference's).
  if (m > 0) {
    std::vector<double> Jc(static_cast<size_t>(m) * p);
    for (int i = 0; i < m; ++i) st.symv(st.S[i].data(), cons[i].term1.data(), y, Jc.data() + static_cast<size_t>(i) * p);
    for (int i = 0; i < m; ++i) {  // Householder QR of the rows (J' columns), pivot by pivot
      double* ri = Jc.data() + static_cast<size_t>(i) * p;
      double nrm = 0.0;
      for (int a = i; a < p; ++a) nrm += ri[a] * ri[a];
      nrm = std::sqrt(nrm);
      if (!(nrm >= DBL_EPSILON)) {
        res.message = SPIS_MSG_SINGULAR_C;
        return res;  // y = y0
      }
      const double alpha = ri[i] > 0 ? -nrm : nrm;
      std::vector<double> v(ri, ri + p);
      for (int a = 0; a < i; ++a) v[a] = 0.0;
      v[i] -= alpha;
      double vv = 0.0;
      for (int a = i; a < p; ++a) vv += v[a] * v[a];
      if (vv == 0.0) continue;
      for (int k = i + 1; k < m; ++k) {
        double* rk = Jc.data() + static_cast<size_t>(k) * p;
        double t = 0.0;
        for (int a = i; a < p; ++a) t += v[a] * rk[a];
        t = 2.0 * t / vv;
        for (int a = i; a < p; ++a) rk[a] -= t * v[a];
      }
    }
  }

  // the constraints scaled to unit gradient at y0: an equality constraint's feasible set does not
  // depend on its scale, but the merit's penalty weight does (the swe mass constraint's gradient
  // is roundoff, |term1| ~ 1e-11, at a restart whose x0 already conserves mass: unscaled, its
  // multiplier is ~1e9 and sets mu).  The signed checker and the tau targets are relative, so
  // they carry over unchanged.
  std::vector<QuadCon> sc(cons, cons + m);
  st.orig = cons;
  st.inv_s.assign(m, 1.0);
  std::vector<double> gi(p);
  for (int i = 0; i < m; ++i) {
    st.symv(st.S[i].data(), cons[i].term1.data(), y0, gi.data());
    double nrm = 0.0;
    for (int a = 0; a < p; ++a) nrm += gi[a] * gi[a];
    nrm = std::sqrt(nrm);
    if (!(nrm > 0.0) || !std::isfinite(nrm)) continue;
    const double f = 1.0 / nrm;
    st.inv_s[i] = f;
    sc[i].term0 *= f;
    for (double& t : sc[i].term1) t *= f;
    for (double& t : sc[i].term2) t *= f;
    for (double& t : st.S[i]) t *= f;
  }
  const QuadCon* cs = sc.data();
  auto run_from = [&](double* ys, std::vector<double>& lam) {
    init_lam(cs, ys, lam);
    if (lam0 != nullptr && lam0->empty()) *lam0 = lam;  // the first start's (tests)
    return sqp_run(st, cs, ys, lam, max_iter);
  };
  auto accept_s = [&](const Run& run, const double* yr, std::vector<double>& lam) {
    if (run.stop == Stop::kSingular || run.stop == Stop::kNonFinite || run.stop == Stop::kIterLimit) return false;
    for (int a = 0; a < p; ++a)
      if (!std::isfinite(yr[a])) return false;
    if (run.stop != Stop::kFloor && !first_order_ok(st, cs, yr, lam)) return false;
    return second_order_ok(st, cs, yr, lam);
  };

  // starts, the first verified constrained minimum wins: 1) the reference's warm start y0
  // (solvers.py:225-227), as SLSQP; 2) the unconstrained minimiser (R y = g), the point SLSQP's
  // first QP step heads for; 3) y = 0, i.e. x0 itself (feasible at a restart whose x0 satisfies
  // the constraints)
  std::vector<std::vector<double>> ys(3, std::vector<double>(p, 0.0));
  for (int a = 0; a < p; ++a) ys[0][a] = y0[a];
  for (int i = p - 1; i >= 0; --i) {
    double t = g[i];
    for (int k = i + 1; k < p; ++k) t -= R[static_cast<size_t>(k) * ld + i] * ys[1][k];
    const double d = R[static_cast<size_t>(i) * ld + i];
    ys[1][i] = d != 0.0 ? t / d : 0.0;
  }
  bool y0_zero = true;
  for (int a = 0; a < p; ++a) y0_zero = y0_zero && y0[a] == 0.0;
  const int n_starts = y0_zero ? 2 : 3;
  std::vector<Run> runs;
  int best = -1;
  for (int sidx = 0; sidx < n_starts; ++sidx) {
    std::vector<double> lam;
    runs.push_back(run_from(ys[sidx].data(), lam));
    res.iterations += runs.back().iterations;
    if (accept_s(runs.back(), ys[sidx].data(), lam)) {
      for (int a = 0; a < p; ++a) y[a] = ys[sidx][a];
      return res;
    }
    bool fin = runs.back().stop != Stop::kNonFinite;
    for (int a = 0; a < p; ++a) fin = fin && std::isfinite(ys[sidx][a]);
    if (fin && (best < 0 || runs.back().fn < runs[best].fn)) best = sidx;
  }
  // no start reached a verified constrained minimum: report it (the caller warns, as the
  // reference does for a non-success SLSQP exit, :280-284) and keep the finite point with the
  // smallest KKT residual
  if (best >= 0) {
    for (int a = 0; a < p; ++a) y[a] = ys[best][a];
  } else {
    res.finite = false;
  }
  bool all_singular = true;
  for (const Run& r : runs) all_singular = all_singular && r.stop == Stop::kSingular;
  res.message = all_singular ? SPIS_MSG_SINGULAR_C : SPIS_MSG_ITER_LIMIT;
  return res;
}

}  // namespace spis
