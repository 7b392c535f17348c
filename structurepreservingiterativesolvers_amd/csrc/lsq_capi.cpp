// lsq_capi.cpp — host-only C entry points over lsq.cpp, built into liblsq_host.so so that the
// small least-squares math (Givens QR, Newton-KKT) is unit-tested on CPU without a GPU.
// Not part of the product ABI (include/spis.h); the same lsq.cpp is linked into libspis.so.
#include <cstddef>
#include <vector>

#include "lsq.h"

using namespace spis;

extern "C" {

// y = argmin ||beta e1 - H y||, H (p+1) x p column-major
int lsq_givens_solve(int p, const double* H, double beta, double* y) {
  GivensQR qr;
  qr.reset(p, beta);
  std::vector<double> col(p + 1);
  for (int j = 0; j < p; ++j) {
    for (int i = 0; i <= j + 1; ++i) col[i] = H[static_cast<size_t>(j) * (p + 1) + i];
    qr.add_column(j, col.data());
  }
  qr.solve(p, y);
  return 0;
}

// constrained: m constraints, term0[m], term1[m*p], term2[m*p*p] (row-major per constraint)
int lsq_kkt_solve(int p, const double* H, double beta, int m, const double* term0, const double* term1,
                  const double* term2, const double* y0, double* y, int* message, int* iterations) {
  GivensQR qr;
  qr.reset(p, beta);
  std::vector<double> col(p + 1);
  for (int j = 0; j < p; ++j) {
    for (int i = 0; i <= j + 1; ++i) col[i] = H[static_cast<size_t>(j) * (p + 1) + i];
    qr.add_column(j, col.data());
  }
  std::vector<QuadCon> cons(m);
  for (int i = 0; i < m; ++i) {
    cons[i].term0 = term0[i];
    cons[i].term1.assign(term1 + static_cast<size_t>(i) * p, term1 + static_cast<size_t>(i + 1) * p);
    cons[i].term2.assign(term2 + static_cast<size_t>(i) * p * p, term2 + static_cast<size_t>(i + 1) * p * p);
  }
  KKTResult r = kkt_newton(p, qr.R(), qr.ld(), qr.g(), m, cons.data(), y0, y);
  *message = r.message;
  *iterations = r.iterations;
  return r.finite ? 0 : 1;
}

// the first start's initial multipliers of kkt_newton (lam0_out[m]); same arguments as lsq_kkt_solve
int lsq_kkt_init_multipliers(int p, const double* H, double beta, int m, const double* term0, const double* term1,
                             const double* term2, const double* y0, double* lam0_out) {
  GivensQR qr;
  qr.reset(p, beta);
  std::vector<double> col(p + 1);
  for (int j = 0; j < p; ++j) {
    for (int i = 0; i <= j + 1; ++i) col[i] = H[static_cast<size_t>(j) * (p + 1) + i];
    qr.add_column(j, col.data());
  }
  std::vector<QuadCon> cons(m);
  for (int i = 0; i < m; ++i) {
    cons[i].term0 = term0[i];
    cons[i].term1.assign(term1 + static_cast<size_t>(i) * p, term1 + static_cast<size_t>(i + 1) * p);
    cons[i].term2.assign(term2 + static_cast<size_t>(i) * p * p, term2 + static_cast<size_t>(i + 1) * p * p);
  }
  std::vector<double> y(p), lam0;
  (void)kkt_newton(p, qr.R(), qr.ld(), qr.g(), m, cons.data(), y0, y.data(), 100, &lam0);
  if (static_cast<int>(lam0.size()) != m) return 1;
  for (int i = 0; i < m; ++i) lam0_out[i] = lam0[i];
  return 0;
}

double lsq_con_value(int p, double term0, const double* term1, const double* term2, const double* y) {
  QuadCon c;
  c.term0 = term0;
  c.term1.assign(term1, term1 + p);
  c.term2.assign(term2, term2 + static_cast<size_t>(p) * p);
  return con_value(c, p, y);
}
}
