// ilu_capi.cpp — host-only C entry point over ilu_plan.cpp, built into liblsq_host.so so that the
// device ILU plan (levels, blocks, index maps) is checked on CPU without a GPU: the launch is
// emulated in ticket order.  Not part of the product ABI; the same ilu_plan.cpp is in libspis.so.
#include <cstring>
#include <string>

#include "ilu_plan.h"

using namespace spis;

extern "C" {

// stats[8] = {levels L, levels U, blocks L, blocks U, steps L, steps U, far steps L, far steps U}; 0 = success
int ilu_plan_emulate(int64_t n, const int32_t* l_rowptr, const int32_t* l_col, const double* l_val,
                     const int32_t* u_rowptr, const int32_t* u_col, const double* u_val, const int32_t* perm_r,
                     const int32_t* perm_c, const double* q, double* z, int64_t* stats, char* errbuf, int errlen) {
  TriPlan L, U;
  std::string err;
  bool ok = build_ilu_plans(n, l_rowptr, l_col, l_val, u_rowptr, u_col, u_val, perm_r, perm_c, &L, &U, &err);
  if (ok) {
    stats[0] = L.levels;
    stats[1] = U.levels;
    stats[2] = L.n_blocks();
    stats[3] = U.n_blocks();
    stats[4] = static_cast<int64_t>(L.step_row.size()) - 1;
    stats[5] = static_cast<int64_t>(U.step_row.size()) - 1;
    if (q && z) ok = emulate_ilu_apply(L, U, q, z, &err, stats + 6);
  }
  if (!ok && errbuf && errlen > 0) {
    std::strncpy(errbuf, err.c_str(), errlen - 1);
    errbuf[errlen - 1] = 0;
  }
  return ok ? 0 : 1;
}

}  // extern "C"
