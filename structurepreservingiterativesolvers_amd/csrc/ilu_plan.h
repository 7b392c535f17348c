// ilu_plan.h — host-side plan of the device ILU apply (K8, sptrsv.h): level sets, solve order,
// blocks and steps of one triangular factor.  Pure C++ (no HIP) so the CPU tests can check the
// plan, and a sequential emulation of the launch in ticket order, without a GPU.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace spis {

constexpr int kTriRows = 64;       // rows per step (one per lane)
constexpr int kTriBlockCap = 256;  // rows per block (the wave's LDS window)
constexpr int kTriBlockNnz = 2048; // entries per staged block (the wave's LDS copy of its rows)
constexpr unsigned long long kTriSentinel = 0xFFF7FFF7FFF7FFF7ull;  // a negative signalling NaN
constexpr int kLongRow = 512;      // a level with a longer row is solved a row per wave, from HBM
constexpr int kLongStep = 4;       // rows per step of such a level

struct TriPlan {
  int64_t n = 0;
  int32_t levels = 0;
  std::vector<int32_t> rowptr, col, in_idx, out_idx, blk_row, blk_step, step_row;
  std::vector<int32_t> step_long;  // [ns] 1: the step's rows are solved one per wave (lanes split the row)
  std::vector<int32_t> blk_ent;    // [nb+1] first entry of each block (rowptr at blk_row)
  std::vector<int32_t> blk_long;   // [nb] 1: a long-row block (not staged in LDS; one step)
  std::vector<int32_t> pos;  // original row -> position in solve order
  std::vector<double> val, diag;
  int32_t n_blocks() const { return static_cast<int32_t>(blk_row.size()) - 1; }
};

// L (upper=false): CSR of a unit lower-triangular factor; a stored diagonal must be 1 and is
//   dropped.  U (upper=true): CSR of an upper-triangular factor with a non-zero diagonal.
// in_map / out_map (may be null for out_map): in_idx[t] = in_map[row], out_idx[t] = out_map[row]
// for the row at position t.  Returns false with *err set on malformed input.
bool build_tri_plan(int64_t n, const int32_t* rowptr, const int32_t* col, const double* val, bool upper,
                    const int32_t* in_map, const int32_t* out_map, TriPlan* out, std::string* err);

// Plans of z = Pc U^{-1} L^{-1} Pr q for Pr A Pc = L U (perm_r / perm_c as SuperLU stores them:
// y[perm_r[i]] = q[i], z[i] = v[perm_c[i]]).
bool build_ilu_plans(int64_t n, const int32_t* l_rowptr, const int32_t* l_col, const double* l_val,
                     const int32_t* u_rowptr, const int32_t* u_col, const double* u_val, const int32_t* perm_r,
                     const int32_t* perm_c, TriPlan* L, TriPlan* U, std::string* err);

// The launch executed sequentially in ticket order (L's blocks, then U's), reading values through
// the same LDS-window / granule split; fails if any value is read before it was produced (which
// on the GPU would be a wait on a later ticket).  Uses separate multiply and subtract roundings.
bool emulate_ilu_apply(const TriPlan& L, const TriPlan& U, const double* q, double* z, std::string* err,
                       int64_t* far_steps = nullptr);  // [2]: staged steps reading another block's rows

}  // namespace spis
