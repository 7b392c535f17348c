// sptrsv.h — K8: device apply of an incomplete-LU preconditioner.
// Internal header of libspis.so; the public boundary is include/spis.h (spis_ilu_*).
//
// z = Pc U^{-1} L^{-1} Pr q for Pr A Pc = L U (SuperLU's factors as scipy's spilu returns them;
// the reference calls pre.solve at solvers.py:152-154,190).  Both triangular solves run in ONE
// launch, sync-free: rows are renumbered by level (rows of a level depend only on earlier levels),
// grouped into blocks of consecutive levels, and blocks are handed out to waves in level order
// by an atomic ticket, L's blocks before U's.  A value computed by another wave is read from a
// 64-bit granule (the double itself, published with ONE sc1 store; the consumer polls it with sc1
// loads until it is no longer the sentinel); a value computed earlier by the same wave is read
// from that wave's LDS window.  Every wave only ever waits on rows of smaller tickets, which were
// taken by running waves, so the launch cannot deadlock whatever the dispatch order.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "ilu_plan.h"  // kTriRows, kTriBlockCap, kTriSentinel

namespace spis {

// one triangular factor in solve order (position t = rank of the row in (level, index) order)
struct TriDev {
  const int32_t* rowptr;    // [n+1] entries of the row at position t
  const int32_t* col;       // position of each dependency (strictly earlier in solve order)
  const double* val;
  const double* diag;       // U: the diagonal (divided by, as SuperLU does); L: null (unit)
  const int32_t* in_idx;    // L: index of q to read; U: position of y in L's granule array
  const int32_t* out_idx;   // U: index of z to write; L: null
  const int32_t* blk_row;   // [nb+1] block b covers positions [blk_row[b], blk_row[b+1])
  const int32_t* blk_step;  // [nb+1] steps of block b
  const int32_t* step_row;  // [ns+1] step s covers positions [step_row[s], step_row[s+1]) (<= 64)
  const int32_t* step_long; // [ns] 1: rows of step s solved one per wave (lanes split each row)
  const int32_t* blk_ent;   // [nb+1] first entry of block b
  const int32_t* blk_long;  // [nb] 1: long-row block (one step, read from HBM, not staged)
  int32_t nb;
};

// gran: [2n] granules, y (L's solution) then v (U's), set to the sentinel by the launcher; ticket: one u32 (zeroed by the
// launcher); err: set non-zero when a bounded spin gave up (the value is then published as NaN).
hipError_t launch_ilu_apply(int64_t n, const TriDev& L, const TriDev& U, const double* q, double* gran,
                            double* z, unsigned* ticket, unsigned* err, hipStream_t s);

}  // namespace spis
