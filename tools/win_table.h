// win_table.h — host-side tables of the windowed SpMV experiment (K1w, tools/spmv_variants.hip spmv_win_kernel;
// measured slower than K1dp, DESIGN.md §3 "LDS-staged x windows").
//
// Each row block of the solver's SpMV table gathers x at a few hundred to ~2,000 distinct
// columns, in a handful of narrow ranges (swe: the block's own DoF group and the coupled groups'
// matching ranges).  K1w loads those ranges as whole 64-column chunks with coalesced loads into
// LDS, one block ahead, and the products then gather from LDS: no dependent global round trip
// between a block's column indices and its x values.  The tables built here:
//   - the block boundaries, split (by rows) so that no block touches more than kWinChunks
//     distinct chunks (a row is never split: rows stay bit-identical);
//   - per block, its chunk ids (col / 64), ascending, padded with -1 to kWinChunks;
//   - per nonzero, its window position lidx = slot * 64 + col % 64 (uint16), which replaces the
//     32-bit column in the kernel's matrix stream (10 instead of 12 B per nonzero).
#pragma once

#include <algorithm>
#include <cstdint>
#include <vector>

namespace spis {

#ifndef SPIS_WIN_CHUNKS
#define SPIS_WIN_CHUNKS 32
#endif
constexpr int kWinChunks = SPIS_WIN_CHUNKS;  // 64-column chunks per block window: 32 -> 2,048 columns, 32 KB as (x1, x2) pairs

// distinct 64-column chunks of rows [r0, r1)
inline int win_chunks(const int32_t* rp, const int32_t* ci, int32_t r0, int32_t r1, std::vector<int32_t>& tmp) {
  tmp.clear();
  for (int64_t e = rp[r0]; e < rp[r1]; ++e) tmp.push_back(ci[e] >> 6);
  std::sort(tmp.begin(), tmp.end());
  return static_cast<int>(std::unique(tmp.begin(), tmp.end()) - tmp.begin());
}

// split blocks (row boundaries blk) whose window exceeds kWinChunks; false if a single row does
inline bool win_split_blocks(const int32_t* rp, const int32_t* ci, std::vector<int32_t>& blk) {
  std::vector<int32_t> out{blk.front()}, tmp;
  std::vector<std::pair<int32_t, int32_t>> todo;
  for (size_t b = 0; b + 1 < blk.size(); ++b) {
    todo.assign(1, {blk[b], blk[b + 1]});
    while (!todo.empty()) {
      const auto [r0, r1] = todo.back();
      todo.pop_back();
      if (win_chunks(rp, ci, r0, r1, tmp) <= kWinChunks) {
        out.push_back(r1);
        continue;
      }
      if (r1 - r0 < 2) return false;
      const int32_t rm = r0 + (r1 - r0) / 2;
      todo.push_back({rm, r1});  // the lower half is taken next (LIFO): boundaries stay ascending
      todo.push_back({r0, rm});
    }
  }
  blk.swap(out);
  return true;
}

// chunk ids per block, in the order of the table the kernel walks (order[i] = natural block of
// table entry i; empty = natural order), and the window position of every nonzero
inline void win_build(const int32_t* rp, const int32_t* ci, const std::vector<int32_t>& blk,
                      const std::vector<int64_t>& order, std::vector<int32_t>& chunks, std::vector<uint16_t>& lidx) {
  const int64_t nb = static_cast<int64_t>(blk.size()) - 1;
  std::vector<int32_t> nat(static_cast<size_t>(nb) * kWinChunks, -1), tmp;
  lidx.assign(static_cast<size_t>(rp[blk.back()] - rp[blk.front()]), 0);
  for (int64_t b = 0; b < nb; ++b) {
    const int nc = win_chunks(rp, ci, blk[b], blk[b + 1], tmp);
    std::copy(tmp.begin(), tmp.begin() + nc, nat.begin() + b * kWinChunks);
    for (int64_t e = rp[blk[b]]; e < rp[blk[b + 1]]; ++e) {
      const int slot = static_cast<int>(std::lower_bound(tmp.begin(), tmp.begin() + nc, ci[e] >> 6) - tmp.begin());
      lidx[e - rp[blk.front()]] = static_cast<uint16_t>(slot * 64 + (ci[e] & 63));
    }
  }
  if (order.empty()) {
    chunks.swap(nat);
    return;
  }
  chunks.assign(nat.size(), -1);
  for (int64_t i = 0; i < nb; ++i)
    std::copy(nat.begin() + order[i] * kWinChunks, nat.begin() + (order[i] + 1) * kWinChunks,
              chunks.begin() + i * kWinChunks);
}

}  // namespace spis
