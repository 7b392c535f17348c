// col16.h — host-side 16-bit column encoding of the SpMV row blocks (spis.cpp at upload,
// tools/kbench, the host test library).
#pragma once
#include <algorithm>
#include <cstdint>
#include <vector>

namespace spis {

// A row block of an FE operator gathers from a few narrow ranges of x (swe: its own DoF group's
// neighbourhood and the two coupled groups' matching ranges; at C3 every 2048-nnz block spans
// <= 4 ranges of < 4096 columns).  Each block therefore gets up to kCol16Bases base columns, and
// each nonzero's column becomes a 2-bit base index and a 14-bit offset: 2 B per nonzero instead
// of 4 (the matrix stream 12 -> 10 B per nonzero).  The kernels decode col = base[k] + offset, so
// every gather, product and row sum is unchanged (bit-identical).  false (no copy) when a block
// needs more than kCol16Bases ranges of 2^14 columns.
constexpr int kCol16Bases = 4;
constexpr int kCol16Bits = 14;

// blk: row-block boundaries [nb + 1]; col16: nnz entries; bases: 4 per block
inline bool build_col16(const int32_t* rp, const int32_t* ci, const std::vector<int32_t>& blk,
                        std::vector<uint16_t>& col16, std::vector<int32_t>& bases) {
  const int64_t nb = static_cast<int64_t>(blk.size()) - 1;
  if (nb < 1) return false;
  const int64_t nnz = rp[blk[nb]];
  col16.assign(static_cast<size_t>(std::max<int64_t>(nnz, 1)), 0);
  bases.assign(static_cast<size_t>(kCol16Bases * nb), 0);
  std::vector<int32_t> u;
  for (int64_t b = 0; b < nb; ++b) {
    const int32_t e0 = rp[blk[b]], e1 = rp[blk[b + 1]];
    if (e1 == e0) continue;
    u.assign(ci + e0, ci + e1);
    std::sort(u.begin(), u.end());
    int k = 0;
    int32_t start[kCol16Bases];
    for (size_t i = 0; i < u.size();) {  // greedy ranges of 2^14 columns over the sorted columns
      if (k == kCol16Bases) return false;
      start[k] = u[i];
      const int64_t lim = static_cast<int64_t>(u[i]) + (int64_t(1) << kCol16Bits);
      while (i < u.size() && u[i] < lim) ++i;
      ++k;
    }
    for (int j = 0; j < k; ++j) bases[kCol16Bases * b + j] = start[j];
    for (int32_t e = e0; e < e1; ++e) {
      int j = k - 1;
      while (start[j] > ci[e]) --j;  // the last range starting at or below the column
      col16[e] = static_cast<uint16_t>((j << kCol16Bits) | (ci[e] - start[j]));
    }
  }
  return true;
}

}  // namespace spis
