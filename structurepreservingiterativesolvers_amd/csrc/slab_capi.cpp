// slab_capi.cpp — host-only C entry points over slab_order.h and col16.h, built into
// liblsq_host.so so that the slab order and the 16-bit column copy of the SpMV row blocks are
// checked on CPU.  Not part of the product ABI.
#include <vector>

#include "col16.h"
#include "slab_order.h"

extern "C" {

// blk[nb1] = row-block boundaries; pairs_out[4 (nb1 - 1)] = (row start, nz start, row end, nz end)
// per block in slab order.  Returns 1 when reordered, 0 when the natural order stands.
// keyed = 1: blocks of one slab by their rows' mean position (slab key, SPIS_OPT_SLAB_KEY)
int slab_order_blocks_keyed(int64_t n, const int32_t* rp, const int32_t* ci, const int32_t* blk, int64_t nb1,
                            int32_t* pairs_out, int32_t keyed) {
  std::vector<int32_t> b(blk, blk + nb1), pairs;
  if (!spis::build_slab_order(n, rp, ci, b, pairs, keyed != 0)) return 0;
  for (size_t i = 0; i < pairs.size(); ++i) pairs_out[i] = pairs[i];
  return 1;
}

int slab_order_blocks(int64_t n, const int32_t* rp, const int32_t* ci, const int32_t* blk, int64_t nb1,
                      int32_t* pairs_out) {
  return slab_order_blocks_keyed(n, rp, ci, blk, nb1, pairs_out, 0);
}

// col16_out[nnz], bases_out[4 (nb1 - 1)]: the 16-bit column copy (col16.h); 1 = built, 0 = a block
// needs more than 4 ranges of 2^14 columns
int col16_encode(const int32_t* rp, const int32_t* ci, const int32_t* blk, int64_t nb1, uint16_t* col16_out,
                 int32_t* bases_out) {
  std::vector<int32_t> b(blk, blk + nb1), bases;
  std::vector<uint16_t> c16;
  if (!spis::build_col16(rp, ci, b, c16, bases)) return 0;
  const int64_t nnz = rp[blk[nb1 - 1]];
  for (int64_t i = 0; i < nnz; ++i) col16_out[i] = c16[i];
  for (size_t i = 0; i < bases.size(); ++i) bases_out[i] = bases[i];
  return 1;
}

}  // extern "C"
