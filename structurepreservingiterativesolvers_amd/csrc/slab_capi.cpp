// slab_capi.cpp — host-only C entry point over slab_order.h, built into liblsq_host.so so that the
// slab order of the SpMV row blocks is checked on CPU.  Not part of the product ABI.
#include <vector>

#include "slab_order.h"

extern "C" {

// blk[nb1] = row-block boundaries; pairs_out[4 (nb1 - 1)] = (row start, nz start, row end, nz end)
// per block in slab order.  Returns 1 when reordered, 0 when the natural order stands.
int slab_order_blocks(int64_t n, const int32_t* rp, const int32_t* ci, const int32_t* blk, int64_t nb1,
                      int32_t* pairs_out) {
  std::vector<int32_t> b(blk, blk + nb1), pairs;
  if (!spis::build_slab_order(n, rp, ci, b, pairs)) return 0;
  for (size_t i = 0; i < pairs.size(); ++i) pairs_out[i] = pairs[i];
  return 1;
}

}  // extern "C"
