// slab_order.h — host-side slab order of the SpMV row blocks (spis.cpp at upload, tools/kbench,
// the host test library).
#pragma once
#include <algorithm>
#include <cstdint>
#include <utility>
#include <vector>

namespace spis {

// Slab order of the row blocks for the XCD-local walk (each XCD takes a contiguous eighth of the
// table, so its gathers of x stay in its own L2 when its rows' columns are close).  FE matrices
// often number DoF groups one after another (swe RT2 x DG0: edge, interior and cell DoFs): a
// contiguous eighth of the rows is then one group's slab, whose columns sit in three distant
// ranges of x shared with two other XCDs (C3: each 128-B line of x fetched by 3.0 XCDs).  One
// pass of label propagation fixes that: rows get kSlabLabels labels by contiguous nnz ranges,
// then each row takes the label most of its columns carry (a coupled DoF of another group adopts
// the slab of the DoFs it couples to), a block the label most of its rows carry, and the blocks
// are stably sorted by label (C3: 3.0 -> 1.14 XCDs per line).  Rows are unchanged (each row
// sum bit-identical); only which workgroup adds a row into its partial dot products changes.
// Square matrices only (a column is a row); false when the order would equal the contiguous one.
constexpr int kSlabLabels = 64;
// the rows' slab labels (one propagation pass over the matrix's pattern); false if too small.
// key (optional): each row's position inside its slab, the mean index of its columns that carry
// its label (the row's own index when none do).  The dominant DoF group's numbering is then the
// common coordinate of every group in the slab: an swe interior-RT or rho row gets the position of
// its cell's edges (slab key, build_slab_order).
inline bool slab_labels(int64_t n, const int32_t* rp, const int32_t* ci, std::vector<uint8_t>& lab,
                        std::vector<double>* key = nullptr) {
  const int64_t nnz = rp[n];
  if (n < 1 || nnz < 1) return false;
  std::vector<uint8_t> lab0(n);
  lab.assign(n, 0);
  if (key) key->assign(n, 0.0);
  for (int64_t r = 0; r < n; ++r)
    lab0[r] = static_cast<uint8_t>(std::min<int64_t>(kSlabLabels - 1, static_cast<int64_t>(rp[r]) * kSlabLabels / nnz));
  int cnt[kSlabLabels];
  for (int64_t r = 0; r < n; ++r) {
    std::fill(cnt, cnt + kSlabLabels, 0);
    for (int32_t i = rp[r]; i < rp[r + 1]; ++i) ++cnt[lab0[ci[i]]];
    int best = lab0[r];  // ties (and empty rows) keep the row's own label
    for (int l = 0; l < kSlabLabels; ++l)
      if (cnt[l] > cnt[best]) best = l;
    lab[r] = static_cast<uint8_t>(best);
    if (key) {
      double s = 0.0;
      int m = 0;
      for (int32_t i = rp[r]; i < rp[r + 1]; ++i)
        if (lab0[ci[i]] == best) {
          s += ci[i];
          ++m;
        }
      (*key)[r] = m > 0 ? s / m : static_cast<double>(r);
    }
  }
  return true;
}

// a stable order of items by label (then by key within a label, when given); false when it is
// the natural one
inline bool slab_sort(const std::vector<uint8_t>& item_lab, std::vector<int64_t>& order,
                      const std::vector<double>* item_key = nullptr) {
  const int64_t m = static_cast<int64_t>(item_lab.size());
  order.resize(m);
  for (int64_t i = 0; i < m; ++i) order[i] = i;
  if (item_key) {
    const std::vector<double>& k = *item_key;
    std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
      return item_lab[a] != item_lab[b] ? item_lab[a] < item_lab[b] : k[a] < k[b];
    });
  } else {
    std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return item_lab[a] < item_lab[b]; });
  }
  for (int64_t i = 0; i < m; ++i)
    if (order[i] != i) return true;
  return false;
}

// the row blocks blk in slab order of the rows' labels lab; with key (slab_labels' row positions)
// the blocks of one slab follow their rows' mean position, so the slab's DoF groups are walked
// side by side instead of one group after another.  Each XCD's workgroups take its eighth's blocks
// round-robin, about 100 consecutive blocks at a time, and at C5 a slab holds ~1,500 blocks: in
// group order a slab's interior and rho blocks re-gather the x lines its edge blocks gathered
// ~1,000 blocks earlier, long after the XCD's 4 MB L2 has turned over.
inline bool build_slab_order(const int32_t* rp, const std::vector<uint8_t>& lab, const std::vector<int32_t>& blk,
                             std::vector<int32_t>& pairs, std::vector<int64_t>* order_out = nullptr,
                             const std::vector<double>* key = nullptr) {
  const int64_t nb = static_cast<int64_t>(blk.size()) - 1;
  if (nb < 16) return false;
  std::vector<uint8_t> blab(nb);
  std::vector<double> bkey(key ? nb : 0);
  int cnt[kSlabLabels];
  for (int64_t b = 0; b < nb; ++b) {  // a block: the label most of its rows carry
    std::fill(cnt, cnt + kSlabLabels, 0);
    for (int32_t r = blk[b]; r < blk[b + 1]; ++r) ++cnt[lab[r]];
    int best = 0;
    for (int l = 1; l < kSlabLabels; ++l)
      if (cnt[l] > cnt[best]) best = l;
    blab[b] = static_cast<uint8_t>(best);
    if (key) {  // the mean position of the block's rows that carry its label
      double s = 0.0;
      for (int32_t r = blk[b]; r < blk[b + 1]; ++r)
        if (lab[r] == best) s += (*key)[r];
      bkey[b] = cnt[best] > 0 ? s / cnt[best] : static_cast<double>(blk[b]);
    }
  }
  std::vector<int64_t> order;
  if (!slab_sort(blab, order, key ? &bkey : nullptr)) return false;
  pairs.resize(4 * nb);  // per block (row start, nz start, row end, nz end): the kernels' int2 pairs
  for (int64_t i = 0; i < nb; ++i) {
    const int64_t b = order[i];
    pairs[4 * i] = blk[b];
    pairs[4 * i + 1] = rp[blk[b]];
    pairs[4 * i + 2] = blk[b + 1];
    pairs[4 * i + 3] = rp[blk[b + 1]];
  }
  if (order_out) order_out->swap(order);
  return true;
}

inline bool build_slab_order(int64_t n, const int32_t* rp, const int32_t* ci, const std::vector<int32_t>& blk,
                             std::vector<int32_t>& pairs, bool keyed = false) {
  std::vector<uint8_t> lab;
  std::vector<double> key;
  return static_cast<int64_t>(blk.size()) > 16 && slab_labels(n, rp, ci, lab, keyed ? &key : nullptr) &&
         build_slab_order(rp, lab, blk, pairs, nullptr, keyed ? &key : nullptr);
}

}  // namespace spis
