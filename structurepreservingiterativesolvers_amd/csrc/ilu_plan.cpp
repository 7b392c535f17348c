// ilu_plan.cpp — see ilu_plan.h.
#include "ilu_plan.h"

#include <algorithm>
#include <cmath>
#include <cstring>

namespace spis {

namespace {
bool bad(std::string* err, const std::string& m) {
  if (err) *err = m;
  return false;
}
}  // namespace

bool build_tri_plan(int64_t n, const int32_t* rowptr, const int32_t* col, const double* val, bool upper,
                    const int32_t* in_map, const int32_t* out_map, TriPlan* out, std::string* err) {
  const char* name = upper ? "U" : "L";
  if (n < 0 || n > INT32_MAX - 1) return bad(err, "bad n");
  if (rowptr[0] != 0) return bad(err, std::string(name) + ": rowptr[0] != 0");
  for (int64_t i = 0; i < n; ++i)
    if (rowptr[i + 1] < rowptr[i]) return bad(err, std::string(name) + ": rowptr not monotone");
  TriPlan& P = *out;
  P = TriPlan();
  P.n = n;
  // strict part and diagonal; levels (L: ascending rows, U: descending)
  std::vector<int32_t> lev(n, 0);
  P.diag.assign(upper ? n : 0, 0.0);
  for (int64_t ii = 0; ii < n; ++ii) {
    const int64_t i = upper ? n - 1 - ii : ii;
    int32_t l = 0;
    bool has_diag = false;
    for (int32_t e = rowptr[i]; e < rowptr[i + 1]; ++e) {
      const int32_t c = col[e];
      if (c < 0 || c >= n) return bad(err, std::string(name) + ": column index out of range");
      if (c == i) {
        if (upper) {
          P.diag[i] = val[e];
          has_diag = val[e] != 0.0;
        } else if (val[e] != 1.0) {
          return bad(err, "L: stored diagonal entry is not 1 (unit lower factor expected)");
        }
        continue;
      }
      if (upper ? c < i : c > i) return bad(err, std::string(name) + ": entry on the wrong side of the diagonal");
      l = std::max(l, lev[c] + 1);
    }
    if (upper && !has_diag) return bad(err, "U: zero or missing diagonal entry");
    lev[i] = l;
    P.levels = std::max(P.levels, l + 1);
  }
  // solve order: by level, then row index (counting sort)
  std::vector<int32_t> lstart(P.levels + 1, 0);
  for (int64_t i = 0; i < n; ++i) ++lstart[lev[i] + 1];
  for (int l = 0; l < P.levels; ++l) lstart[l + 1] += lstart[l];
  std::vector<int32_t> ord(n), fill(lstart.begin(), lstart.end() - (P.levels ? 1 : 0));
  P.pos.assign(n, 0);
  for (int64_t i = 0; i < n; ++i) {
    const int32_t t = fill[lev[i]]++;
    ord[t] = static_cast<int32_t>(i);
    P.pos[i] = t;
  }
  // strict entries per row, for the long-row rule
  std::vector<int32_t> len(n, 0);
  for (int64_t i = 0; i < n; ++i)
    for (int32_t e = rowptr[i]; e < rowptr[i + 1]; ++e) len[i] += col[e] != i;
  // blocks, each homogeneous: levels holding a row longer than kLongRow -> one block per
  // kLongStep rows (solved a row per wave, read from HBM); other levels are cut into steps of
  // <= 64 rows and <= kTriBlockNnz entries; a level that is one step is packed with its
  // neighbours into a block of <= kTriBlockCap rows / kTriBlockNnz entries (staged in LDS),
  // a level of several steps gets one block per step (they run in parallel)
  P.blk_row.push_back(0);
  P.blk_step.push_back(0);
  P.step_row.push_back(0);
  int32_t cur = 0, cur_nnz = 0;  // rows / entries in the open block
  auto flush = [&](bool is_long) {
    if (cur == 0) return;
    P.blk_row.push_back(P.step_row.back());
    P.blk_step.push_back(static_cast<int32_t>(P.step_row.size()) - 1);
    P.blk_long.push_back(is_long);
    cur = cur_nnz = 0;
  };
  std::vector<int32_t> cuts;  // step boundaries of one level
  for (int l = 0; l < P.levels; ++l) {
    const int32_t a = lstart[l], b = lstart[l + 1];
    bool is_long = false;
    for (int32_t t = a; t < b; ++t) is_long = is_long || len[ord[t]] > kLongRow;
    if (is_long) {
      flush(false);
      for (int32_t r = a; r < b; r += kLongStep) {
        P.step_row.push_back(std::min(b, r + kLongStep));
        P.step_long.push_back(1);
        cur = std::min(b, r + kLongStep) - r;
        flush(true);
      }
      continue;
    }
    cuts.clear();
    int32_t rows = 0, ents = 0;
    for (int32_t t = a; t < b; ++t) {
      if (rows == kTriRows || ents + len[ord[t]] > kTriBlockNnz) {
        cuts.push_back(t);
        rows = ents = 0;
      }
      ++rows;
      ents += len[ord[t]];
    }
    cuts.push_back(b);
    if (cuts.size() > 1) {
      flush(false);
      for (int32_t cut : cuts) {
        cur = cut - P.step_row.back();
        P.step_row.push_back(cut);
        P.step_long.push_back(0);
        flush(false);
      }
    } else {
      if (cur + (b - a) > kTriBlockCap || cur_nnz + ents > kTriBlockNnz) flush(false);
      P.step_row.push_back(b);
      P.step_long.push_back(0);
      cur += b - a;
      cur_nnz += ents;
    }
  }
  flush(false);
  // rows in solve order, dependencies as positions; L keeps ascending columns, U descending
  P.rowptr.assign(n + 1, 0);
  P.in_idx.assign(n, 0);
  if (out_map) P.out_idx.assign(n, 0);
  std::vector<double> d(upper ? n : 0);
  for (int32_t t = 0; t < n; ++t) {
    const int32_t i = ord[t];
    const int32_t e0 = rowptr[i], e1 = rowptr[i + 1];
    for (int32_t k = 0; k < e1 - e0; ++k) {
      const int32_t e = upper ? e1 - 1 - k : e0 + k;
      if (col[e] == i) continue;
      P.col.push_back(P.pos[col[e]]);
      P.val.push_back(val[e]);
    }
    P.rowptr[t + 1] = static_cast<int32_t>(P.col.size());
    P.in_idx[t] = in_map[i];
    if (out_map) P.out_idx[t] = out_map[i];
    if (upper) d[t] = P.diag[i];
  }
  if (upper) P.diag.swap(d);
  P.blk_ent.resize(P.blk_row.size());
  for (size_t i = 0; i < P.blk_row.size(); ++i) P.blk_ent[i] = P.rowptr[P.blk_row[i]];
  return true;
}

bool build_ilu_plans(int64_t n, const int32_t* l_rowptr, const int32_t* l_col, const double* l_val,
                     const int32_t* u_rowptr, const int32_t* u_col, const double* u_val, const int32_t* perm_r,
                     const int32_t* perm_c, TriPlan* L, TriPlan* U, std::string* err) {
  std::vector<int32_t> ipr(n, -1), ipc(n, -1);
  for (int64_t i = 0; i < n; ++i) {
    if (perm_r[i] < 0 || perm_r[i] >= n || ipr[perm_r[i]] >= 0) return bad(err, "perm_r is not a permutation");
    if (perm_c[i] < 0 || perm_c[i] >= n || ipc[perm_c[i]] >= 0) return bad(err, "perm_c is not a permutation");
    ipr[perm_r[i]] = static_cast<int32_t>(i);
    ipc[perm_c[i]] = static_cast<int32_t>(i);
  }
  // L row j reads q[ipr[j]] (y[perm_r[i]] = q[i]); U row j reads y_j, writes z[ipc[j]]
  if (!build_tri_plan(n, l_rowptr, l_col, l_val, false, ipr.data(), nullptr, L, err)) return false;
  return build_tri_plan(n, u_rowptr, u_col, u_val, true, L->pos.data(), ipc.data(), U, err);
}

bool emulate_ilu_apply(const TriPlan& L, const TriPlan& U, const double* q, double* z, std::string* err,
                       int64_t* far_steps) {
  if (far_steps) far_steps[0] = far_steps[1] = 0;
  const int64_t n = L.n;
  std::vector<double> gy(n), gv(n);
  double sentinel;
  const unsigned long long s = kTriSentinel;
  std::memcpy(&sentinel, &s, 8);
  std::fill(gy.begin(), gy.end(), sentinel);
  std::fill(gv.begin(), gv.end(), sentinel);
  auto is_sent = [&](double v) { return std::memcmp(&v, &s, 8) == 0; };
  std::vector<char> done_in_window;
  for (int pass = 0; pass < 2; ++pass) {
    const TriPlan& F = pass ? U : L;
    std::vector<double>& gout = pass ? gv : gy;
    for (int32_t b = 0; b < F.n_blocks(); ++b) {
      const int32_t r0 = F.blk_row[b], r1 = F.blk_row[b + 1];
      std::vector<double> sv(r1 - r0, sentinel);
      if (r1 - r0 > kTriBlockCap) return bad(err, "block larger than the LDS window");
      if (!F.blk_long[b] && F.blk_ent[b + 1] - F.blk_ent[b] > kTriBlockNnz)
        return bad(err, "staged block holds more entries than its LDS copy");
      if (F.blk_long[b] != F.step_long[F.blk_step[b]] || (F.blk_long[b] && F.blk_step[b + 1] - F.blk_step[b] != 1))
        return bad(err, "long-row blocks must be single long steps");
      for (int32_t st = F.blk_step[b]; st < F.blk_step[b + 1]; ++st) {
        if (F.step_row[st + 1] - F.step_row[st] > (F.step_long[st] ? kLongStep : kTriRows))
          return bad(err, "step wider than its kind allows");
        std::vector<std::pair<int32_t, double>> res;
        bool far = false;
        for (int32_t row = F.step_row[st]; row < F.step_row[st + 1]; ++row) {
          double acc = pass ? gy[F.in_idx[row]] : q[F.in_idx[row]];
          if (pass && is_sent(acc)) return bad(err, "U row read y before L produced it");
          double sum = 0.0;  // long-row steps: the wave's sum of the row, subtracted once
          for (int32_t e = F.rowptr[row]; e < F.rowptr[row + 1]; ++e) {
            const int32_t c = F.col[e];
            const double v = c >= r0 ? sv[c - r0] : gout[c];
            far = far || c < r0;
            if (c >= row || is_sent(v)) return bad(err, "dependency not produced by an earlier step/ticket");
            const volatile double prod = F.val[e] * v;  // separate roundings (no FMA)
            if (F.step_long[st]) sum += prod;
            else acc -= prod;
          }
          if (F.step_long[st]) acc -= sum;
          if (pass) acc /= F.diag[row];
          res.emplace_back(row, acc);
        }
        if (far && far_steps && !F.blk_long[b]) ++far_steps[pass];
        for (auto& rv : res) {  // a step's results become visible after the step
          sv[rv.first - r0] = rv.second;
          gout[rv.first] = rv.second;
          if (pass) z[F.out_idx[rv.first]] = rv.second;
        }
      }
    }
  }
  return true;
}

}  // namespace spis
