// kernels.h — device kernels of the CGMRES/FGMRES inner loop (gfx950, fp64).
// Internal header of libspis.so; the public boundary is include/spis.h.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace spis {

constexpr int kBlock = 256;      // threads per workgroup (4 waves of 64)
constexpr int kRowCap = 256;     // rows per SpMV row block (one thread per row)
constexpr int kNnzCap = 2048;    // nnz staged in LDS per row block (16 KiB fp64)
constexpr int kItemCap = 2048;   // merge items (rows + nnz) per row block
constexpr int kDualCap = 1024;   // nnz / items per row block of the fused dual SpMV (2 x 8 KiB LDS)
constexpr int kSpmvGrid = 2048;  // max SpMV workgroups (= max epilogue partials)
constexpr int kPipeCap = 2048;   // nnz per row block of the pipelined SpMVs (K1p / K1dp: kNnzCap / kItemCap table)
constexpr int kPipeGridFixed = 768;  // pipelined SpMV workgroups on several ranks (MI355X: 256 CUs x 3 resident)
constexpr int kRedGrid = 1024;   // max BLAS-1 workgroups (= max reduction partials)
constexpr int kMaxK = 1024;      // max Krylov dimension handled by the GEMV's LDS copy of y
constexpr int kGramChunk = 32;   // vector elements staged per Gram chunk
constexpr int kGramMaxVec = 64;  // max vectors on either side of one Gram launch (<= 256 4x4 tiles)
constexpr int kYArg = 128;
constexpr int kCgsMax = 32;      // basis vectors per step of the opt-in CGS2 orthogonalisation
constexpr int kMgsPer = 4;       // 16-B pairs per lane per round in MGS / normalise (loads issued first)
constexpr int kConGramGrid = 1024;  // max workgroups (partial slots) of the fused constraint Gram      // GEMV coefficients passed by value up to this p

struct YArg {
  double v[kYArg];
};

// SpMV epilogues (fused into the row reduction of the same launch)
enum Epilogue : int {
  kEpiPlain = 0,    // y = A x
  kEpiDot = 1,      // y = A x ; partial += aux . y       (first MGS dot, solvers.py:194)
  kEpiResNorm = 2,  // partial += (A x - b)^2, no store   (true residual, solvers.py:290)
  kEpiR0 = 3        // y = b - A x ; partial += y^2       (r0 and beta, solvers.py:167-175)
};

struct CsrView {
  int64_t n_rows;
  const int32_t* indptr;
  const int32_t* indices;
  const double* vals;
  const int32_t* blk_row;  // row-block boundaries [n_blk + 1]
  int32_t n_blk;
  // XCD-swizzled block walk: workgroups dealt to XCD x (blockIdx % 8) take a contiguous eighth of
  // each grid-stride round of row blocks.  On the dual SpMV's 1024 table it cuts the reads from
  // 287 to 223 MB per launch and runs 46.7 -> 45.5 us alone (kbench), but 51 -> 52-53 us inside
  // the solver: off.  K1 launches on a swizzled table follow it, so partials group alike.
  bool swz = false;
  // Pipelined SpMV (K1p / K1dp): with a (row start, nz start) table per row block, the
  // launch_spmv* entry points run the software-pipelined kernels instead (next block's val/col and
  // row data loaded while the current block's gathers are in flight).  walk: 0 = grid-stride over
  // blockIdx; 1 = XCD-local (workgroups blockIdx % 8 == x walk the x-th eighth of the blocks).
  const int2* blk_meta = nullptr;
  int walk = 0;
  // C16 (col16.h): 16-bit columns + per-block base columns, in the table's block order
  const uint16_t* col16 = nullptr;
  const int4* blk_base = nullptr;
};

// grid sizes (a fixed count when partials are all-reduced across ranks)
int spmv_grid(const CsrView& A, bool fixed);
int blas_grid(int64_t n, bool fixed);

// Events carried by a kernel's own dispatch (hipExtLaunchKernel): `start` / `stop` are recorded
// at the launch's start / completion without a separate marker packet on the stream (a marker
// costs ~6 us of queue time between dependent kernels).
struct LaunchEv {
  hipEvent_t start = nullptr;
  hipEvent_t stop = nullptr;
};

// (zf, gen, kEpiR0 on the pipelined table only: *zf != gen means x is all zeros (launch_copy_flag)
// and A finite: r = aux bit for bit without reading the matrix)
hipError_t launch_spmv(const CsrView& A, int epi, const double* x, double* y, const double* aux,
                       double* partials, int grid, hipStream_t s, const LaunchEv* ev = nullptr,
                       const unsigned* zf = nullptr, unsigned gen = 0);
// K1d: residual SpMV of x1 (||A x1 - b||^2 partials -> part1) and Arnoldi SpMV of x2 (w = A x2,
// q0.w partials -> part2) reading the matrix once; both bit-identical to launch_spmv's.  A must
// carry the kDualCap row-block table; grid <= kSpmvGrid (the partial arrays' length)
hipError_t launch_spmv_dual(const CsrView& A, const double* x1, const double* b, double* part1,
                            const double* x2, double* w, const double* q0, double* part2, int grid,
                            hipStream_t s, const LaunchEv* ev = nullptr);
// K1p / K1dp (A.blk_meta on a kPipeCap table): mode 0-3 = launch_spmv's epilogue (x1, aux1, y1,
// part1); mode 4 = the dual (x1, aux1 = b, part1: residual; x2, aux2 = q0, y2 = w, part2: Arnoldi);
// mode 6 = two true residuals (x1, x2 against aux1 = aux2 = b: ||.||^2 partials, nothing stored)
hipError_t launch_spmv_pipe(const CsrView& A, int mode, const double* x1, const double* aux1, double* y1,
                            double* part1, const double* x2, const double* aux2, double* y2, double* part2,
                            int grid, hipStream_t s, const LaunchEv* ev = nullptr, const unsigned* zf = nullptr,
                            unsigned gen = 0);
// y -= h_i q_i, h_i = sum(part_in); part_out = q_next . y (or y . y if q_next == nullptr)
hipError_t launch_mgs_step(int64_t n, double* y, const double* qi, const double* qnext,
                           const double* part_in, int n_in, double* part_out, double* h_out,
                           int grid, hipStream_t s, const LaunchEv* ev = nullptr,
                           const double* xpart = nullptr, int n_x = 0, double* x_out = nullptr,
                           unsigned long long* flag = nullptr, const unsigned long long* seq = nullptr);
// (xpart, n_x, x_out): workgroup 0 additionally reduces xpart in sum_partials order into *x_out;
// with flag (host memory), it then publishes *seq there after a system-scope release
// h = sqrt(sum(part_in)); q_next = y / h (if h != 0)
// K2p: the whole MGS chain of one Arnoldi step (j+1 steps + normalise, solvers.py:193-198) in ONE
// persistent launch: w and three basis-vector slices live in registers, each step's partial dots
// are gathered by workgroup 0 through 8-byte {tag, half} granules (sc1 stores / polls), summed in
// a fixed order and handed back the same way.  Per step HBM reads q_{i+1} only (8 N), prefetched behind the
// previous step's exchange; w is not written back (q_{j+1} = w / h is).  Single GPU, N <= 2^20.
constexpr int kChainMaxWG = 256;                       // <= 256 partials per exchange
constexpr int64_t kChainMaxPairs = int64_t(kChainMaxWG) * kBlock * 8;  // PER <= 8 double2 (N <= 2^20)
// K2b (with a dedicated gathering workgroup only): w alone in registers, 255 workgroups of 512
// threads x <= 40 pairs (N <= 10.4 M)
constexpr int64_t kChainBigMaxPairs = int64_t(kChainMaxWG - 1) * 512 * 40;
inline bool mgs_chain_fits(int64_t n, bool aggregator = false) {
  return (n >> 1) <= (aggregator ? kChainBigMaxPairs : kChainMaxPairs);
}
hipError_t launch_mgs_chain(int64_t n, const double* w, double* Q, int64_t pitch, int j, const double* part_in,
                            int n_in, double* hcol, unsigned long long* gran, unsigned* epoch, unsigned* err,
                            hipStream_t s, const LaunchEv* ev, const double* xpart, int n_x, double* x_out,
                            unsigned long long* flag, const unsigned long long* seq, bool aggregator = false,
                            bool nt = false, double* gsub = nullptr, const double* yx_host = nullptr, int px = 0,
                            const double* x0 = nullptr, double* xo = nullptr, int tw = 0);
// (tw: K2q with nt — q_0 .. q_{tw-1} and x0 with ordinary loads, to stay Infinity-Cache resident)
// (nt: the chain's basis loads are nontemporal — the matrix stays Infinity-Cache resident)
// gsub != nullptr selects K2q, the pipelined chain (dot products one MGS step early by the
// distributive law; gsub[m] = q_m . q_{m-1}, written by chain m, read by the later chains of the
// same basis); gran then needs kChainGranLag granules.  Beyond K2p's size it falls back to K2b.
// K2q only: px > 0 fuses the GEMV xo = Q[:, :px] yx + x0 (px <= j, p <= kYArg; K4's arithmetic).
constexpr int kChainGranLag = 12 * kChainMaxWG + 16;
constexpr int kLagDW = 8;  // K2q data waves per workgroup (+1 exchange wave): PER <= 4 pairs per thread
constexpr int kLagDepth = 2;  // K2q: dot products this many MGS steps early (1 or 2)
void set_chain_lag(int lag);  // tuning tools only (tools/chainbench): 1 or 2, process-wide
void set_store_wt(int mask);   // write-through (sc1) output stores: 1 K2q, 2 SpMV, 4 the rest, 8 K2w (default 1; process-wide)
constexpr int kLagNS = 5;     // K2q basis ring: q_{i-1} .. q_{i+3} in registers
constexpr int kChainGsub = 2 * kMaxK + 8;  // K2q gsub: G(m, m-1) at [m], G(m, m-2) at [kMaxK + m]
hipError_t launch_normalize(int64_t n, const double* y, double* qnext, const double* part_in,
                            int n_in, double* h_out, hipStream_t s, int grid, const LaunchEv* ev = nullptr);

// K2c (opt-in CGS2): part = nv x grid partials of q_i . w; update w -= Q coef with, if dot, the
// nv x grid partials of q_i . w' (else ||w'||^2 partials, grid of them); finalize: workgroup i
// reduces vector i's partials into c[i] and, with h_out, writes add[i] + c[i] there.
hipError_t launch_cgs_dot(int64_t n, const double* w, const double* Q, int64_t pitch, int nv, double* part, int grid,
                          hipStream_t s, const LaunchEv* ev = nullptr);
// px > 0 (dot = false): the same pass also writes xo = Q[:, :px] yx + x0 over rows [0, n_gx) (yx on
// the host, px <= kYArg; rows >= n are ghost rows, whose basis entries the halo exchange filled)
hipError_t launch_cgs_update(int64_t n, double* w, const double* Q, int64_t pitch, int nv, const double* coef,
                             bool dot, double* part, int grid, hipStream_t s, bool nt = false, int px = 0,
                             const double* yx = nullptr, const double* x0 = nullptr, double* xo = nullptr,
                             int64_t n_gx = 0);
// K2w (multi-GPU MGS, one reduction for the projections): partials of q_l . w (l < nv) and of
// q_l . q_{nv-1} (l < nv - 1) -> part rows [0, nv) and [nv, 2 nv - 1), grid columns each
// nt: nontemporal basis loads (the matrix stays Infinity-Cache resident between SpMVs, as K2q's),
// except for the first tw basis vectors.  slots != nullptr (the fold): no part rows; the launch's
// last workgroups reduce the partials (published as tagged halves in slots, 2 (2 kCgsMax - 1)
// kRedGrid words; tag: a fresh nonzero value per launch) into d[0, 2 nv - 1) bitwise as
// launch_cgs_finalize(part, grid, 2 nv - 1, d, .., zero_to) would; a timed-out wait sets *err
hipError_t launch_icwy_dot(int64_t n, const double* w, const double* Q, int64_t pitch, int nv, double* part, int grid,
                           hipStream_t s, const LaunchEv* ev = nullptr, bool nt = false, int tw = 0,
                           unsigned long long* slots = nullptr, unsigned tag = 0, double* d = nullptr,
                           int zero_to = 0, unsigned* err = nullptr);
// K2w's update: every workgroup first forms the coefficients from those 2 nv - 1 dots (reduced, d):
// Gram row nv - 1 into G (kCgsMax x kCgsMax, by workgroup 0), h_l = q_l . w - sum_{m<l} h_m G(l, m)
// in l order (h_out: the H column, by workgroup 0), then w -= Q h with the ||w'||^2 partials, and
// with px > 0 the fused GEMV as launch_cgs_update; rpart (nullable): workgroup 0 also reduces a true
// residual's r_in partials and publishes it as launch_finalize(rpart, r_in, r_out, 0, .., flag, seq)
hipError_t launch_icwy_update(int64_t n, double* w, const double* Q, int64_t pitch, int nv, const double* d,
                              double* G, double* h_out, double* part, int grid, hipStream_t s, bool nt = false,
                              int px = 0, const double* yx = nullptr, const double* x0 = nullptr,
                              double* xo = nullptr, int64_t n_gx = 0, const double* rpart = nullptr, int r_in = 0,
                              double* r_out = nullptr, unsigned long long* flag = nullptr,
                              const unsigned long long* seq = nullptr, int tw = 0);
// K2s (one GPU, n <= 256 icwy_onepass_max_grid()): K2w's dot pass, coefficients, update (with the
// fused GEMV for px > 0 and the residual hand-off as launch_icwy_update), norm and normalise in
// one launch over register-resident basis slices; h_col: the H column (H[nv, nv-1] included);
// slots: (2 (2 kCgsMax - 1) + 2) kRedGrid + 4 kCgsMax words; tag: fresh nonzero per launch
constexpr int64_t kIcwySlotWords = 2 * (2 * kCgsMax - 1) * static_cast<int64_t>(kRedGrid) + 2 * (2 * kCgsMax - 1) +
                                   2 * static_cast<int64_t>(kRedGrid) + 2;
int icwy_onepass_max_grid();
// the largest n K2s takes: one resident 256-element chunk per workgroup, or two (the second streamed)
int64_t icwy_onepass_max_n();
hipError_t launch_icwy_onepass(int64_t n, double* w, const double* Q, int64_t pitch, int nv, double* G, double* h_col,
                               unsigned long long* slots, unsigned tag, unsigned* err, hipStream_t s,
                               const LaunchEv* ev, int px = 0, const double* yx = nullptr,
                               const double* x0 = nullptr, double* xo = nullptr, const double* rpart = nullptr,
                               int r_in = 0, double* r_out = nullptr, unsigned long long* flag = nullptr,
                               const unsigned long long* seq = nullptr);
hipError_t launch_cgs_finalize(const double* part, int n_in, int nv, double* c, const double* add, double* h_out,
                               hipStream_t s, int zero_to = 0, bool pin = false);
// the incremental constraint Gram's dots: part[i * grid + blk] = partial of L.v[i] . u (i < nvec);
// reduce with launch_cgs_finalize(part, grid, nvec, ...)
constexpr int kMdMax = 40;
struct VecList {
  const double* v[kMdMax];
};
// (the last n2 of the nvec vectors are dotted with u2 instead; px > 0: also xo = x0 + sum_{i < px}
// y[i] L.v[i], the update GEMV riding along)
hipError_t launch_multidot(int64_t n, const double* u, const VecList& L, int nvec, double* part, int grid,
                           hipStream_t s, const double* u2 = nullptr, int n2 = 0, int px = 0,
                           const double* y = nullptr, const double* x0 = nullptr, double* xo = nullptr);
// x = Z[:, :p] y + x0 ; y on the host (p <= kYArg: passed as a kernel argument) or in HBM
hipError_t launch_gemv(int64_t n, int p, const double* Z, int64_t pitch, const double* y,
                       bool y_on_host, const double* x0, double* x, hipStream_t s,
                       const LaunchEv* ev = nullptr, bool nt = false);
// W[c] = M Z[c] for c < nvec (vectors at stride ldx / ldy)
hipError_t launch_spmm(const CsrView& A, const double* X, int64_t ldx, int nvec, double* Y,
                       int64_t ldy, hipStream_t s);
size_t gram_lds_bytes(int nu, int nv);
// Ut (n x (p+1), row-major) = [Z[:, :p], x0]^T
// (perm: K7m's column order, position 2i = column i, 2i + 1 = column i + 16; p + 1 <= 32)
hipError_t launch_transpose_basis(int64_t n, int p, const double* Z, int64_t pitch, const double* x0,
                                  double* Ut, hipStream_t s, bool perm = false);
// G = [U^T M U | U^T v_0 .. U^T v_{nvv-1}] from Ut (M may be null: linear terms only);
// partials: constraint_gram_partials() x (np1*np1 + nvv*np1) doubles
int constraint_gram_partials();
hipError_t launch_constraint_gram(int64_t n, int np1, const CsrView* M, const double* Ut, int nvv,
                                  const double* const* v, double* partials, double* G, hipStream_t s);
// K7m: the same reduction on the f64 matrix cores from M's CSR (np1 <= 32, Ut in perm order).
// split: the row bounds of the 8 XCD groups (balanced by nonzeros + rows; gram_split)
struct GramSplit {
  int32_t row[9];
};
void gram_split(int64_t n, const int32_t* indptr, GramSplit* out);
// K7t (symmetric M): slot table of 4-row-group segments packed into blocks of ns = kSymSlots slots:
// block b's entries (row-in-group g, slot t) at b * 4 ns + g ns + t, mask[b] = segment-start
// bits | (slots used << 32); G (np1 x np1) = H + H^T
constexpr int kSymSlots = 16;  // (32 measured slower: 166 vs 124 us at C3, profiles/r03_k7t_slots_kernel_stats.csv)
struct SymTabView {
  const int32_t* col;
  const double* val;
  const unsigned long long* mask;
  int32_t nblk;
  int32_t ns;
};
// a column reduction riding in another launch: out[j] = sum over rows of part[row][j], j < npairs
// (reduce_cols_kernel's arithmetic); the transpose's linear terms ride in K7t's H + H^T launch
struct ColReduce {
  int npairs;
  int rows;
  const double* part;
  double* out;
};
hipError_t launch_constraint_gram_sym(int np1, const SymTabView& T, const double* Ut, double* partials, double* G,
                                      hipStream_t s, bool pin = false, const ColReduce* lin = nullptr);
// Ut in the perm order plus the linear terms Gv[c][a] = sum_r U[r][a] v_c[r] (vpart: partials of
// kTransposeGrid x nvv np1; Gv: nvv x np1); np1 <= 32, nvv <= 4
constexpr int kTransposeGrid = 2048;
// pipe: the pipelined transpose (transpose_basis_pipe_kernel) when Ut is 16-byte aligned, else the
// one-tile-at-a-time kernel (bitwise the same Ut and terms)
hipError_t launch_transpose_basis_lin(int64_t n, int p, const double* Z, int64_t pitch, const double* x0,
                                      double* Ut, int nvv, const double* const* v, double* vpart, double* Gv,
                                      hipStream_t s, bool pin = false, bool pipe = true,
                                      ColReduce* defer = nullptr);  // defer: no reduce launch, *defer describes it
hipError_t launch_constraint_gram_mfma(int64_t n, int np1, const CsrView* M, const GramSplit* split,
                                       const double* Ut, int nvv, const double* const* v, double* partials,
                                       double* G, hipStream_t s);
// partial dot / sum of squares
hipError_t launch_dot(int64_t n, const double* x, const double* y, double* part_out, int grid,
                      hipStream_t s);
// out[0] = sum(part) (op 0) or sqrt(sum(part)) (op 1)
hipError_t launch_finalize(const double* part, int n_in, double* out, int op, hipStream_t s,
                           const LaunchEv* ev = nullptr, unsigned long long* flag = nullptr,
                           const unsigned long long* seq = nullptr);
// both reductions of a paired residual SpMV in one launch, each published as launch_finalize's
hipError_t launch_finalize2(const double* part1, const double* part2, int n_in, double* out1, double* out2,
                            hipStream_t s, unsigned long long* flag);
hipError_t launch_axpy(int64_t n, double h, const double* x, double* y, hipStream_t s);
hipError_t launch_copy(int64_t n, const double* x, double* y, hipStream_t s);
// y = x; *flag = gen if any x[e] != 0
hipError_t launch_copy_flag(int64_t n, const double* x, double* y, unsigned* flag, unsigned gen, hipStream_t s);
// streaming read of n doubles (16-B aligned, n even): evicts L2 and the Infinity Cache
hipError_t launch_stream_read(int64_t n, const double* x, double* sink, hipStream_t s);
// send[i] = x[idx[i]]
// send row i = src row idx[i] (row-major, cols doubles per row), i < m
hipError_t launch_gather_rows(int64_t m, int cols, const int32_t* idx, const double* src, double* send,
                              hipStream_t s);
hipError_t launch_gather(int64_t m, const int32_t* idx, const double* x, double* send,
                         hipStream_t s);
// G_partial[block][a*nv+b] over the block's chunks; then reduced into G
hipError_t launch_gram(int64_t n, int nu, const double* const* U, int nv, const double* const* V,
                       double* partials, int grid, double* G, hipStream_t s);

}  // namespace spis
