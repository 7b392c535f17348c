// spis.cpp — libspis.so: context, CSR upload + SpMV schedule, halo exchange (RCCL), BLAS-1
// primitives and the CGMRES / FGMRES / prototypical-CGMRES driver (include/spis.h).
//
// The driver restates solvers.py:131-323 (cgmres), :58-127 (gmres) and :328-445 (cgmres_p)
// around device-resident data: the Krylov basis Q (and Z when preconditioned) lives in HBM as
// row-major (k+1, pitch) fp64, every N-length operation is a HIP kernel (kernels.hip), and only
// the Hessenberg column (j+2 scalars), residual partials and the small LS solution cross PCIe.
// One host synchronisation per iteration: the GEMV + true-residual SpMV of iteration j are
// enqueued together with the Arnoldi step of iteration j+1 (which does not depend on them), and
// the host then waits once for both; a stop at j discards the speculative Arnoldi work.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "ilu_plan.h"
#include "kernels.h"
#include "slab_order.h"
#include "col16.h"
#include "lsq.h"
#include "sptrsv.h"
#include "spis.h"

using namespace spis;

// ------------------------------------------------------------------------------------------------
// errors
// ------------------------------------------------------------------------------------------------
static thread_local std::string g_last_error;

static int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

#define HIP_TRY(expr)                                                                         \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess)                                                                     \
      return fail(SPIS_ERR_HIP, "%s:%d: %s -> %s", __FILE__, __LINE__, #expr,               \
                  hipGetErrorString(_e));                                                     \
  } while (0)

#define NCCL_TRY(expr)                                                                        \
  do {                                                                                        \
    ncclResult_t _r = (expr);                                                                 \
    if (_r != ncclSuccess)                                                                    \
      return fail(SPIS_ERR_RCCL, "%s:%d: %s -> %s", __FILE__, __LINE__, #expr,              \
                  ncclGetErrorString(_r));                                                    \
  } while (0)

#define ST_TRY(expr)                  \
  do {                                \
    int _s = (expr);                  \
    if (_s != SPIS_OK) return _s;     \
  } while (0)

#define ABI_GUARD(...)                                                           \
  try {                                                                          \
    __VA_ARGS__                                                                  \
  } catch (const std::bad_alloc&) {                                              \
    return fail(SPIS_ERR_ALLOC, "host allocation failed");                      \
  } catch (...) {                                                                \
    return fail(SPIS_ERR_STATE, "unexpected C++ exception");                    \
  }

static double now_s() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

static int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

// ------------------------------------------------------------------------------------------------
// objects
// ------------------------------------------------------------------------------------------------
// icwy_d layout: the one-reduce MGS's 2 nv - 1 dots (nv <= kCgsMax), slack, then partR (the true
// residual partials), so that one all-reduce on several GPUs carries both
constexpr int kIcwyROff = 2 * kCgsMax + 8;

struct spis_context {
  int device = 0;
  hipStream_t stream = nullptr;
  double* partA = nullptr;  // reduction partials, ping
  double* partB = nullptr;  // reduction partials, pong
  double* partR = nullptr;  // true-residual partials
  double* dscal = nullptr;  // small device scalars (kMaxK + 8)
  double* pinned = nullptr;  // pinned, device-mapped host staging (kernels write h / partials here)
  double* pinned_dev = nullptr;  // the same memory as seen from the device
  size_t pinned_len = 0;     // doubles
  hipEvent_t ev_arn = nullptr, ev_upd[2] = {nullptr, nullptr};  // solver pipeline events
  hipEvent_t ev_gram = nullptr;  // constrained step: the Gram tile has reached pinned memory
  hipEvent_t ev_xd = nullptr, ev_xd2 = nullptr;  // x_{k-1} written (main stream) / copied to the host (stream2)
  hipEvent_t ev_side = nullptr;  // the end of a solve: stream2's work joined (Solver's last wait)
  unsigned long long seq = 0;  // last completion sequence number handed to a publishing kernel
  double* gram_part = nullptr;
  size_t gram_part_len = 0;
  double* gram_G = nullptr;
  const double** gram_ptrs = nullptr;  // device array of 2 * kGramMaxVec pointers
  double* gram_pinned = nullptr;       // host staging of Gram tiles + pointer lists
  double* cg_part = nullptr;           // fused constraint-Gram partials (per wave)
  size_t cg_part_len = 0;
  double* cg_G = nullptr;              // its reduced output (64*64 + 4*64)
  double* cg_vpart = nullptr;          // K7t: the transpose's linear-term partials
  double* inc_u = nullptr;             // incremental Gram: M z_a (n)
  int64_t inc_u_len = 0;
  double* inc_part = nullptr;          // its multidot partials (values x grid)
  size_t inc_part_len = 0;
  double* inc_res = nullptr;           // its reduced values (device), copied to con_pinned
  size_t inc_res_len = 0;
  ncclComm_t comm = nullptr;
  // several ranks through a host callback instead of RCCL (spis_comm_init_host): the same
  // distributed code path with the collectives staged through host memory, so that several
  // ranks can share one GPU (RCCL refuses that) when the path is rehearsed on a one-GPU box
  spis_host_coll_fn host_coll = nullptr;
  void* host_user = nullptr;
  std::vector<double> host_stage;  // send | recv staging of a host collective
  int nranks = 1, rank = 0;
  bool dist_on() const { return comm != nullptr || host_coll != nullptr; }
  std::vector<spis_workspace*> pool;
  // live kernel timing (spis_profile_*): HIP events on this stream around each timed launch
  bool prof = false;
  int prof_period = 1;            // time every prof_period-th Arnoldi iteration
  int prof_iter = 0;              // iteration counter for the sampling
  int prof_phase = 0;             // advanced per solve: the sampled iterations rotate through every position
  bool fuse_spmv = true;            // residual SpMV of U_j + Arnoldi SpMV of A_{j+2} in one launch
  bool cgs2 = false;                // opt-in CGS2 orthogonalisation (SPIS_OPT_ORTHOG = 1)
  double* cgs_part = nullptr;       // kCgsMax x kRedGrid partials
  double* cgs_c = nullptr;          // c1 [kCgsMax] | c2 [kCgsMax]
  // several GPUs (SPIS_OPT_DIST_MGS): 1 = MGS's projections in one reduction per Arnoldi step
  // (K2w, icwy_*), 0 = one MGS step launch + all-reduce per projection
  int dist_mgs = 1;
  double* icwy_part = nullptr;      // 2 kCgsMax x kRedGrid partials
  double* icwy_d = nullptr;         // the 2 nv - 1 reduced dots, then (at kIcwyROff) partR
  unsigned long long* icwy_slots = nullptr;  // K2w fold / K2s: tagged partial halves (kIcwySlotWords)
  unsigned icwy_tag = 0;                     // the last fold's tag (never 0 on a launch)
  double* icwy_G = nullptr;         // kCgsMax x kCgsMax Gram rows G(l, m) = q_l . q_m, m < l
  double* ut_send = nullptr;        // several GPUs: the Ut rows a constraint matrix's halo sends
  size_t ut_send_len = 0;
  // constraint reduction (SPIS_OPT_CON_GRAM): 0 generic (M Z SpMM + tiled Gram), 1 K7 on the CSR, 2 K7t for
  // symmetric matrices / K7m otherwise, 3 K7m for every matrix
  int con_gram = 2;
  int mgs_chain = 3;                // persistent MGS chain (SPIS_OPT_MGS_CHAIN): 0 off, 1 K2p gathered by workgroup 0, 2 by a dedicated workgroup, 3 K2q pipelined
  int nt_basis = 2;                 // the chain's basis loads nontemporal (SPIS_OPT_NT_BASIS): 0 off, 1 on, 2 auto
  int col16 = 1;                    // the pipelined SpMV on the 16-bit column copy: 1 beyond the Infinity Cache, 2 always (SPIS_OPT_COL16)
  int slab_key = 1;                 // SPIS_OPT_SLAB_KEY: slab order's blocks by position within a slab (at upload)
  // A/B switches, read from the environment once at context creation (SPIS_OPT_GRAM_INC,
  // SPIS_OPT_X0_ZERO_TEST, SPIS_OPT_TRANSPOSE_PIPE; the K2w ones for tools/chainbench only)
  bool gram_inc = true, x0_zero_test = true, transpose_pipe = true;
  bool k2w_fold = true, k2w_onepass = true;
  int k2w_tw = -1;
  int64_t k2w_small_n = -1;
  int spmv_pipe = 5;                // solver SpMVs: 0 = K1/K1d; K1p/K1dp 1 = grid-stride, 2 = XCD-local walk; 5 = auto (2 or 1); 7 = 2 on the natural block order
  // U_j's GEMV on stream2 beside A_{j+1}'s chain when the chain does not carry it (outside L mode,
  // or a constrained LS_j); the dual SpMV waits for it through a stream write / wait on a device word
  hipStream_t stream2 = nullptr;
  double* con_pinned = nullptr;  // the synchronous reduction's results
  size_t con_pinned_len = 0;
  void* gemv_flag = nullptr;  // device word: the side stream's GEMV count
  uint64_t gemv_seq = 0;
  unsigned long long* chain_gran = nullptr;  // exchange granules (kChainGranLag: K2p / K2b / K2q layouts)
  double* chain_gsub = nullptr;              // K2q: Gram entries q_m . q_{m-1}, q_m . q_{m-2} (kChainGsub)
  unsigned* chain_epoch = nullptr;           // tag base, advanced by each chain
  unsigned* chain_err = nullptr;             // pinned, device-mapped: a chain exchange timed out
  unsigned* chain_err_dev = nullptr;
  unsigned* x0_flag = nullptr;  // device word: the solve's generation when its x0 has a nonzero entry
  unsigned x0_gen = 0;
  bool icwy_spin_off = false;  // a one-reduce hand-off (K2w fold / K2s) timed out: finalize launches
  std::vector<hipEvent_t> ev_free;
  struct Pending { int kind; hipEvent_t a, b; };
  std::vector<Pending> ev_pending;
  double prof_ms[SPIS_PROF_KINDS] = {0};
  int64_t prof_n[SPIS_PROF_KINDS] = {0};
  // stream-ordered caching allocator behind spis_malloc / spis_free: freed blocks go to a
  // size-keyed free list and are handed out again in stream order (every user of a block runs on
  // this context's stream), so a steady-state solve loop makes no hipMalloc / hipFree calls
  std::multimap<size_t, void*> free_blocks;
  std::unordered_map<void*, size_t> live_blocks;
  size_t cached_bytes = 0;
};

struct spis_matrix {
  spis_context* ctx = nullptr;
  uint64_t uid = 0;  // unique per upload (cache keys must not use the reusable object address)
  int64_t n_rows = 0, n_cols = 0, nnz = 0;
  int32_t* indptr = nullptr;
  int32_t* indices = nullptr;
  double* vals = nullptr;
  int32_t* blk_row = nullptr;
  int32_t n_blk = 0, n_long = 0;
  int32_t* blk_row_d = nullptr;  // row blocks of <= kDualCap nnz / items for the fused dual SpMV
  int32_t n_blk_d = 0;
  int2* blk_meta_d = nullptr;    // blk_row's blocks (<= kPipeCap nnz) as (row start, nz start): the pipelined kernels' table
  int2* blk_slab_d = nullptr;    // the same blocks as (start, end) pairs in slab order (XCD-local walk 2), or null
  uint16_t* col16_d = nullptr;   // C16 copy of the columns (col16.h), or null
  int4* base_nat_d = nullptr;     // its per-block bases, natural block order
  int4* base_slab_d = nullptr;    // the same in slab order
  bool all_zero = false;
  bool all_finite = true;  // every stored value finite (A x0 with x0 = 0 is then exactly 0)
  GramSplit gram_rows{};  // K7m's XCD-group row ranges (natural row order)
  // K7t's slot table (symmetric matrices; sym_state -1 unknown, 0 not symmetric, 1 built)
  int sym_state = -1;
  int32_t* sym_col = nullptr;
  double* sym_val = nullptr;
  unsigned long long* sym_mask = nullptr;
  int32_t sym_nblk = 0;
  // spis_matrix_set_global: each local column's global index and whether the global matrix is
  // symmetric (several GPUs: a rank's rows of a symmetric matrix are not square, so K7t pairs
  // entries by global index)
  std::vector<int64_t> gid;
  int gsym = -1;
  // halo plan
  int32_t n_ghost = 0;
  std::vector<int32_t> nbr, scnt, rcnt, soff, roff;
  int64_t n_send = 0;
  int32_t* send_idx = nullptr;
  double* send_buf = nullptr;
  CsrView view() const { return CsrView{n_rows, indptr, indices, vals, blk_row, n_blk}; }
  CsrView dual_view() const;
  bool use_col16() const;
};

struct ConCache {
  double* MZ = nullptr;  // (k) x pitch_n : M z_i
  int cols = 0;
  double* Mx0 = nullptr;
  bool mx0_done = false;
  // incremental Gram (con_step_*): the reduced entries of this solve's columns so far, index k = x0:
  // gc(a, b) = z_a . M z_b, gv(a) = v . z_a; gcols = columns held (-1: none, x0's own terms neither)
  int gcols = -1;
  std::vector<double> gc, gv;
};

struct spis_workspace {
  spis_context* ctx = nullptr;
  int64_t n = 0, pitch = 0, pitch_n = 0;
  int k = 0;
  bool sep_z = false;
  double* Q = nullptr;
  double* Zb = nullptr;  // == Q when not preconditioned
  double* w = nullptr;   // Arnoldi vector
  double* xj = nullptr;   // iterate x_j of even j (with ghost space)
  double* xj2 = nullptr;  // x_j of odd j: an update may be enqueued while the previous x is still read
  double* r0 = nullptr;
  double* x0 = nullptr;  // copy of x0 (n)
  double* ext = nullptr;  // scratch SpMV input with ghost space (constraint / preconditioner halos)
  double* ydev = nullptr;
  double* Ut = nullptr;  // transposed [Z, x0] for the fused constraint reduction (n x (p+1))
  int Ut_cols = 0;       // its allocated row capacity (32 or 64)
  int64_t Ut_rows = 0;   // its allocated rows (n, plus a constraint matrix's ghost rows on several GPUs)
  int32_t ext_len = 0;
  std::vector<ConCache> con;
  std::vector<double> y_all;  // k*k host copy of every iteration's y
  std::vector<double> H;      // (k+1) x k column-major Hessenberg (host)
  std::vector<QuadCon> last_con;  // reduced class-form constraints of the last constrained step
  int last_con_p = 0;             // its p (0: none)
  int steps = 0;
  int n_iter_y = 0;           // iterations with a stored y
  bool broke_at_start = false;
};

// ------------------------------------------------------------------------------------------------
// helpers
// ------------------------------------------------------------------------------------------------
static bool fixed_grid(const spis_context* c) { return c->dist_on(); }

// C16 (SPIS_OPT_COL16): 1 = when val/col exceed the 256 MB Infinity Cache (C5 dual 470 vs
// 494 us: HBM-bound, 2 B less per nonzero pays; C3, cache-resident: 39.5 vs 37.6 us, the
// 16-bit loads and the decode cost more than the bytes saved), 2 = always, 0 = never
bool spis_matrix::use_col16() const {
  if (col16_d == nullptr || ctx->col16 == 0) return false;
  return ctx->col16 == 2 || 12.0 * static_cast<double>(nnz) > 256.0 * 1024 * 1024;
}

// the solver's SpMV table: kDualCap row blocks, run by the pipelined kernels unless disabled
CsrView spis_matrix::dual_view() const {
  CsrView v{n_rows, indptr, indices, vals, blk_row_d, n_blk_d, false};
  int mode = ctx->spmv_pipe;
  // auto: the XCD-local walk while val/col fit the 256 MB Infinity Cache (C3 dual SpMV 42-43 vs
  // 44-45 us grid-stride), the grid-stride walk beyond (C5, 1.5 GB: 502 vs 574 us)
  // (the slab-ordered table wins at both sizes: C5 dual 485 vs 498 us grid-stride)
  if (mode == 5) mode = blk_slab_d != nullptr || 12.0 * static_cast<double>(nnz) <= 256.0 * 1024 * 1024 ? 2 : 1;
  if (mode == 7) mode = 2;  // XCD-local walk on the contiguous table (A/B against the slab order)
  else if (mode == 2 && blk_slab_d != nullptr) {
    v.blk_meta = blk_slab_d;
    v.n_blk = n_blk;
    v.walk = 2;
    if (use_col16()) {
      v.col16 = col16_d;
      v.blk_base = base_slab_d;
    }
    return v;
  }
  if (mode > 0) {
    v.blk_meta = blk_meta_d;
    v.n_blk = n_blk;
    v.walk = (mode & 1) == 0 ? 1 : 0;
    if (use_col16()) {
      v.col16 = col16_d;
      v.blk_base = base_nat_d;
    }
  }
  return v;
}

// ---- live kernel timing ------------------------------------------------------------------------
static hipEvent_t prof_event(spis_context* c) {
  if (!c->ev_free.empty()) {
    hipEvent_t e = c->ev_free.back();
    c->ev_free.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);  // timing only: no L2 flush
  return e;
}

// Sampled live timing: a start/stop event pair carried by the timed launches themselves
// (hipExtLaunchKernel), so sampling adds no marker packets to the stream.
struct ProfEv {
  spis_context* c;
  int kind;
  hipEvent_t a = nullptr, b = nullptr;
  ProfEv(spis_context* c_, int kind_) : c(c_), kind(kind_) {
    if (c->prof && ((c->prof_iter + c->prof_phase) % c->prof_period) == 0) {
      a = prof_event(c);
      b = prof_event(c);
    }
  }
  bool on() const { return a != nullptr; }
  LaunchEv first() const { LaunchEv e; e.start = a; return e; }
  LaunchEv last() const { LaunchEv e; e.stop = b; return e; }
  LaunchEv both() const { LaunchEv e; e.start = a; e.stop = b; return e; }
  ~ProfEv() {
    if (a) c->ev_pending.push_back({kind, a, b});
  }
};

// after a stream synchronisation: fold completed event pairs into the totals
static void prof_drain(spis_context* c) {
  size_t keep = 0;
  for (size_t i = 0; i < c->ev_pending.size(); ++i) {
    auto& p = c->ev_pending[i];
    if (hipEventQuery(p.b) != hipSuccess) {  // still in flight (speculative Arnoldi step)
      c->ev_pending[keep++] = p;
      continue;
    }
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
      c->prof_ms[p.kind] += ms;
      c->prof_n[p.kind] += 1;
    }
    c->ev_free.push_back(p.a);
    c->ev_free.push_back(p.b);
  }
  c->ev_pending.resize(keep);
}

// several ranks through the host callback (spis_comm_init_host): the stream drained, the
// operands staged through host memory, the callback does the collective (tests: torch.distributed
// over gloo); ordering across ranks is the callers', exactly as for RCCL
static int host_allreduce(spis_context* c, double* buf, int64_t count, hipStream_t st) {
  HIP_TRY(hipStreamSynchronize(st));
  c->host_stage.resize(static_cast<size_t>(count));
  HIP_TRY(hipMemcpy(c->host_stage.data(), buf, sizeof(double) * count, hipMemcpyDeviceToHost));
  if (c->host_coll(c->host_user, SPIS_COLL_ALLREDUCE, c->host_stage.data(), count, 0, nullptr, nullptr, nullptr,
                   nullptr) != 0)
    return fail(SPIS_ERR_CALLBACK, "host all-reduce failed");
  HIP_TRY(hipMemcpy(buf, c->host_stage.data(), sizeof(double) * count, hipMemcpyHostToDevice));
  return SPIS_OK;
}

// send[soff[i] * w ...] to nbr[i] and recv[roff[i] * w ...] from it, w doubles per halo entry;
// the receive side is contiguous (ghost rows in neighbour order)
static int host_exchange(spis_context* c, const spis_matrix* M, const double* send_dev, double* recv_dev, int w,
                         hipStream_t st) {
  HIP_TRY(hipStreamSynchronize(st));
  const int nn = static_cast<int>(M->nbr.size());
  const int64_t ns = static_cast<int64_t>(M->n_send) * w, nr = static_cast<int64_t>(M->n_ghost) * w;
  c->host_stage.resize(static_cast<size_t>(ns + nr));
  std::vector<int64_t> sc(nn), rc(nn);
  for (int i = 0; i < nn; ++i) {
    sc[i] = static_cast<int64_t>(M->scnt[i]) * w;
    rc[i] = static_cast<int64_t>(M->rcnt[i]) * w;
  }
  if (ns > 0) HIP_TRY(hipMemcpy(c->host_stage.data(), send_dev, sizeof(double) * ns, hipMemcpyDeviceToHost));
  if (c->host_coll(c->host_user, SPIS_COLL_EXCHANGE, c->host_stage.data(), ns, nn, M->nbr.data(), sc.data(),
                   rc.data(), c->host_stage.data() + ns) != 0)
    return fail(SPIS_ERR_CALLBACK, "host halo exchange failed");
  if (nr > 0) HIP_TRY(hipMemcpy(recv_dev, c->host_stage.data() + ns, sizeof(double) * nr, hipMemcpyHostToDevice));
  return SPIS_OK;
}

// a one-rank communicator's sum is the identity: no collective launch (halo exchanges still run:
// a one-rank operator may declare ghosts it receives from itself)
static int allreduce_on(spis_context* c, double* buf, int64_t count, hipStream_t st) {
  if (!c->dist_on() || count <= 0 || c->nranks == 1) return SPIS_OK;
  if (c->host_coll) return host_allreduce(c, buf, count, st);
  NCCL_TRY(ncclAllReduce(buf, buf, count, ncclDouble, ncclSum, c->comm, st));
  return SPIS_OK;
}

static int allreduce(spis_context* c, double* buf, int64_t count) { return allreduce_on(c, buf, count, c->stream); }

static int exchange(spis_context* c, const spis_matrix* M, double* x) {
  if (!c->dist_on() || M->nbr.empty()) return SPIS_OK;
  HIP_TRY(launch_gather(M->n_send, M->send_idx, x, M->send_buf, c->stream));
  if (c->host_coll) return host_exchange(c, M, M->send_buf, x + M->n_rows, 1, c->stream);
  NCCL_TRY(ncclGroupStart());
  for (size_t i = 0; i < M->nbr.size(); ++i) {
    if (M->scnt[i] > 0)
      NCCL_TRY(ncclSend(M->send_buf + M->soff[i], M->scnt[i], ncclDouble, M->nbr[i], c->comm, c->stream));
    if (M->rcnt[i] > 0)
      NCCL_TRY(ncclRecv(x + M->n_rows + M->roff[i], M->rcnt[i], ncclDouble, M->nbr[i], c->comm, c->stream));
  }
  NCCL_TRY(ncclGroupEnd());
  return SPIS_OK;
}

// several GPUs: the ghost rows of a row-major (n_rows + n_ghost, cols) array (Ut of a constraint
// reduction) from their owners, through M's halo plan (one grouped send/recv of whole rows)
static int exchange_rows(spis_context* c, const spis_matrix* M, double* U, int cols, hipStream_t st) {
  if (!c->dist_on() || M->nbr.empty()) return SPIS_OK;
  const size_t need = static_cast<size_t>(std::max<int64_t>(M->n_send, 1)) * cols;
  if (c->ut_send_len < need) {
    if (c->ut_send) HIP_TRY(hipFree(c->ut_send));
    c->ut_send = nullptr;
    c->ut_send_len = 0;
    HIP_TRY(hipMalloc(&c->ut_send, sizeof(double) * need));
    c->ut_send_len = need;
  }
  HIP_TRY(launch_gather_rows(M->n_send, cols, M->send_idx, U, c->ut_send, st));
  if (c->host_coll) return host_exchange(c, M, c->ut_send, U + static_cast<size_t>(M->n_rows) * cols, cols, st);
  NCCL_TRY(ncclGroupStart());
  for (size_t i = 0; i < M->nbr.size(); ++i) {
    if (M->scnt[i] > 0)
      NCCL_TRY(ncclSend(c->ut_send + static_cast<size_t>(M->soff[i]) * cols, static_cast<size_t>(M->scnt[i]) * cols,
                        ncclDouble, M->nbr[i], c->comm, st));
    if (M->rcnt[i] > 0)
      NCCL_TRY(ncclRecv(U + static_cast<size_t>(M->n_rows + M->roff[i]) * cols, static_cast<size_t>(M->rcnt[i]) * cols,
                        ncclDouble, M->nbr[i], c->comm, st));
  }
  NCCL_TRY(ncclGroupEnd());
  return SPIS_OK;
}

static int ensure_pinned(spis_context* c, size_t len) {
  if (c->pinned_len >= len) return SPIS_OK;
  if (c->pinned) {
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipHostFree(c->pinned));
  }
  c->pinned = nullptr;
  // fine-grained (coherent) and mapped: kernels store h columns / residual partials straight
  // into host memory, uncached on the GPU side, so a device-scope event release suffices
  HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&c->pinned), len * sizeof(double),
                        hipHostMallocMapped | hipHostMallocCoherent));
  std::memset(c->pinned, 0, len * sizeof(double));  // completion flags start below any seq
  void* dp = nullptr;
  HIP_TRY(hipHostGetDevicePointer(&dp, c->pinned, 0));
  c->pinned_dev = static_cast<double*>(dp);
  c->pinned_len = len;
  return SPIS_OK;
}

// spin on an event (the solver's one host wait per iteration: lower wake-up latency than a
// blocking synchronize; the host thread has nothing else to do meanwhile)
static int wait_event(hipEvent_t e) {
  for (;;) {
    const hipError_t r = hipEventQuery(e);
    if (r == hipSuccess) return SPIS_OK;
    if (r != hipErrorNotReady) return fail(SPIS_ERR_HIP, "hipEventQuery: %s", hipGetErrorString(r));
    __builtin_ia32_pause();
  }
}

// y = M x where x is a local vector (owned part valid); ghosts gathered through scratch if needed
static int spmv_local(spis_context* c, spis_workspace* ws, const spis_matrix* M, const double* x,
                      double* y, hipStream_t st = nullptr) {  // st: one GPU only (several: c->stream)
  const int g = spmv_grid(M->view(), fixed_grid(c));
  if (c->dist_on() && M->n_ghost > 0) {
    if (!ws->ext || ws->ext_len < M->n_rows + M->n_ghost) {
      if (ws->ext) HIP_TRY(hipFree(ws->ext));
      ws->ext_len = static_cast<int32_t>(M->n_rows + M->n_ghost);
      HIP_TRY(hipMalloc(&ws->ext, sizeof(double) * ws->ext_len));
    }
    HIP_TRY(launch_copy(M->n_rows, x, ws->ext, c->stream));
    ST_TRY(exchange(c, M, ws->ext));
    HIP_TRY(launch_spmv(M->view(), kEpiPlain, ws->ext, y, nullptr, nullptr, g, c->stream));
    return SPIS_OK;
  }
  // one GPU: the pipelined kernel on the matrix's K1p table (rows bit-identical to K1's)
  // (else K1 on the row-block table)
  const CsrView pv = M->dual_view().blk_meta != nullptr ? M->dual_view() : M->view();
  HIP_TRY(launch_spmv(pv, kEpiPlain, x, y, nullptr, nullptr, spmv_grid(pv, false), st != nullptr ? st : c->stream));
  return SPIS_OK;
}

// G (nu x nv, host row-major) = U^T V, tiled by kGramMaxVec-vector panels; all-reduced
static int gram(spis_context* c, int64_t n, int nu, const double* const* U, int nv,
                const double* const* V, double* G_host) {
  const int T = 64;
  const int grid = fixed_grid(c) ? 512 : static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(512, (n + kGramChunk - 1) / kGramChunk)));
  const size_t need = static_cast<size_t>(grid) * T * T;
  if (c->gram_part_len < need) {
    if (c->gram_part) HIP_TRY(hipFree(c->gram_part));
    HIP_TRY(hipMalloc(&c->gram_part, need * sizeof(double)));
    c->gram_part_len = need;
  }
  if (!c->gram_G) HIP_TRY(hipMalloc(&c->gram_G, sizeof(double) * T * T));
  if (!c->gram_ptrs) HIP_TRY(hipMalloc(reinterpret_cast<void**>(&c->gram_ptrs), sizeof(double*) * 2 * kGramMaxVec));
  if (!c->gram_pinned)
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&c->gram_pinned), sizeof(double) * (T * T + 2 * kGramMaxVec),
                          hipHostMallocDefault));
  for (int u0 = 0; u0 < nu; u0 += T) {
    const int tu = std::min(T, nu - u0);
    for (int v0 = 0; v0 < nv; v0 += T) {
      const int tv = std::min(T, nv - v0);
      const double** hp = reinterpret_cast<const double**>(c->gram_pinned + T * T);
      for (int a = 0; a < tu; ++a) hp[a] = U[u0 + a];
      for (int b = 0; b < tv; ++b) hp[kGramMaxVec + b] = V[v0 + b];
      HIP_TRY(hipMemcpyAsync(c->gram_ptrs, hp, sizeof(double*) * 2 * kGramMaxVec, hipMemcpyHostToDevice, c->stream));
      HIP_TRY(launch_gram(n, tu, c->gram_ptrs, tv, c->gram_ptrs + kGramMaxVec, c->gram_part, grid, c->gram_G, c->stream));
      ST_TRY(allreduce(c, c->gram_G, static_cast<int64_t>(tu) * tv));
      HIP_TRY(hipMemcpyAsync(c->gram_pinned, c->gram_G, sizeof(double) * tu * tv, hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      for (int a = 0; a < tu; ++a)
        for (int b = 0; b < tv; ++b)
          G_host[static_cast<size_t>(u0 + a) * nv + v0 + b] = c->gram_pinned[static_cast<size_t>(a) * tv + b];
    }
  }
  return SPIS_OK;
}

// ------------------------------------------------------------------------------------------------
// library / context
// ------------------------------------------------------------------------------------------------
extern "C" int spis_abi_version(void) { return SPIS_ABI_VERSION; }
extern "C" const char* spis_last_error(void) { return g_last_error.c_str(); }

extern "C" int spis_device_count(int32_t* count) {
  ABI_GUARD({
    if (!count) return fail(SPIS_ERR_ARG, "null count");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *count = n;
    return SPIS_OK;
  })
}

extern "C" int spis_context_create(int32_t device, spis_context** out) {
  ABI_GUARD({
    if (!out) return fail(SPIS_ERR_ARG, "null out");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
      return fail(SPIS_ERR_HIP, "no HIP device visible (libspis needs an MI355X)");
    if (device < 0 || device >= n) return fail(SPIS_ERR_ARG, "device %d out of range [0,%d)", device, n);
    HIP_TRY(hipSetDevice(device));
    std::unique_ptr<spis_context> c(new spis_context());
    c->device = device;
    HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking));
    HIP_TRY(hipMalloc(&c->gemv_flag, 16));
    HIP_TRY(hipMemset(c->gemv_flag, 0, 16));
    const int np = std::max(kSpmvGrid, kRedGrid);
    HIP_TRY(hipMalloc(&c->partA, sizeof(double) * np));
    HIP_TRY(hipMalloc(&c->partB, sizeof(double) * np));
    // partR lives behind the one-reduce MGS's dot vector (icwy_d): on several GPUs the residual
    // partials then ride in the same all-reduce as the dots (arnoldi_post_icwy)
    HIP_TRY(hipMalloc(&c->dscal, sizeof(double) * (kMaxK + 8)));
    HIP_TRY(hipMalloc(&c->cgs_part, sizeof(double) * kCgsMax * kRedGrid));
    HIP_TRY(hipMalloc(&c->cgs_c, sizeof(double) * 2 * kCgsMax));
    HIP_TRY(hipMalloc(&c->icwy_part, sizeof(double) * 2 * kCgsMax * kRedGrid));
    HIP_TRY(hipMalloc(&c->icwy_d, sizeof(double) * (kIcwyROff + np)));
    HIP_TRY(hipMalloc(&c->icwy_slots, sizeof(unsigned long long) * kIcwySlotWords));
    HIP_TRY(hipMemset(c->icwy_slots, 0, sizeof(unsigned long long) * kIcwySlotWords));
    HIP_TRY(hipMemset(c->icwy_d, 0, sizeof(double) * (kIcwyROff + np)));
    c->partR = c->icwy_d + kIcwyROff;
    HIP_TRY(hipMalloc(&c->icwy_G, sizeof(double) * kCgsMax * kCgsMax));
    HIP_TRY(hipMemset(c->icwy_G, 0, sizeof(double) * kCgsMax * kCgsMax));
    HIP_TRY(hipMalloc(&c->chain_gran, sizeof(unsigned long long) * kChainGranLag));
    HIP_TRY(hipMemset(c->chain_gran, 0, sizeof(unsigned long long) * kChainGranLag));
    HIP_TRY(hipMalloc(&c->chain_gsub, sizeof(double) * kChainGsub));
    HIP_TRY(hipMemset(c->chain_gsub, 0, sizeof(double) * kChainGsub));
    HIP_TRY(hipMalloc(&c->chain_epoch, 16));
    HIP_TRY(hipMemset(c->chain_epoch, 0, 16));
    {  // the tag base starts at 1: K2q's E_0 carries tag base + 0, which must never equal the 0
       // tags of the zero-initialised exchange slots
      const unsigned one = 1;
      HIP_TRY(hipMemcpy(c->chain_epoch, &one, sizeof one, hipMemcpyHostToDevice));
    }
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&c->chain_err), 16, hipHostMallocMapped));
    *c->chain_err = 0;
    HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->chain_err_dev), c->chain_err, 0));
    ST_TRY(ensure_pinned(c.get(), 4 * kMaxK + 2 * np));
    // pipeline events only order host reads of the coherent pinned slots: device-scope release
    // (a system-scope one writes back and invalidates L2 at every iteration, ~8 us each);
    // (SPIS_EVENT_MODE below selects the scope for measurements)
    // SPIS_EVENT_MODE: 0 system-scope release, 1 device scope (default), 2 no release fence
    auto env_flag = [](const char* name, bool dflt) {
      const char* v = std::getenv(name);
      return v == nullptr ? dflt : std::atoi(v) != 0;
    };
    c->gram_inc = env_flag("SPIS_GRAM_INC", true);
    c->x0_zero_test = env_flag("SPIS_X0_ZERO_TEST", true);
    c->transpose_pipe = env_flag("SPIS_TRANSPOSE_PIPE", true);
    {  // write-through output stores, a mask (kernels.hip g_store_wt; process-wide): from
       // SPIS_STORE_WT once, at the process's first context (spis_set_option changes it later)
      static const bool once = [] {
        const char* e = std::getenv("SPIS_STORE_WT");
        set_store_wt(e ? std::atoi(e) : 1);
        return true;
      }();
      (void)once;
    }
    c->k2w_fold = env_flag("SPIS_K2W_FOLD", true);
    c->k2w_onepass = env_flag("SPIS_K2W_ONEPASS", true);
    if (const char* v = std::getenv("SPIS_K2W_TW")) c->k2w_tw = std::atoi(v);
    if (const char* v = std::getenv("SPIS_K2W_SMALL_N")) c->k2w_small_n = std::atoll(v);
    const char* se = std::getenv("SPIS_EVENT_MODE");
    const int mode = se ? std::atoi(se) : 1;
    const unsigned evf = hipEventDisableTiming | (mode == 1 ? hipEventReleaseToDevice : 0u) |
                         (mode == 2 ? hipEventDisableSystemFence : 0u);
    HIP_TRY(hipEventCreateWithFlags(&c->ev_arn, evf));
    HIP_TRY(hipEventCreateWithFlags(&c->ev_upd[0], evf));
    HIP_TRY(hipEventCreateWithFlags(&c->ev_upd[1], evf));
    HIP_TRY(hipEventCreateWithFlags(&c->ev_gram, hipEventDisableTiming));  // system scope: host reads
    HIP_TRY(hipEventCreateWithFlags(&c->ev_xd, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&c->ev_xd2, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&c->ev_side, hipEventDisableTiming));
    *out = c.release();
    return SPIS_OK;
  })
}

static void release_cache(spis_context* c) {
  for (auto& kv : c->free_blocks) (void)hipFree(kv.second);
  c->free_blocks.clear();
  c->cached_bytes = 0;
}

static void free_workspace(spis_workspace* ws) {
  (void)hipFree(ws->Q);
  if (ws->sep_z) (void)hipFree(ws->Zb);
  (void)hipFree(ws->w);
  (void)hipFree(ws->xj);
  (void)hipFree(ws->xj2);
  (void)hipFree(ws->r0);
  (void)hipFree(ws->x0);
  (void)hipFree(ws->ydev);
  if (ws->ext) (void)hipFree(ws->ext);
  if (ws->Ut) (void)hipFree(ws->Ut);
  for (auto& cc : ws->con) {
    if (cc.MZ) (void)hipFree(cc.MZ);
    if (cc.Mx0) (void)hipFree(cc.Mx0);
  }
  delete ws;
}

extern "C" int spis_context_destroy(spis_context* c) {
  ABI_GUARD({
    if (!c) return SPIS_OK;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    for (auto* ws : c->pool) free_workspace(ws);
    release_cache(c);
    for (auto& kv : c->live_blocks) (void)hipFree(kv.first);
    (void)hipFree(c->partA);
    (void)hipFree(c->partB);
    (void)hipFree(c->dscal);
    (void)hipFree(c->cgs_part);
    (void)hipFree(c->cgs_c);
    (void)hipFree(c->icwy_part);
    (void)hipFree(c->icwy_d);
    (void)hipFree(c->icwy_slots);
    (void)hipFree(c->icwy_G);
    (void)hipFree(c->ut_send);
    (void)hipFree(c->chain_gran);
    (void)hipFree(c->chain_gsub);
    (void)hipFree(c->gemv_flag);
    (void)hipFree(c->chain_epoch);
    if (c->chain_err) (void)hipHostFree(c->chain_err);
    if (c->x0_flag) (void)hipFree(c->x0_flag);
    if (c->gram_part) (void)hipFree(c->gram_part);
    if (c->gram_G) (void)hipFree(c->gram_G);
    if (c->cg_part) (void)hipFree(c->cg_part);
    if (c->cg_G) (void)hipFree(c->cg_G);
    if (c->cg_vpart) (void)hipFree(c->cg_vpart);
    if (c->inc_u) (void)hipFree(c->inc_u);
    if (c->inc_part) (void)hipFree(c->inc_part);
    if (c->inc_res) (void)hipFree(c->inc_res);
    if (c->gram_ptrs) (void)hipFree(c->gram_ptrs);
    if (c->pinned) (void)hipHostFree(c->pinned);
    if (c->gram_pinned) (void)hipHostFree(c->gram_pinned);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    for (auto& p : c->ev_pending) {
      (void)hipEventDestroy(p.a);
      (void)hipEventDestroy(p.b);
    }
    for (auto e : c->ev_free) (void)hipEventDestroy(e);
    (void)hipStreamSynchronize(c->stream2);
    for (auto e : {c->ev_arn, c->ev_upd[0], c->ev_upd[1], c->ev_gram, c->ev_xd, c->ev_xd2, c->ev_side})
      if (e) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(c->stream);
    (void)hipStreamDestroy(c->stream2);
    if (c->con_pinned) (void)hipHostFree(c->con_pinned);
    delete c;
    return SPIS_OK;
  })
}

extern "C" int spis_context_synchronize(spis_context* c) {
  ABI_GUARD({
    if (!c) return fail(SPIS_ERR_ARG, "null context");
    HIP_TRY(hipStreamSynchronize(c->stream));
    return SPIS_OK;
  })
}

extern "C" int spis_context_stream(spis_context* c, void** s) {
  if (!c || !s) return fail(SPIS_ERR_ARG, "null argument");
  *s = c->stream;
  return SPIS_OK;
}

extern "C" int spis_set_option(spis_context* c, int32_t option, int64_t value) {
  ABI_GUARD({
    if (!c) return fail(SPIS_ERR_ARG, "null context");
    HIP_TRY(hipStreamSynchronize(c->stream));
    switch (option) {
      case SPIS_OPT_FUSE_SPMV: c->fuse_spmv = value != 0; return SPIS_OK;
      case SPIS_OPT_CON_GRAM:
        if (value < 0 || value > 3) return fail(SPIS_ERR_ARG, "con gram %lld: 0 .. 3", (long long)value);
        c->con_gram = static_cast<int>(value);
        return SPIS_OK;
      case SPIS_OPT_MGS_CHAIN:
        if (value < 0 || value > 4) return fail(SPIS_ERR_ARG, "mgs chain %lld: 0 .. 4", (long long)value);
        c->mgs_chain = static_cast<int>(value);
        return SPIS_OK;
      case SPIS_OPT_NT_BASIS:
        if (value < 0 || value > 2) return fail(SPIS_ERR_ARG, "nt basis %lld: 0, 1 or 2", (long long)value);
        c->nt_basis = static_cast<int>(value);
        return SPIS_OK;
      case SPIS_OPT_SPMV_PIPE:
        if (value != 0 && value != 1 && value != 2 && value != 5 && value != 7)
          return fail(SPIS_ERR_ARG, "spmv pipe %lld: 0, 1, 2, 5 or 7", (long long)value);
        c->spmv_pipe = static_cast<int>(value);
        return SPIS_OK;
      case SPIS_OPT_COL16:
        if (value < 0 || value > 2) return fail(SPIS_ERR_ARG, "col16 %lld: 0, 1 or 2", (long long)value);
        c->col16 = static_cast<int>(value);
        return SPIS_OK;
      case SPIS_OPT_ORTHOG:
        if (value != 0 && value != 1) return fail(SPIS_ERR_ARG, "orthogonalisation %lld: 0 = MGS, 1 = CGS2", (long long)value);
        c->cgs2 = value == 1;
        return SPIS_OK;
      case SPIS_OPT_DIST_MGS:
        if (value != 0 && value != 1) return fail(SPIS_ERR_ARG, "dist_mgs %lld: 0 or 1", (long long)value);
        c->dist_mgs = static_cast<int>(value);
        return SPIS_OK;
      case SPIS_OPT_SLAB_KEY:
        if (value != 0 && value != 1) return fail(SPIS_ERR_ARG, "slab_key %lld: 0 or 1", (long long)value);
        c->slab_key = static_cast<int>(value);
        return SPIS_OK;
      case SPIS_OPT_GRAM_INC:
      case SPIS_OPT_X0_ZERO_TEST:
      case SPIS_OPT_TRANSPOSE_PIPE:
        if (value != 0 && value != 1) return fail(SPIS_ERR_ARG, "option %d takes 0 or 1", option);
        (option == SPIS_OPT_GRAM_INC ? c->gram_inc : option == SPIS_OPT_X0_ZERO_TEST ? c->x0_zero_test
                                                                                      : c->transpose_pipe) = value == 1;
        return SPIS_OK;
      case SPIS_OPT_K2W_SMALL_N:
        if (value < -1) return fail(SPIS_ERR_ARG, "k2w small n %lld: >= -1", (long long)value);
        c->k2w_small_n = value;
        return SPIS_OK;
      case SPIS_OPT_K2W_TW:
        if (value < -1 || value > kMaxK) return fail(SPIS_ERR_ARG, "k2w tw %lld: -1 .. %d", (long long)value, kMaxK);
        c->k2w_tw = static_cast<int>(value);
        return SPIS_OK;
      case SPIS_OPT_K2W_FOLD:
      case SPIS_OPT_K2W_ONEPASS:
        if (value != 0 && value != 1) return fail(SPIS_ERR_ARG, "option %d takes 0 or 1", option);
        (option == SPIS_OPT_K2W_FOLD ? c->k2w_fold : c->k2w_onepass) = value == 1;
        return SPIS_OK;
      case SPIS_OPT_STORE_WT:
        if (value < 0 || value > 15) return fail(SPIS_ERR_ARG, "store_wt %lld: a mask 0 .. 15", (long long)value);
        HIP_TRY(hipDeviceSynchronize());  // process-wide: no kernel of any context in flight under the old form
        set_store_wt(static_cast<int>(value));
        return SPIS_OK;
      default: return fail(SPIS_ERR_ARG, "unknown option %d", option);
    }
  })
}

extern "C" int spis_profile_enable(spis_context* c, int32_t on) {
  ABI_GUARD({
    if (!c) return fail(SPIS_ERR_ARG, "null context");
    HIP_TRY(hipStreamSynchronize(c->stream));
    prof_drain(c);
    c->prof = on > 0;
    c->prof_period = on > 0 ? on : 1;
    c->prof_iter = 0;
    c->prof_phase = 0;
    for (int i = 0; i < SPIS_PROF_KINDS; ++i) {
      c->prof_ms[i] = 0.0;
      c->prof_n[i] = 0;
    }
    return SPIS_OK;
  })
}

extern "C" int spis_profile_read(spis_context* c, double ms_out[SPIS_PROF_KINDS], int64_t count_out[SPIS_PROF_KINDS]) {
  ABI_GUARD({
    if (!c || !ms_out || !count_out) return fail(SPIS_ERR_ARG, "null argument");
    HIP_TRY(hipStreamSynchronize(c->stream));
    prof_drain(c);
    for (int i = 0; i < SPIS_PROF_KINDS; ++i) {
      ms_out[i] = c->prof_ms[i];
      count_out[i] = c->prof_n[i];
    }
    return SPIS_OK;
  })
}

// Standalone timing of the solver's SpMV launches on the solver's own table and kernel choice
// (dual_view, spmv_grid), for the bench's roofline: kind 0 = the Arnoldi SpMV (w = A z, q0.w
// partials, solvers.py:191), kind 1 = the fused dual (||A x - b||^2 of x_j with A z of z_{j+2},
// :290 + :191).  cold = 1: a 1 GiB streaming read before every timed launch evicts L2 and the
// 256 MB Infinity Cache, so the matrix and the vectors come from HBM; cold = 0: back to back.
// us_out = mean launch duration over reps (the launch's own start/stop events).
extern "C" int spis_spmv_bench(spis_context* c, spis_matrix* A, int32_t kind, int32_t cold, int32_t reps,
                               double* us_out) {
  ABI_GUARD({
    if (!c || !A || !us_out || reps < 1 || kind < 0 || kind > 1) return fail(SPIS_ERR_ARG, "bad argument");
    if (A->ctx != c || A->n_rows != A->n_cols || c->dist_on()) return fail(SPIS_ERR_ARG, "single-GPU square matrix only");
    HIP_TRY(hipSetDevice(c->device));
    const int64_t n = A->n_rows;
    const int64_t pn = (n + 63) / 64 * 64;
    const int64_t big = int64_t(1) << 27;  // 1 GiB of doubles
    double* buf = nullptr;
    HIP_TRY(hipMalloc(&buf, sizeof(double) * (5 * pn + 2 * kSpmvGrid + 8 + (cold ? big : 0))));
    std::unique_ptr<double, void (*)(double*)> guard(buf, [](double* p) { (void)hipFree(p); });
    double *x = buf, *z = buf + pn, *bb = buf + 2 * pn, *w = buf + 3 * pn, *q0 = buf + 4 * pn;
    double *p1 = buf + 5 * pn, *p2 = p1 + kSpmvGrid, *sink = p2 + kSpmvGrid, *fl = sink + 8;
    {
      std::vector<double> h(static_cast<size_t>(pn));
      for (int64_t i = 0; i < pn; ++i) h[i] = i < n ? 1e-3 * static_cast<double>((i * 104729) % 997) - 0.4 : 0.0;
      for (double* d : {x, z, bb, q0}) HIP_TRY(hipMemcpy(d, h.data(), sizeof(double) * pn, hipMemcpyHostToDevice));
    }
    if (cold) HIP_TRY(hipMemsetAsync(fl, 0, sizeof(double) * big, c->stream));
    hipEvent_t e0, e1;
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    const CsrView v = A->dual_view();
    const int g = spmv_grid(v, false);
    double tot = 0.0;
    int st = SPIS_OK;
    for (int r = -2; r < reps && st == SPIS_OK; ++r) {
      if (cold) {
        hipError_t e = launch_stream_read(big, fl, sink, c->stream);
        if (e != hipSuccess) { st = fail(SPIS_ERR_HIP, "flush: %s", hipGetErrorString(e)); break; }
      }
      const LaunchEv le{e0, e1};
      const hipError_t e = kind == 0 ? launch_spmv(v, kEpiDot, z, w, q0, p2, g, c->stream, &le)
                                     : launch_spmv_dual(v, x, bb, p1, z, w, q0, p2, g, c->stream, &le);
      if (e != hipSuccess) { st = fail(SPIS_ERR_HIP, "spmv: %s", hipGetErrorString(e)); break; }
      if (hipEventSynchronize(e1) != hipSuccess) { st = fail(SPIS_ERR_HIP, "event"); break; }
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, e0, e1) != hipSuccess) { st = fail(SPIS_ERR_HIP, "elapsed"); break; }
      if (r >= 0) tot += ms;
    }
    (void)hipStreamSynchronize(c->stream);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (st != SPIS_OK) return st;
    *us_out = 1e3 * tot / reps;
    return SPIS_OK;
  })
}

// ------------------------------------------------------------------------------------------------
// RCCL
// ------------------------------------------------------------------------------------------------
extern "C" int spis_comm_unique_id(uint8_t id_out[128]) {
  ABI_GUARD({
    if (!id_out) return fail(SPIS_ERR_ARG, "null id");
    ncclUniqueId id;
    NCCL_TRY(ncclGetUniqueId(&id));
    std::memcpy(id_out, id.internal, 128);
    return SPIS_OK;
  })
}

extern "C" int spis_comm_init(spis_context* c, int32_t nranks, int32_t rank, const uint8_t id[128]) {
  ABI_GUARD({
    if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return fail(SPIS_ERR_ARG, "bad comm args");
    if (c->dist_on()) return fail(SPIS_ERR_STATE, "context already has a communicator");
    // a 1-rank communicator is created too: it switches the context to the distributed code
    // path (fixed grids, all-reduces, halo exchanges — e.g. to itself), which tests use
    HIP_TRY(hipSetDevice(c->device));
    ncclUniqueId uid;
    std::memcpy(uid.internal, id, 128);
    NCCL_TRY(ncclCommInitRank(&c->comm, nranks, uid, rank));
    c->nranks = nranks;
    c->rank = rank;
    return SPIS_OK;
  })
}

extern "C" int spis_comm_init_host(spis_context* c, int32_t nranks, int32_t rank, spis_host_coll_fn fn, void* user) {
  ABI_GUARD({
    if (!c || !fn || nranks < 1 || rank < 0 || rank >= nranks) return fail(SPIS_ERR_ARG, "bad comm args");
    if (c->dist_on()) return fail(SPIS_ERR_STATE, "context already has a communicator");
    c->host_coll = fn;
    c->host_user = user;
    c->nranks = nranks;
    c->rank = rank;
    return SPIS_OK;
  })
}

extern "C" int spis_comm_allreduce_sum(spis_context* c, double* buf, int64_t count) {
  ABI_GUARD({
    if (!c) return fail(SPIS_ERR_ARG, "null context");
    ST_TRY(allreduce(c, buf, count));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return SPIS_OK;
  })
}

extern "C" int spis_comm_size(spis_context* c, int32_t* nranks_out, int32_t* transport_out) {
  ABI_GUARD({
    if (!c || !nranks_out || !transport_out) return fail(SPIS_ERR_ARG, "null argument");
    *nranks_out = 0;
    *transport_out = 0;
    if (c->comm) {
      int n = 0;
      NCCL_TRY(ncclCommCount(c->comm, &n));
      *nranks_out = n;
      *transport_out = 1;
    } else if (c->host_coll) {
      *nranks_out = c->nranks;
      *transport_out = 2;
    }
    return SPIS_OK;
  })
}

extern "C" int spis_comm_barrier(spis_context* c) {
  ABI_GUARD({
    if (!c) return fail(SPIS_ERR_ARG, "null context");
    ST_TRY(allreduce(c, c->dscal, 1));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return SPIS_OK;
  })
}

// ------------------------------------------------------------------------------------------------
// matrices
// ------------------------------------------------------------------------------------------------
// Row blocks: greedy walk over rows; a block closes before it would exceed kRowCap rows,
// kNnzCap nnz or kItemCap merge items (rows + nnz).  A row with more than kNnzCap entries forms
// a block of its own (workgroup-wide reduction in the kernel).  For bounded FE rows this is the
// merge-path partition snapped to row boundaries: every block carries ~kItemCap items.
static void build_row_blocks(int64_t n, const int32_t* rp, std::vector<int32_t>& blk, int32_t& n_long,
                             int64_t nnz_cap = kNnzCap, int64_t item_cap = kItemCap) {
  blk.clear();
  blk.push_back(0);
  n_long = 0;
  int64_t rows = 0, nnz = 0;
  for (int64_t r = 0; r < n; ++r) {
    const int64_t len = static_cast<int64_t>(rp[r + 1]) - rp[r];
    if (len > nnz_cap) {
      if (rows > 0) blk.push_back(static_cast<int32_t>(r));
      blk.push_back(static_cast<int32_t>(r + 1));
      ++n_long;
      rows = nnz = 0;
      continue;
    }
    if (rows > 0 && (rows + 1 > kRowCap || nnz + len > nnz_cap || rows + 1 + nnz + len > item_cap)) {
      blk.push_back(static_cast<int32_t>(r));
      rows = nnz = 0;
    }
    ++rows;
    nnz += len;
  }
  if (rows > 0) blk.push_back(static_cast<int32_t>(n));
}

extern "C" int spis_csr_upload(spis_context* c, int64_t n_rows, int64_t n_cols, int64_t nnz,
                               const int32_t* indptr, const int32_t* indices, const double* data,
                               const spis_halo_desc* halo, spis_matrix** out) {
  ABI_GUARD({
    if (!c || !out || !indptr || (nnz > 0 && (!indices || !data)))
      return fail(SPIS_ERR_ARG, "null argument");
    if (n_rows < 0 || n_cols < 0 || nnz < 0 || n_rows >= (int64_t(1) << 31) || nnz >= (int64_t(1) << 31))
      return fail(SPIS_ERR_ARG, "sizes out of int32 range");
    if (indptr[0] != 0 || indptr[n_rows] != nnz) return fail(SPIS_ERR_ARG, "indptr[0] != 0 or indptr[n] != nnz");
    const int32_t n_ghost = halo ? halo->n_ghost : 0;
    if (n_cols != n_rows + n_ghost)
      return fail(SPIS_ERR_ARG, "n_cols (%lld) must equal n_rows + n_ghost (%lld)", (long long)n_cols,
                  (long long)(n_rows + n_ghost));
    for (int64_t r = 0; r < n_rows; ++r)
      if (indptr[r + 1] < indptr[r]) return fail(SPIS_ERR_ARG, "indptr not monotone at row %lld", (long long)r);
    bool all_zero = true, all_finite = true;
    for (int64_t i = 0; i < nnz; ++i) {
      if (indices[i] < 0 || indices[i] >= n_cols)
        return fail(SPIS_ERR_ARG, "column index %d out of range at %lld", indices[i], (long long)i);
      if (data[i] != 0.0) all_zero = false;
      if (!std::isfinite(data[i])) all_finite = false;
    }
    HIP_TRY(hipSetDevice(c->device));
    std::unique_ptr<spis_matrix> M(new spis_matrix());
    static std::atomic<uint64_t> next_uid{1};
    M->uid = next_uid++;
    M->ctx = c;
    M->n_rows = n_rows;
    M->n_cols = n_cols;
    M->nnz = nnz;
    M->all_zero = all_zero;
    M->all_finite = all_finite;
    gram_split(n_rows, indptr, &M->gram_rows);
    std::vector<int32_t> blk;
    build_row_blocks(n_rows, indptr, blk, M->n_long);
    M->n_blk = static_cast<int32_t>(blk.size()) - 1;
    HIP_TRY(hipMalloc(&M->indptr, sizeof(int32_t) * (n_rows + 1)));
    HIP_TRY(hipMalloc(&M->indices, sizeof(int32_t) * std::max<int64_t>(nnz, 1)));
    HIP_TRY(hipMalloc(&M->vals, sizeof(double) * std::max<int64_t>(nnz, 1)));
    HIP_TRY(hipMalloc(&M->blk_row, sizeof(int32_t) * blk.size()));
    HIP_TRY(hipMemcpy(M->indptr, indptr, sizeof(int32_t) * (n_rows + 1), hipMemcpyHostToDevice));
    if (nnz > 0) {
      HIP_TRY(hipMemcpy(M->indices, indices, sizeof(int32_t) * nnz, hipMemcpyHostToDevice));
      HIP_TRY(hipMemcpy(M->vals, data, sizeof(double) * nnz, hipMemcpyHostToDevice));
    }
    HIP_TRY(hipMemcpy(M->blk_row, blk.data(), sizeof(int32_t) * blk.size(), hipMemcpyHostToDevice));
    {  // the pipelined kernels walk blk_row's blocks (kNnzCap = kPipeCap): in kbench at C3, 2048-nnz
       // blocks at 3 workgroups per CU vs 1024 at 5: dual SpMV 52.6 vs 56.4 us cold, 41.2 vs 41.1 warm
      static_assert(kNnzCap == kPipeCap && kItemCap == kPipeCap, "pipelined table = blk_row");
      std::vector<int2> meta(blk.size());
      for (size_t i = 0; i < blk.size(); ++i) meta[i] = make_int2(blk[i], indptr[blk[i]]);
      HIP_TRY(hipMalloc(&M->blk_meta_d, sizeof(int2) * meta.size()));
      HIP_TRY(hipMemcpy(M->blk_meta_d, meta.data(), sizeof(int2) * meta.size(), hipMemcpyHostToDevice));
      std::vector<int32_t> pairs;
      std::vector<int64_t> order;
      std::vector<uint8_t> lab;
      std::vector<double> key;
      std::vector<double>* kp = c->slab_key ? &key : nullptr;
      if (n_ghost == 0 && static_cast<int64_t>(blk.size()) > 16 && slab_labels(n_rows, indptr, indices, lab, kp) &&
          build_slab_order(indptr, lab, blk, pairs, &order, kp)) {
        HIP_TRY(hipMalloc(&M->blk_slab_d, sizeof(int32_t) * pairs.size()));
        HIP_TRY(hipMemcpy(M->blk_slab_d, pairs.data(), sizeof(int32_t) * pairs.size(), hipMemcpyHostToDevice));
      }
      // C16: the 16-bit column copy with each block's bases, in natural and in slab order
      std::vector<uint16_t> c16;
      std::vector<int32_t> bases;
      if (nnz > 0 && build_col16(indptr, indices, blk, c16, bases)) {
        HIP_TRY(hipMalloc(&M->col16_d, sizeof(uint16_t) * c16.size()));
        HIP_TRY(hipMemcpy(M->col16_d, c16.data(), sizeof(uint16_t) * c16.size(), hipMemcpyHostToDevice));
        HIP_TRY(hipMalloc(&M->base_nat_d, sizeof(int32_t) * bases.size()));
        HIP_TRY(hipMemcpy(M->base_nat_d, bases.data(), sizeof(int32_t) * bases.size(), hipMemcpyHostToDevice));
        if (M->blk_slab_d != nullptr) {
          std::vector<int32_t> bs(bases.size());
          for (size_t i = 0; i < order.size(); ++i)
            std::copy(bases.begin() + kCol16Bases * order[i], bases.begin() + kCol16Bases * (order[i] + 1),
                      bs.begin() + kCol16Bases * i);
          HIP_TRY(hipMalloc(&M->base_slab_d, sizeof(int32_t) * bs.size()));
          HIP_TRY(hipMemcpy(M->base_slab_d, bs.data(), sizeof(int32_t) * bs.size(), hipMemcpyHostToDevice));
        }
      }
    }
    {  // the fused residual + Arnoldi SpMV stages two product arrays: half-size blocks keep its LDS
      int32_t n_long_d = 0;  // at 16 KiB per workgroup (kbench: 52 vs 62 us at C3)
      build_row_blocks(n_rows, indptr, blk, n_long_d, kDualCap, kDualCap);
      M->n_blk_d = static_cast<int32_t>(blk.size()) - 1;
      HIP_TRY(hipMalloc(&M->blk_row_d, sizeof(int32_t) * blk.size()));
      HIP_TRY(hipMemcpy(M->blk_row_d, blk.data(), sizeof(int32_t) * blk.size(), hipMemcpyHostToDevice));
    }
    if (halo && halo->n_neighbors > 0) {
      M->n_ghost = n_ghost;
      const int nn = halo->n_neighbors;
      M->nbr.assign(halo->neighbors, halo->neighbors + nn);
      M->scnt.assign(halo->send_counts, halo->send_counts + nn);
      M->rcnt.assign(halo->recv_counts, halo->recv_counts + nn);
      M->soff.assign(nn, 0);
      M->roff.assign(nn, 0);
      int64_t so = 0, ro = 0;
      for (int i = 0; i < nn; ++i) {
        M->soff[i] = static_cast<int32_t>(so);
        M->roff[i] = static_cast<int32_t>(ro);
        so += M->scnt[i];
        ro += M->rcnt[i];
      }
      if (ro != n_ghost) return fail(SPIS_ERR_ARG, "sum(recv_counts)=%lld != n_ghost=%d", (long long)ro, n_ghost);
      for (int64_t i = 0; i < so; ++i)
        if (halo->send_idx[i] < 0 || halo->send_idx[i] >= n_rows) return fail(SPIS_ERR_ARG, "send_idx out of range");
      M->n_send = so;
      HIP_TRY(hipMalloc(&M->send_idx, sizeof(int32_t) * std::max<int64_t>(so, 1)));
      HIP_TRY(hipMalloc(&M->send_buf, sizeof(double) * std::max<int64_t>(so, 1)));
      if (so > 0) HIP_TRY(hipMemcpy(M->send_idx, halo->send_idx, sizeof(int32_t) * so, hipMemcpyHostToDevice));
    } else if (n_ghost > 0) {
      M->n_ghost = n_ghost;  // ghost columns without peers: caller fills them
    }
    *out = M.release();
    return SPIS_OK;
  })
}

extern "C" int spis_matrix_destroy(spis_matrix* M) {
  ABI_GUARD({
    if (!M) return SPIS_OK;
    (void)hipSetDevice(M->ctx->device);
    (void)hipStreamSynchronize(M->ctx->stream);
    (void)hipFree(M->indptr);
    (void)hipFree(M->indices);
    (void)hipFree(M->vals);
    (void)hipFree(M->blk_row);
    (void)hipFree(M->blk_row_d);
    (void)hipFree(M->blk_meta_d);
    (void)hipFree(M->col16_d);
    (void)hipFree(M->base_nat_d);
    (void)hipFree(M->base_slab_d);
    (void)hipFree(M->blk_slab_d);
    for (void* p : {static_cast<void*>(M->sym_col), static_cast<void*>(M->sym_val), static_cast<void*>(M->sym_mask)})
      if (p) (void)hipFree(p);
    if (M->send_idx) (void)hipFree(M->send_idx);
    if (M->send_buf) (void)hipFree(M->send_buf);
    delete M;
    return SPIS_OK;
  })
}

// ------------------------------------------------------------------------------------------------
// device ILU preconditioner (K8, sptrsv.h): the plan is built on the host once per factorisation
// (levels, solve order, blocks), uploaded, and every apply is two memsets + one launch
// ------------------------------------------------------------------------------------------------
struct DevTri {
  std::vector<void*> bufs;
  TriDev view{};
};

struct spis_ilu {
  spis_context* ctx = nullptr;
  int64_t n = 0;
  DevTri L, U;
  double* gran = nullptr;        // [2n] granules: y then v
  unsigned* ticket = nullptr;
  unsigned* err_host = nullptr;  // pinned, device-mapped: a bounded spin gave up
  unsigned* err_dev = nullptr;
  int64_t stats[8] = {0};
};

template <typename T>
static int upload_vec(DevTri& d, const std::vector<T>& v, const T** out) {
  *out = nullptr;
  if (v.empty()) return SPIS_OK;
  void* p = nullptr;
  HIP_TRY(hipMalloc(&p, sizeof(T) * v.size()));
  d.bufs.push_back(p);
  HIP_TRY(hipMemcpy(p, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice));
  *out = static_cast<const T*>(p);
  return SPIS_OK;
}

static int upload_tri(DevTri& d, const TriPlan& P) {
  ST_TRY(upload_vec(d, P.rowptr, &d.view.rowptr));
  ST_TRY(upload_vec(d, P.col, &d.view.col));
  ST_TRY(upload_vec(d, P.val, &d.view.val));
  ST_TRY(upload_vec(d, P.diag, &d.view.diag));
  ST_TRY(upload_vec(d, P.in_idx, &d.view.in_idx));
  ST_TRY(upload_vec(d, P.out_idx, &d.view.out_idx));
  ST_TRY(upload_vec(d, P.blk_row, &d.view.blk_row));
  ST_TRY(upload_vec(d, P.blk_step, &d.view.blk_step));
  ST_TRY(upload_vec(d, P.step_row, &d.view.step_row));
  ST_TRY(upload_vec(d, P.step_long, &d.view.step_long));
  ST_TRY(upload_vec(d, P.blk_ent, &d.view.blk_ent));
  ST_TRY(upload_vec(d, P.blk_long, &d.view.blk_long));
  d.view.nb = P.n_blocks();
  return SPIS_OK;
}

static void free_ilu(spis_ilu* P) {
  for (void* b : P->L.bufs) (void)hipFree(b);
  for (void* b : P->U.bufs) (void)hipFree(b);
  if (P->gran) (void)hipFree(P->gran);
  if (P->ticket) (void)hipFree(P->ticket);
  if (P->err_host) (void)hipHostFree(P->err_host);
  delete P;
}

static int ilu_enqueue(spis_ilu* P, const double* q, double* z, hipStream_t s) {
  HIP_TRY(launch_ilu_apply(P->n, P->L.view, P->U.view, q, P->gran, z, P->ticket, P->err_dev, s));
  return SPIS_OK;
}

static int ilu_check(spis_ilu* P) {  // after a synchronisation of the stream the applies ran on
  if (*reinterpret_cast<volatile unsigned*>(P->err_host) != 0) {
    *P->err_host = 0;
    return fail(SPIS_ERR_STATE, "device ILU apply: a triangular-solve wait timed out (values set to NaN)");
  }
  return SPIS_OK;
}

extern "C" int spis_ilu_create(spis_context* c, int64_t n, const int32_t* l_rowptr, const int32_t* l_col,
                               const double* l_val, const int32_t* u_rowptr, const int32_t* u_col,
                               const double* u_val, const int32_t* perm_r, const int32_t* perm_c,
                               spis_ilu** out) {
  ABI_GUARD({
    if (!c || !out || !l_rowptr || !u_rowptr || !perm_r || !perm_c) return fail(SPIS_ERR_ARG, "null argument");
    if (n < 0 || n >= (int64_t(1) << 30)) return fail(SPIS_ERR_ARG, "n out of range");
    if ((l_rowptr[n] > 0 && (!l_col || !l_val)) || (u_rowptr[n] > 0 && (!u_col || !u_val)))
      return fail(SPIS_ERR_ARG, "null factor arrays");
    TriPlan L, U;
    std::string err;
    if (!build_ilu_plans(n, l_rowptr, l_col, l_val, u_rowptr, u_col, u_val, perm_r, perm_c, &L, &U, &err))
      return fail(SPIS_ERR_ARG, "ILU factors: %s", err.c_str());
    HIP_TRY(hipSetDevice(c->device));
    std::unique_ptr<spis_ilu, void (*)(spis_ilu*)> P(new spis_ilu(), free_ilu);
    P->ctx = c;
    P->n = n;
    ST_TRY(upload_tri(P->L, L));
    ST_TRY(upload_tri(P->U, U));
    HIP_TRY(hipMalloc(&P->gran, sizeof(double) * std::max<int64_t>(2 * n, 2)));
    HIP_TRY(hipMalloc(&P->ticket, 16));
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&P->err_host), 16, hipHostMallocMapped));
    *P->err_host = 0;
    HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&P->err_dev), P->err_host, 0));
    const int64_t st[8] = {L.levels, U.levels, L.n_blocks(), U.n_blocks(),
                           static_cast<int64_t>(L.step_row.size()) - 1, static_cast<int64_t>(U.step_row.size()) - 1,
                           static_cast<int64_t>(L.col.size()), static_cast<int64_t>(U.col.size())};
    std::copy(st, st + 8, P->stats);
    *out = P.release();
    return SPIS_OK;
  })
}

extern "C" int spis_ilu_apply(spis_ilu* P, const double* q_dev, double* z_dev) {
  ABI_GUARD({
    if (!P || (P->n > 0 && (!q_dev || !z_dev))) return fail(SPIS_ERR_ARG, "null argument");
    if (q_dev == z_dev && P->n > 0) return fail(SPIS_ERR_ARG, "q and z must not alias");
    HIP_TRY(hipSetDevice(P->ctx->device));
    ST_TRY(ilu_enqueue(P, q_dev, z_dev, P->ctx->stream));
    HIP_TRY(hipStreamSynchronize(P->ctx->stream));
    return ilu_check(P);
  })
}

extern "C" int spis_ilu_info(spis_ilu* P, int64_t info[8]) {
  if (!P || !info) return fail(SPIS_ERR_ARG, "null argument");
  std::copy(P->stats, P->stats + 8, info);
  return SPIS_OK;
}

extern "C" int spis_ilu_destroy(spis_ilu* P) {
  ABI_GUARD({
    if (!P) return SPIS_OK;
    (void)hipSetDevice(P->ctx->device);
    (void)hipStreamSynchronize(P->ctx->stream);
    free_ilu(P);
    return SPIS_OK;
  })
}

// several GPUs: the global index of each of A's local columns (owned columns first, in the rows'
// order, then the ghosts) and whether the global matrix is exactly symmetric; K7t then pairs a
// rank's entries (r, c) by global index (distributed.py computes both from the global matrix)
extern "C" int spis_matrix_set_global(spis_matrix* M, const int64_t* col_gid, int32_t symmetric) {
  ABI_GUARD({
    if (!M || !col_gid) return fail(SPIS_ERR_ARG, "null argument");
    if (M->n_rows > M->n_cols) return fail(SPIS_ERR_ARG, "spis_matrix_set_global: more rows than columns");
    M->gid.assign(col_gid, col_gid + M->n_cols);
    M->gsym = symmetric ? 1 : 0;
    if (M->sym_state == 1) {  // the table was built without the global numbering
      (void)hipFree(M->sym_col);
      (void)hipFree(M->sym_val);
      (void)hipFree(M->sym_mask);
      M->sym_col = nullptr;
      M->sym_val = nullptr;
      M->sym_mask = nullptr;
    }
    M->sym_state = -1;
    return SPIS_OK;
  })
}

extern "C" int spis_matrix_info(spis_matrix* M, int64_t info[8]) {
  if (!M || !info) return fail(SPIS_ERR_ARG, "null argument");
  info[0] = M->n_rows;
  info[1] = M->n_cols;
  info[2] = M->nnz;
  info[3] = M->n_blk;
  info[4] = M->n_long;
  info[5] = M->n_ghost;
  info[6] = M->all_zero ? 1 : 0;
  info[7] = 0;
  return SPIS_OK;
}

// ------------------------------------------------------------------------------------------------
// memory + primitives
// ------------------------------------------------------------------------------------------------
static size_t alloc_class(int64_t bytes) {  // 256-B classes below 1 MiB, 64 KiB classes above
  const size_t b = static_cast<size_t>(std::max<int64_t>(bytes, 16));
  return b < (1u << 20) ? (b + 255) / 256 * 256 : (b + 65535) / 65536 * 65536;
}

static constexpr size_t kCacheLimit = size_t(16) << 30;  // bytes kept on the free list

extern "C" int spis_malloc(spis_context* c, int64_t bytes, void** out) {
  ABI_GUARD({
    if (!c || !out || bytes < 0) return fail(SPIS_ERR_ARG, "bad argument");
    HIP_TRY(hipSetDevice(c->device));
    const size_t sz = alloc_class(bytes);
    void* p = nullptr;
    auto it = c->free_blocks.find(sz);
    if (it != c->free_blocks.end()) {
      p = it->second;
      c->free_blocks.erase(it);
      c->cached_bytes -= sz;
    } else {
      hipError_t e = hipMalloc(&p, sz);
      if (e != hipSuccess) {  // give the cached blocks back and retry once
        (void)hipGetLastError();
        HIP_TRY(hipStreamSynchronize(c->stream));
        release_cache(c);
        HIP_TRY(hipMalloc(&p, sz));
      }
    }
    c->live_blocks[p] = sz;
    // zero-filled, ordered before every later use of the block on this stream (no host wait)
    HIP_TRY(hipMemsetAsync(p, 0, sz, c->stream));
    *out = p;
    return SPIS_OK;
  })
}

extern "C" int spis_free(spis_context* c, void* p) {
  ABI_GUARD({
    if (!c) return fail(SPIS_ERR_ARG, "null context");
    if (!p) return SPIS_OK;
    auto it = c->live_blocks.find(p);
    if (it == c->live_blocks.end()) return fail(SPIS_ERR_ARG, "spis_free: pointer not from spis_malloc");
    const size_t sz = it->second;
    c->live_blocks.erase(it);
    if (c->cached_bytes + sz <= kCacheLimit) {  // reusable in stream order: no wait
      c->free_blocks.emplace(sz, p);
      c->cached_bytes += sz;
      return SPIS_OK;
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipFree(p));
    return SPIS_OK;
  })
}

// the copies finish by an event spin (a blocking stream synchronize wakes the host up tens of us
// late: a drop-in call downloads x and uploads b each time)
extern "C" int spis_memcpy_h2d(spis_context* c, void* dst, const void* src, int64_t bytes) {
  ABI_GUARD({
    if (!c || (bytes > 0 && (!dst || !src))) return fail(SPIS_ERR_ARG, "bad argument");
    if (bytes > 0) HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipEventRecord(c->ev_gram, c->stream));
    return wait_event(c->ev_gram);
  })
}

extern "C" int spis_memcpy_d2h(spis_context* c, void* dst, const void* src, int64_t bytes) {
  ABI_GUARD({
    if (!c || (bytes > 0 && (!dst || !src))) return fail(SPIS_ERR_ARG, "bad argument");
    if (bytes > 0) HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipEventRecord(c->ev_gram, c->stream));
    return wait_event(c->ev_gram);
  })
}

extern "C" int spis_host_alloc(int64_t bytes, void** out) {
  ABI_GUARD({
    if (!out || bytes < 0) return fail(SPIS_ERR_ARG, "bad argument");
    *out = nullptr;
    HIP_TRY(hipHostMalloc(out, static_cast<size_t>(std::max<int64_t>(bytes, 8)), hipHostMallocDefault));
    return SPIS_OK;
  })
}

extern "C" int spis_host_free(void* p) {
  ABI_GUARD({
    if (p) HIP_TRY(hipHostFree(p));
    return SPIS_OK;
  })
}

extern "C" int spis_host_register(void* p, int64_t bytes) {
  ABI_GUARD({
    if (!p || bytes <= 0) return fail(SPIS_ERR_ARG, "bad argument");
    HIP_TRY(hipHostRegister(p, static_cast<size_t>(bytes), hipHostRegisterDefault));
    return SPIS_OK;
  })
}

extern "C" int spis_host_unregister(void* p) {
  ABI_GUARD({
    if (p) HIP_TRY(hipHostUnregister(p));
    return SPIS_OK;
  })
}

extern "C" int spis_memcpy_h2d_async(spis_context* c, void* dst, const void* src, int64_t bytes) {
  ABI_GUARD({
    if (!c || (bytes > 0 && (!dst || !src))) return fail(SPIS_ERR_ARG, "bad argument");
    if (bytes > 0) HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
    return SPIS_OK;
  })
}

extern "C" int spis_copy_to_host(spis_context* c, double* dst, const double* src, int64_t n) {
  ABI_GUARD({
    if (!c || n < 0 || (n > 0 && (!dst || !src))) return fail(SPIS_ERR_ARG, "bad argument");
    void* dd = nullptr;
    if (n > 0 && hipHostGetDevicePointer(&dd, dst, 0) == hipSuccess && dd != nullptr) {
      HIP_TRY(launch_copy(n, src, static_cast<double*>(dd), c->stream));
    } else {
      (void)hipGetLastError();
      if (n > 0) HIP_TRY(hipMemcpyAsync(dst, src, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream));
    }
    HIP_TRY(hipEventRecord(c->ev_gram, c->stream));
    return wait_event(c->ev_gram);
  })
}

extern "C" int spis_spmv(spis_context* c, spis_matrix* A, double* x, double* y) {
  ABI_GUARD({
    if (!c || !A || !x || !y) return fail(SPIS_ERR_ARG, "null argument");
    ST_TRY(exchange(c, A, x));
    HIP_TRY(launch_spmv(A->dual_view(), kEpiPlain, x, y, nullptr, nullptr, spmv_grid(A->dual_view(), fixed_grid(c)),
                        c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return SPIS_OK;
  })
}

extern "C" int spis_residual_norm(spis_context* c, spis_matrix* A, double* x, const double* b, double* out) {
  ABI_GUARD({
    if (!c || !A || !x || !b || !out) return fail(SPIS_ERR_ARG, "null argument");
    ST_TRY(exchange(c, A, x));
    const int g = spmv_grid(A->dual_view(), fixed_grid(c));
    HIP_TRY(launch_spmv(A->dual_view(), kEpiResNorm, x, nullptr, b, c->partA, g, c->stream));
    ST_TRY(allreduce(c, c->partA, g));
    HIP_TRY(launch_finalize(c->partA, g, c->dscal, 1, c->stream));
    HIP_TRY(hipMemcpyAsync(out, c->dscal, sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return SPIS_OK;
  })
}

static int dot_impl(spis_context* c, int64_t n, const double* x, const double* y, double* out, int op) {
  const int g = blas_grid(n, fixed_grid(c));
  HIP_TRY(launch_dot(n, x, y, c->partA, g, c->stream));
  ST_TRY(allreduce(c, c->partA, g));
  HIP_TRY(launch_finalize(c->partA, g, c->dscal, op, c->stream));
  HIP_TRY(hipMemcpyAsync(out, c->dscal, sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SPIS_OK;
}

extern "C" int spis_dot(spis_context* c, int64_t n, const double* x, const double* y, double* out) {
  ABI_GUARD({
    if (!c || !x || !y || !out || n < 0) return fail(SPIS_ERR_ARG, "bad argument");
    return dot_impl(c, n, x, y, out, 0);
  })
}

extern "C" int spis_nrm2(spis_context* c, int64_t n, const double* x, double* out) {
  ABI_GUARD({
    if (!c || !x || !out || n < 0) return fail(SPIS_ERR_ARG, "bad argument");
    return dot_impl(c, n, x, x, out, 1);
  })
}

extern "C" int spis_axpy(spis_context* c, int64_t n, double h, const double* x, double* y) {
  ABI_GUARD({
    if (!c || !x || !y || n < 0) return fail(SPIS_ERR_ARG, "bad argument");
    HIP_TRY(launch_axpy(n, h, x, y, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return SPIS_OK;
  })
}

extern "C" int spis_gemv(spis_context* c, int64_t n, int32_t p, const double* Z, int64_t pitch,
                         const double* y_host, const double* x0, double* x) {
  ABI_GUARD({
    if (!c || !Z || !y_host || !x0 || !x || n < 0 || p < 1 || p > kMaxK || pitch < n)
      return fail(SPIS_ERR_ARG, "bad argument");
    if (p <= kYArg) {
      HIP_TRY(launch_gemv(n, p, Z, pitch, y_host, true, x0, x, c->stream));
    } else {
      for (int i = 0; i < p; ++i) c->pinned[i] = y_host[i];
      HIP_TRY(hipMemcpyAsync(c->dscal, c->pinned, sizeof(double) * p, hipMemcpyHostToDevice, c->stream));
      HIP_TRY(launch_gemv(n, p, Z, pitch, c->dscal, false, x0, x, c->stream));
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    return SPIS_OK;
  })
}

extern "C" int spis_gram(spis_context* c, int64_t n, int32_t nu, const double* const* U, int32_t nv,
                         const double* const* V, double* G) {
  ABI_GUARD({
    if (!c || !U || !V || !G || nu < 1 || nv < 1 || n < 0) return fail(SPIS_ERR_ARG, "bad argument");
    return gram(c, n, nu, U, nv, V, G);
  })
}

// ------------------------------------------------------------------------------------------------
// constraint terms (class form), solvers.py:21-40, all constraints of a step at once:
//   MZ = M Z (one multi-vector SpMM launch per matrix, columns cached across the constrained
//   steps of a solve because the basis never changes), then ONE Gram
//   G = [z_0 .. z_{p-1}, x0]^T [M_1 Z, v_1, M_1 x0, M_2 Z, v_2, M_2 x0, ...]
// from which term0 / term1 / term2 of every constraint are read off.
// ------------------------------------------------------------------------------------------------
// fused path (p + 1 <= 64, <= 4 linear terms): transpose [Z, x0] once, then one pass per
// constraint matrix (K7t / K7m on the matrix cores, K7 on the CSR) — no M Z columns are materialised
// K7t's slot table (kernels.h SymTabView) of a square matrix that equals its transpose exactly;
// *ok = false otherwise.  Built once per matrix (ns = kSymSlots slots per block).
static int ensure_symtab(spis_context* c, spis_matrix* M, SymTabView* out, bool* ok) {
  constexpr int ns = kSymSlots;
  if (M->sym_state < 0) {
    M->sym_state = 0;
    const int64_t n = M->n_rows, nnz = M->nnz;
    // a rank's rows of a globally symmetric matrix (spis_matrix_set_global): entries are paired
    // by global index, the local numbering (owned, then ghosts) stays the Ut row index
    const bool global = !M->gid.empty() && M->gsym == 1 && static_cast<int64_t>(M->gid.size()) == M->n_cols;
    if (M->n_cols != n && !global) {
      *ok = false;
      return SPIS_OK;
    }
    std::vector<int32_t> rp(n + 1), ci(std::max<int64_t>(nnz, 1));
    std::vector<double> va(std::max<int64_t>(nnz, 1));
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipMemcpy(rp.data(), M->indptr, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToHost));
    if (nnz > 0) {
      HIP_TRY(hipMemcpy(ci.data(), M->indices, sizeof(int32_t) * nnz, hipMemcpyDeviceToHost));
      HIP_TRY(hipMemcpy(va.data(), M->vals, sizeof(double) * nnz, hipMemcpyDeviceToHost));
    }
    // exact symmetry: every row's (col, value) multiset equals the transpose's (the caller
    // declared it for a rank's rows of a global matrix)
    bool sym = true;
    if (!global) {
      std::vector<int64_t> tp(n + 1, 0);
      for (int64_t e = 0; e < nnz; ++e) ++tp[ci[e] + 1];
      for (int64_t r = 0; r < n; ++r) tp[r + 1] += tp[r];
      std::vector<int64_t> fill(tp.begin(), tp.end() - 1);
      std::vector<std::pair<int32_t, double>> te(std::max<int64_t>(nnz, 1));
      for (int64_t r = 0; r < n; ++r)
        for (int32_t e = rp[r]; e < rp[r + 1]; ++e) te[fill[ci[e]]++] = {static_cast<int32_t>(r), va[e]};
      std::vector<std::pair<int32_t, double>> row;
      for (int64_t r = 0; r < n && sym; ++r) {
        if (tp[r + 1] - tp[r] != rp[r + 1] - rp[r]) {
          sym = false;
          break;
        }
        row.clear();
        for (int32_t e = rp[r]; e < rp[r + 1]; ++e) row.push_back({ci[e], va[e]});
        auto lt = [](const std::pair<int32_t, double>& x, const std::pair<int32_t, double>& y) {
          return x.first != y.first ? x.first < y.first : x.second < y.second;
        };
        std::sort(row.begin(), row.end(), lt);
        std::vector<std::pair<int32_t, double>> trow(te.begin() + tp[r], te.begin() + tp[r + 1]);
        std::sort(trow.begin(), trow.end(), lt);
        for (size_t i = 0; i < row.size() && sym; ++i)
          sym = row[i].first == trow[i].first && row[i].second == trow[i].second;
      }
    }
    // the pairing key: the global index (identity on one GPU)
    auto key = [&](int64_t col) { return global ? M->gid[col] : col; };
    if (sym) {
      // segments of 4-row groups: slot 0 = each row's own U row (value M_rr / 2, duplicates summed),
      // then its entries with c > r in CSR order, padded (col = the row itself, value 0)
      std::vector<int32_t> tcol;
      std::vector<double> tval;
      std::vector<unsigned long long> tmask;
      int used = 0;            // slots used in the open block
      unsigned long long start_bits = 0;
      auto open_block = [&]() {
        tcol.resize(tcol.size() + 4 * static_cast<size_t>(ns), 0);
        tval.resize(tval.size() + 4 * static_cast<size_t>(ns), 0.0);
        tmask.push_back(0);
        used = 0;
        start_bits = 0;
      };
      auto close_block = [&]() {
        if (!tmask.empty()) tmask.back() = start_bits | (static_cast<unsigned long long>(used) << 32);
      };
      std::vector<int32_t> up[4];
      std::vector<double> upv[4];
      double diag[4];
      const int64_t ngroups = (n + 3) / 4;
      for (int64_t q = 0; q < ngroups; ++q) {
        int longest = 0;
        for (int g = 0; g < 4; ++g) {
          up[g].clear();
          upv[g].clear();
          diag[g] = 0.0;
          const int64_t r = 4 * q + g;
          if (r >= n) continue;
          const int64_t kr = key(r);  // a row's global index is its owned column's
          for (int32_t e = rp[r]; e < rp[r + 1]; ++e) {
            const int64_t kc = key(ci[e]);
            if (kc == kr) diag[g] += va[e];
            else if (kc > kr) {
              up[g].push_back(ci[e]);
              upv[g].push_back(va[e]);
            }
          }
          longest = std::max<int>(longest, static_cast<int>(up[g].size()));
        }
        // segments: own slot + up to ns - 1 entries each
        int done = 0;
        bool first = true;
        while (first || done < longest) {
          const int take = std::min(ns - 1, longest - done);
          const int need = 1 + take;
          if (tmask.empty() || used + need > ns) {
            close_block();
            open_block();
          }
          const size_t base = (tmask.size() - 1) * 4 * static_cast<size_t>(ns);
          start_bits |= 1ull << used;
          for (int g = 0; g < 4; ++g) {
            const int64_t r = 4 * q + g;
            const int32_t own = r < n ? static_cast<int32_t>(r) : 0;
            tcol[base + g * ns + used] = own;
            tval[base + g * ns + used] = (first && r < n) ? 0.5 * diag[g] : 0.0;
            for (int t = 0; t < take; ++t) {
              const int k = done + t;
              const bool has = k < static_cast<int>(up[g].size());
              tcol[base + g * ns + used + 1 + t] = has ? up[g][k] : own;
              tval[base + g * ns + used + 1 + t] = has ? upv[g][k] : 0.0;
            }
          }
          used += need;
          done += take;
          first = false;
        }
      }
      close_block();
      if (tmask.empty()) open_block(), close_block();
      auto up_ = [&](auto** dst, const auto& v) -> int {
        using T = typename std::remove_reference<decltype(v)>::type::value_type;
        HIP_TRY(hipMalloc(dst, sizeof(T) * std::max<size_t>(v.size(), 1)));
        if (!v.empty()) HIP_TRY(hipMemcpy(*dst, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice));
        return SPIS_OK;
      };
      ST_TRY(up_(&M->sym_col, tcol));
      ST_TRY(up_(&M->sym_val, tval));
      ST_TRY(up_(&M->sym_mask, tmask));
      M->sym_nblk = static_cast<int32_t>(tmask.size());
      M->sym_state = 1;
    }
  }
  *ok = M->sym_state == 1;
  if (*ok) *out = SymTabView{M->sym_col, M->sym_val, M->sym_mask, M->sym_nblk, ns};
  return SPIS_OK;
}

// host buffer of one step's reductions: constraint ci's G (np1 x np1) at ci * np1^2, then the
// linear terms (one np1 row per constraint with a v) at m * np1^2
static size_t con_result_len(int m, int p) {
  const size_t np1 = static_cast<size_t>(p) + 1;
  return static_cast<size_t>(m) * np1 * np1 + 4 * np1;
}

static int ensure_host_buf(double** buf, size_t* len, size_t need) {
  if (*len >= need) return SPIS_OK;
  if (*buf) HIP_TRY(hipHostFree(*buf));
  *buf = nullptr;
  *len = 0;
  HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(buf), sizeof(double) * need, hipHostMallocDefault));
  *len = need;
  return SPIS_OK;
}

// Enqueues the transpose and every constraint matrix's Gram of one step on stream st, each result
// copied to dst (layout: con_result_len).  One-time buffers and matrix copies are made first
// (they may synchronise the main stream, on first use only).
// a constrained step's reduction results polled in pinned memory: each value its own flag, armed with
// this sentinel (a signalling NaN no kernel writes) before the launches
constexpr uint64_t kConSentinel = 0x7FF4DEAD5EC0FFEDull;
using PollRanges = std::vector<std::pair<size_t, size_t>>;  // (offset, count) in c->con_pinned

static int con_gram_enqueue(spis_context* c, spis_workspace* ws, int m, const spis_constraint_desc* cons, int64_t n,
                            int p, const double* Z, int64_t pitch, const double* x0, hipStream_t st, double* dst,
                            PollRanges* poll = nullptr) {
  const int np1 = p + 1;
  const int ut_cols = np1 <= 32 ? 32 : 64;  // Ut is N x np1 row-major: size for this p bucket
  // several GPUs: a constraint matrix's ghost columns read the Ut rows of their owners, received
  // after the local rows (exchange_rows, per matrix: each has its own halo plan)
  int64_t ut_rows = std::max<int64_t>(n, 1);
  for (int ci = 0; ci < m; ++ci)
    if (c->dist_on() && cons[ci].M != nullptr) ut_rows = std::max<int64_t>(ut_rows, n + cons[ci].M->n_ghost);
  if (ws->Ut && (ws->Ut_cols < ut_cols || ws->Ut_rows < ut_rows)) {
    HIP_TRY(hipFree(ws->Ut));
    ws->Ut = nullptr;
  }
  if (!ws->Ut) {
    HIP_TRY(hipMalloc(&ws->Ut, sizeof(double) * ut_rows * ut_cols));
    ws->Ut_cols = ut_cols;
    ws->Ut_rows = ut_rows;
  }
  const size_t need = static_cast<size_t>(constraint_gram_partials()) * (np1 * np1 + 4 * np1);
  if (c->cg_part_len < need) {
    if (c->cg_part) HIP_TRY(hipFree(c->cg_part));
    HIP_TRY(hipMalloc(&c->cg_part, need * sizeof(double)));
    c->cg_part_len = need;
  }
  if (!c->cg_G) HIP_TRY(hipMalloc(&c->cg_G, sizeof(double) * (64 * 64 + 4 * 64)));
  std::vector<const double*> vlist;
  for (int ci = 0; ci < m; ++ci)
    if (cons[ci].v_dev) vlist.push_back(cons[ci].v_dev);
  struct Launch {
    int ci;
    bool sym;
    SymTabView tv;
  };
  // con_gram 2: K7t for symmetric matrices, K7m otherwise, the linear terms from the transpose;
  // 3: K7m for every matrix.  Both read Ut in the MFMA column order.  1 (and p + 1 > 32): K7 on the CSR.
  const int eg = c->con_gram;
  const bool mfma = np1 <= 32 && eg >= 2;
  // K7t pairs (r, c) with (c, r): on several GPUs by global index, for the matrices declared
  // symmetric with their global numbering (spis_matrix_set_global); the others take K7m
  const bool tsym = mfma && eg == 2;
  std::vector<Launch> plan;
  for (int ci = 0; ci < m; ++ci) {
    if (cons[ci].M == nullptr || cons[ci].M->all_zero) continue;
    Launch L{ci, false, {}};
    if (tsym) ST_TRY(ensure_symtab(c, cons[ci].M, &L.tv, &L.sym));
    plan.push_back(L);
  }
  const size_t voff = static_cast<size_t>(m) * np1 * np1;
  const int nv = static_cast<int>(vlist.size());
  bool v_done = nv == 0;
  bool all_sym = tsym;
  for (const Launch& L : plan) all_sym = all_sym && L.sym;
  if (poll != nullptr && all_sym && !c->dist_on()) {
    // one GPU, K7t only: the reductions store every value into dst (pinned) themselves, system
    // scope, each its own flag (the host polls them, con_step_wait): no copy packets and no
    // system-scope event release in front of the host's KKT solve
    poll->clear();
    if (nv > 0) poll->push_back({voff, static_cast<size_t>(nv) * np1});
    for (const Launch& L : plan) poll->push_back({static_cast<size_t>(L.ci) * np1 * np1, static_cast<size_t>(np1) * np1});
    for (const auto& rg : *poll)
      for (size_t q = 0; q < rg.second; ++q) reinterpret_cast<volatile uint64_t*>(dst)[rg.first + q] = kConSentinel;
    void* dp = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&dp, dst, 0));
    double* dstd = static_cast<double*>(dp);
    if (!c->cg_vpart) HIP_TRY(hipMalloc(&c->cg_vpart, sizeof(double) * kTransposeGrid * 4 * 32));
    // the linear terms' column reduction rides in the first K7t reduction launch (one launch fewer)
    ColReduce lin{0, 0, nullptr, nullptr};
    HIP_TRY(launch_transpose_basis_lin(n, p, Z, pitch, x0, ws->Ut, nv, vlist.data(), c->cg_vpart, dstd + voff, st,
                                       true, c->transpose_pipe, plan.empty() ? nullptr : &lin));
    for (size_t i = 0; i < plan.size(); ++i)
      HIP_TRY(launch_constraint_gram_sym(np1, plan[i].tv, ws->Ut, c->cg_part,
                                         dstd + static_cast<size_t>(plan[i].ci) * np1 * np1, st, true,
                                         i == 0 && lin.npairs > 0 ? &lin : nullptr));
    return SPIS_OK;
  }
  if (tsym) {  // Ut + the linear terms in one pass over the basis
    if (!c->cg_vpart) HIP_TRY(hipMalloc(&c->cg_vpart, sizeof(double) * kTransposeGrid * 4 * 32));
    HIP_TRY(launch_transpose_basis_lin(n, p, Z, pitch, x0, ws->Ut, nv, vlist.data(), c->cg_vpart,
                                       c->cg_G + 64 * 64, st, false, c->transpose_pipe));
    if (nv > 0) ST_TRY(allreduce_on(c, c->cg_G + 64 * 64, static_cast<int64_t>(nv) * np1, st));  // local rows' sums
    if (nv > 0)
      HIP_TRY(hipMemcpyAsync(dst + voff, c->cg_G + 64 * 64, sizeof(double) * nv * np1, hipMemcpyDeviceToHost, st));
    v_done = true;
  } else {
    HIP_TRY(launch_transpose_basis(n, p, Z, pitch, x0, ws->Ut, st, mfma));
  }
  for (const Launch& L : plan) {
    const CsrView mv = cons[L.ci].M->view();
    const int nvv = v_done ? 0 : nv;
    spis_matrix* Mc = cons[L.ci].M;
    if (c->dist_on()) ST_TRY(exchange_rows(c, Mc, ws->Ut, ut_cols, st));
    if (L.sym) {
      HIP_TRY(launch_constraint_gram_sym(np1, L.tv, ws->Ut, c->cg_part, c->cg_G, st));
    } else if (mfma) {
      HIP_TRY(launch_constraint_gram_mfma(n, np1, &mv, &Mc->gram_rows, ws->Ut, nvv, vlist.data(),
                                          c->cg_part, c->cg_G, st));
    } else {
      HIP_TRY(launch_constraint_gram(n, np1, &mv, ws->Ut, nvv, vlist.data(), c->cg_part, c->cg_G, st));
    }
    ST_TRY(allreduce_on(c, c->cg_G, static_cast<int64_t>(np1) * np1 + static_cast<int64_t>(nvv) * np1, st));
    HIP_TRY(hipMemcpyAsync(dst + static_cast<size_t>(L.ci) * np1 * np1, c->cg_G, sizeof(double) * np1 * np1,
                           hipMemcpyDeviceToHost, st));
    if (nvv > 0)
      HIP_TRY(hipMemcpyAsync(dst + voff, c->cg_G + np1 * np1, sizeof(double) * nvv * np1, hipMemcpyDeviceToHost, st));
    v_done = true;
  }
  if (!v_done) {  // linear terms only
    if (mfma)
      HIP_TRY(launch_constraint_gram_mfma(n, np1, nullptr, nullptr, ws->Ut, nv, vlist.data(), c->cg_part,
                                          c->cg_G, st));
    else
      HIP_TRY(launch_constraint_gram(n, np1, nullptr, ws->Ut, nv, vlist.data(), c->cg_part, c->cg_G, st));
    ST_TRY(allreduce_on(c, c->cg_G + np1 * np1, static_cast<int64_t>(nv) * np1, st));
    HIP_TRY(hipMemcpyAsync(dst + voff, c->cg_G + np1 * np1, sizeof(double) * nv * np1, hipMemcpyDeviceToHost, st));
  }
  return SPIS_OK;
}

// term0 / term1 / term2 of every constraint (solvers.py:34-36) from con_gram_enqueue's results
static void con_terms_assemble(int m, const spis_constraint_desc* cons, int p, const double* src, QuadCon* out) {
  const int np1 = p + 1;
  const double* gvall = src + static_cast<size_t>(m) * np1 * np1;
  int iv = 0;
  for (int ci = 0; ci < m; ++ci) {
    QuadCon& q = out[ci];
    q.term1.assign(p, 0.0);
    q.term2.assign(static_cast<size_t>(p) * p, 0.0);
    const bool hasM = cons[ci].M != nullptr && !cons[ci].M->all_zero;
    const double* G = src + static_cast<size_t>(ci) * np1 * np1;
    const double* gv = cons[ci].v_dev ? gvall + static_cast<size_t>(iv++) * np1 : nullptr;
    const double x0Mx0 = hasM ? G[static_cast<size_t>(p) * np1 + p] : 0.0;
    const double vx0 = gv ? gv[p] : 0.0;
    q.term0 = 0.5 * x0Mx0 + cons[ci].c + vx0;  // solvers.py:34
    for (int a = 0; a < p; ++a)                // :35
      q.term1[a] = (gv ? gv[a] : 0.0) + (hasM ? G[static_cast<size_t>(p) * np1 + a] : 0.0);
    if (hasM)                                  // :36
      for (int a = 0; a < p; ++a)
        for (int b = 0; b < p; ++b) q.term2[static_cast<size_t>(a) * p + b] = 0.5 * G[static_cast<size_t>(a) * np1 + b];
  }
}

// fused path, synchronous: every launch of the step, then one wait
struct ConStep;
static int con_step_enqueue(spis_context* c, spis_workspace* ws, int m, const spis_constraint_desc* cons, int64_t n,
                            int p, const double* Z, int64_t pitch, const double* x0, ConStep* cs, bool side);
static void con_step_assemble(spis_context* c, spis_workspace* ws, const spis_constraint_desc* cons,
                              const ConStep& cs, QuadCon* out);
static int constraint_terms_fused(spis_context* c, spis_workspace* ws, int m, const spis_constraint_desc* cons,
                                  int64_t n, int p, const double* Z, int64_t pitch, const double* x0,
                                  QuadCon* out);

// the fused reduction (con_gram_enqueue) serves this step
static bool fused_con_ok(const spis_context* c, int p, int m, const spis_constraint_desc* cons) {
  int nlin = 0;
  for (int ci = 0; ci < m; ++ci) nlin += cons[ci].v_dev ? 1 : 0;
  // several GPUs: K7m on the local rows, the ghost Ut rows exchanged per matrix, G all-reduced
  if (c->dist_on() && !(p + 1 <= 32 && c->con_gram >= 2)) return false;
  return p + 1 <= 64 && nlin <= 4 && c->con_gram != 0;
}

static int constraint_terms_all(spis_context* c, spis_workspace* ws, int m, const spis_constraint_desc* cons,
                                int64_t n, int p, const double* Z, int64_t pitch, const double* x0,
                                QuadCon* out) {
  if (fused_con_ok(c, p, m, cons)) return constraint_terms_fused(c, ws, m, cons, n, p, Z, pitch, x0, out);
  std::vector<const double*> U, V;
  for (int i = 0; i < p; ++i) U.push_back(Z + static_cast<int64_t>(i) * pitch);
  U.push_back(x0);
  struct Idx {
    int mz0 = -1, iv = -1, imx = -1;
  };
  std::vector<Idx> idx(m);
  for (int ci = 0; ci < m; ++ci) {
    const spis_constraint_desc& con = cons[ci];
    ConCache& cc = ws->con[ci];
    const bool mzero = con.M == nullptr || con.M->all_zero;
    if (!mzero) {
      if (con.M->n_rows != n) return fail(SPIS_ERR_ARG, "constraint matrix rows != n");
      if (cc.cols < p) {
        if (!c->dist_on() || con.M->n_ghost == 0) {
          HIP_TRY(launch_spmm(con.M->view(), Z + static_cast<int64_t>(cc.cols) * pitch, pitch, p - cc.cols,
                              cc.MZ + static_cast<int64_t>(cc.cols) * ws->pitch_n, ws->pitch_n, c->stream));
        } else {
          for (int i = cc.cols; i < p; ++i)
            ST_TRY(spmv_local(c, ws, con.M, Z + static_cast<int64_t>(i) * pitch,
                              cc.MZ + static_cast<int64_t>(i) * ws->pitch_n));
        }
        cc.cols = p;
      }
      if (!cc.mx0_done) {
        ST_TRY(spmv_local(c, ws, con.M, x0, cc.Mx0));
        cc.mx0_done = true;
      }
      idx[ci].mz0 = static_cast<int>(V.size());
      for (int i = 0; i < p; ++i) V.push_back(cc.MZ + static_cast<int64_t>(i) * ws->pitch_n);
    }
    if (con.v_dev) {
      idx[ci].iv = static_cast<int>(V.size());
      V.push_back(con.v_dev);
    }
    if (!mzero) {
      idx[ci].imx = static_cast<int>(V.size());
      V.push_back(cc.Mx0);
    }
  }
  const int nu = p + 1, nv = static_cast<int>(V.size());
  std::vector<double> G(static_cast<size_t>(nu) * std::max(nv, 1), 0.0);
  if (nv > 0) ST_TRY(gram(c, n, nu, U.data(), nv, V.data(), G.data()));
  auto g = [&](int a, int b) { return G[static_cast<size_t>(a) * nv + b]; };
  for (int ci = 0; ci < m; ++ci) {
    const Idx& d = idx[ci];
    QuadCon& q = out[ci];
    q.term1.assign(p, 0.0);
    q.term2.assign(static_cast<size_t>(p) * p, 0.0);
    const double x0Mx0 = d.imx >= 0 ? g(p, d.imx) : 0.0;
    const double vx0 = d.iv >= 0 ? g(p, d.iv) : 0.0;
    q.term0 = 0.5 * x0Mx0 + cons[ci].c + vx0;  // 0.5*x0@M@x0 + c + v@x0  (solvers.py:34)
    for (int a = 0; a < p; ++a)                // v@Z + x0@MZ             (:35)
      q.term1[a] = (d.iv >= 0 ? g(a, d.iv) : 0.0) + (d.mz0 >= 0 ? g(p, d.mz0 + a) : 0.0);
    if (d.mz0 >= 0)                            // 0.5*Z.T@MZ              (:36)
      for (int a = 0; a < p; ++a)
        for (int b = 0; b < p; ++b) q.term2[static_cast<size_t>(a) * p + b] = 0.5 * g(a, d.mz0 + b);
  }
  return SPIS_OK;
}

// ---- incremental constraint Gram -------------------------------
// A constrained step with p columns needs, per class-form constraint, G = U^T M U and v . U over
// U = [z_0 .. z_{p-1}, x0] (solvers.py:33-36).  Within one solve Z and x0 never change, so the
// entries of columns reduced at an earlier constrained step stay valid (ConCache gc / gv), and a
// later step reduces only its new columns a: u = M z_a (one SpMV), then [z_0 .. z_a, x0] . u (one
// multidot pass over a + 2 vectors) and v . z_a.  That is CGMRES's constrained suffix after the
// first constrained step (solvers.py:230: every later step is constrained) and every step of
// CGMRES_P (solvers.py:396-401), where the reference recomputes M @ Z and Z.T @ MZ whole.
// Symmetric M only (gc(b, a) = gc(a, b) = z_b . M z_a; the K7t test, exact): a non-symmetric M's
// quadratic term is not symmetric in the reference's algebra either, so it keeps the full path.
// The first constrained step takes the full reduction (transpose + K7t) and seeds the caches,
// unless its p is small enough that columns 0 .. p-1 from scratch cost less (kIncScratch).
constexpr int kIncScratch = 8;

// one value an increment step computes: G(a, b) = z_a . M z_b of constraint ci (m), else its
// v . z_a (gv[a]); a, b = k stand for x0
struct IncSlot {
  int ci, a, b;
  bool m;
};
// one pass over a constraint matrix: u = M z_a (a = k: M x0), dotted with [z_0 .. z_a, x0] (x0)
struct IncPass {
  int ci, a, slot0, nl;
};

struct ConStep {
  bool inc = false;  // increments enqueued (else the full reduction)
  int p = 0, m = 0;
  std::vector<int> from;  // per constraint: first new column (inc)
  hipStream_t st = nullptr;  // the stream the results are copied on (record the wait's event there)
  // inc: the values in partial / result order: the first pass's, the pair dots v . z_a, v . x0,
  // the other passes'
  std::vector<IncSlot> slots;
  std::vector<IncPass> passes;
  int pair0 = 0, npair = 0;
  // the caller's request: the previous step's update GEMV x = x0 + Z[:, :gx_p] y (gx_p <= kYArg) in a
  // multidot that reads z_0 .. z_{gx_p - 1} anyway; gx_done tells whether one took it
  int gx_p = 0;
  const double* gx_y = nullptr;
  double* gx_out = nullptr;
  bool gx_done = false;
  PollRanges poll;  // non-empty: the values arrive as polled pinned slots (no ev_gram to wait for)
};

static bool con_inc_eligible(spis_context* c, spis_workspace* ws, int m, const spis_constraint_desc* cons, int p) {
  if (!fused_con_ok(c, p, m, cons) || p + 2 > kMdMax || static_cast<int>(ws->con.size()) < m) return false;
  if (!c->gram_inc) return false;
  for (int ci = 0; ci < m; ++ci) {
    spis_matrix* M = cons[ci].M;
    if (M == nullptr || M->all_zero) continue;
    if (c->con_gram != 2) return false;  // the symmetric test is K7t's
    SymTabView tv;
    bool sym = false;
    if (ensure_symtab(c, M, &tv, &sym) != SPIS_OK || !sym) return false;
  }
  return true;
}

// the values and passes of one increment step (ConStep::slots / passes, in partial order)
static void con_inc_plan(int m, const spis_constraint_desc* cons, int p, const spis_workspace* ws, ConStep& cs) {
  const int k = ws->k;
  cs.slots.clear();
  cs.passes.clear();
  std::vector<IncSlot> pairs;  // grouped by constraint (one multidot per constraint when not carried)
  for (int ci = 0; ci < m; ++ci) {
    const bool hasM = cons[ci].M != nullptr && !cons[ci].M->all_zero;
    const bool hasV = cons[ci].v_dev != nullptr;
    for (int a = cs.from[ci]; a < p; ++a) {
      if (hasM) cs.passes.push_back({ci, a, 0, a + 2});
      if (hasV) pairs.push_back({ci, a, 0, false});
    }
    if (ws->con[ci].gcols < 0) {  // x0's own terms: x0 . M x0, v . x0
      if (hasM) cs.passes.push_back({ci, k, 0, 1});
      if (hasV) pairs.push_back({ci, k, 0, false});
    }
  }
  auto add_pass = [&](IncPass& ps) {
    ps.slot0 = static_cast<int>(cs.slots.size());
    if (ps.a == k) {
      cs.slots.push_back({ps.ci, k, k, true});
      return;
    }
    for (int b = 0; b <= ps.a; ++b) cs.slots.push_back({ps.ci, ps.a, b, true});
    cs.slots.push_back({ps.ci, ps.a, k, true});
  };
  if (!cs.passes.empty()) add_pass(cs.passes[0]);
  cs.pair0 = static_cast<int>(cs.slots.size());
  cs.npair = static_cast<int>(pairs.size());
  cs.slots.insert(cs.slots.end(), pairs.begin(), pairs.end());
  for (size_t i = 1; i < cs.passes.size(); ++i) add_pass(cs.passes[i]);
}

static int con_inc_enqueue(spis_context* c, spis_workspace* ws, const spis_constraint_desc* cons, int64_t n,
                           const double* Z, int64_t pitch, const double* x0, ConStep& cs) {
  hipStream_t st = cs.st;
  const int k = ws->k;
  const size_t total = cs.slots.size();
  if (total == 0) return SPIS_OK;
  ST_TRY(ensure_host_buf(&c->con_pinned, &c->con_pinned_len, total));
  const int g = fixed_grid(c) ? kRedGrid : static_cast<int>(std::min<int64_t>(kRedGrid, std::max<int64_t>(1, (n + 255) / 256)));
  if (c->inc_part_len < total * g) {
    if (c->inc_part) HIP_TRY(hipFree(c->inc_part));
    HIP_TRY(hipMalloc(&c->inc_part, sizeof(double) * total * g));
    c->inc_part_len = total * g;
  }
  if (c->inc_res_len < total) {
    if (c->inc_res) HIP_TRY(hipFree(c->inc_res));
    HIP_TRY(hipMalloc(&c->inc_res, sizeof(double) * total));
    c->inc_res_len = total;
  }
  auto zv = [&](int a) { return a == k ? x0 : Z + static_cast<int64_t>(a) * pitch; };
  auto part_at = [&](int slot) { return c->inc_part + static_cast<size_t>(slot) * g; };
  if (c->inc_u_len < n) {
    if (c->inc_u) HIP_TRY(hipFree(c->inc_u));
    HIP_TRY(hipMalloc(&c->inc_u, sizeof(double) * std::max<int64_t>(n, 1)));
    c->inc_u_len = n;
  }
  // per pass: u = M z_a (K1p), then [z_0 .. z_a, x0] . u (multidot); the pair dots v . z_a ride in
  // the first pass's multidot when they are one constraint's (the slots follow that pass's), else
  // one multidot per constraint; one finalize for every value.  (A fused SpMV + dots kernel, the
  // dots in the SpMV's row epilogue, ran 75-175 us per pass at C3 against 26 + 8-30 here: its
  // epilogue loads of the dotted vectors are not prefetched: gpurun_out/r05inc3)
  bool carried = false;
  for (size_t i = 0; i < cs.passes.size(); ++i) {
    const IncPass& ps = cs.passes[i];
    VecList L{};
    if (ps.a == k) {
      L.v[0] = x0;
    } else {
      for (int b = 0; b <= ps.a; ++b) L.v[b] = zv(b);
      L.v[ps.a + 1] = x0;
    }
    int nl = ps.nl, n2 = 0;
    const double* u2 = nullptr;
    if (i == 0 && cs.npair > 0 && ps.nl + cs.npair <= kMdMax) {
      const int ci2 = cs.slots[cs.pair0].ci;
      bool one = true;
      for (int q = 0; q < cs.npair; ++q) one = one && cs.slots[cs.pair0 + q].ci == ci2;
      if (one) {
        for (int q = 0; q < cs.npair; ++q) L.v[nl + q] = zv(cs.slots[cs.pair0 + q].a);
        u2 = cons[ci2].v_dev;
        n2 = cs.npair;
        nl += n2;
        carried = true;
      }
    }
    // the GEMV rides in the first pass whose list holds z_0 .. z_{gx_p - 1} (one GPU: x over the
    // local rows is all of x)
    int px = 0;
    if (!cs.gx_done && cs.gx_p > 0 && ps.a != k && ps.a + 1 >= cs.gx_p && !c->dist_on()) {
      px = cs.gx_p;
      cs.gx_done = true;
    }
    ST_TRY(spmv_local(c, ws, cons[ps.ci].M, zv(ps.a), c->inc_u, st));
    HIP_TRY(launch_multidot(n, c->inc_u, L, nl, part_at(ps.slot0), g, st, u2, n2, px, cs.gx_y, x0, cs.gx_out));
  }
  if (!carried)
    for (int q = 0; q < cs.npair;) {
      const int ci = cs.slots[cs.pair0 + q].ci;
      VecList L{};
      int cnt = 0;
      while (q + cnt < cs.npair && cs.slots[cs.pair0 + q + cnt].ci == ci && cnt < kMdMax) {
        L.v[cnt] = zv(cs.slots[cs.pair0 + q + cnt].a);
        ++cnt;
      }
      HIP_TRY(launch_multidot(n, cons[ci].v_dev, L, cnt, part_at(cs.pair0 + q), g, st));
      q += cnt;
    }
  if (!c->dist_on()) {  // the finalize stores the values straight into pinned memory, system scope,
                        // each its own flag (con_step_wait polls them): no copy packet, and no
                        // system-scope event release (an L2 write-back, ~5 us before the next kernel)
    for (size_t i = 0; i < total; ++i) reinterpret_cast<volatile uint64_t*>(c->con_pinned)[i] = kConSentinel;
    void* dp = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&dp, c->con_pinned, 0));
    HIP_TRY(launch_cgs_finalize(c->inc_part, g, static_cast<int>(total), static_cast<double*>(dp), nullptr, nullptr, st,
                                0, true));
    cs.poll.assign(1, {size_t(0), total});
    return SPIS_OK;
  }
  HIP_TRY(launch_cgs_finalize(c->inc_part, g, static_cast<int>(total), c->inc_res, nullptr, nullptr, st));
  ST_TRY(allreduce_on(c, c->inc_res, static_cast<int64_t>(total), st));  // several GPUs: rows summed
  HIP_TRY(hipMemcpyAsync(c->con_pinned, c->inc_res, sizeof(double) * total, hipMemcpyDeviceToHost, st));
  return SPIS_OK;
}

// the increments into the caches (after the wait)
static void con_inc_take(spis_workspace* ws, int m, const ConStep& cs, const double* src) {
  const int k = ws->k;
  for (size_t s = 0; s < cs.slots.size(); ++s) {
    const IncSlot& sl = cs.slots[s];
    ConCache& cc = ws->con[sl.ci];
    if (sl.m) {
      cc.gc[static_cast<size_t>(sl.a) * (k + 1) + sl.b] = src[s];
      cc.gc[static_cast<size_t>(sl.b) * (k + 1) + sl.a] = src[s];
    } else {
      cc.gv[sl.a] = src[s];
    }
  }
  for (int ci = 0; ci < m; ++ci) ws->con[ci].gcols = cs.p;
}

// the full reduction's results (con_gram_enqueue's layout) into the caches
static void con_full_take(spis_workspace* ws, int m, const spis_constraint_desc* cons, int p, const double* src) {
  const int k = ws->k, np1 = p + 1;
  const double* gvall = src + static_cast<size_t>(m) * np1 * np1;
  int iv = 0;
  for (int ci = 0; ci < m; ++ci) {
    ConCache& cc = ws->con[ci];
    const bool hasM = cons[ci].M != nullptr && !cons[ci].M->all_zero;
    const double* Gs = src + static_cast<size_t>(ci) * np1 * np1;
    auto G = [&](int a, int b) -> double& { return cc.gc[static_cast<size_t>(a) * (k + 1) + b]; };
    if (hasM)
      for (int a = 0; a <= p; ++a)
        for (int b = 0; b <= p; ++b) G(a == p ? k : a, b == p ? k : b) = Gs[static_cast<size_t>(a) * np1 + b];
    if (cons[ci].v_dev) {
      const double* gv = gvall + static_cast<size_t>(iv++) * np1;
      for (int a = 0; a < p; ++a) cc.gv[a] = gv[a];
      cc.gv[k] = gv[p];
    }
    cc.gcols = p;
  }
}

// term0 / term1 / term2 (solvers.py:34-36) from the caches
static void con_terms_from_cache(const spis_workspace* ws, int m, const spis_constraint_desc* cons, int p,
                                 QuadCon* out) {
  const int k = ws->k;
  for (int ci = 0; ci < m; ++ci) {
    const ConCache& cc = ws->con[ci];
    auto G = [&](int a, int b) { return cc.gc[static_cast<size_t>(a) * (k + 1) + b]; };
    const bool hasM = cons[ci].M != nullptr && !cons[ci].M->all_zero;
    const bool hasV = cons[ci].v_dev != nullptr;
    QuadCon& q = out[ci];
    q.term1.assign(p, 0.0);
    q.term2.assign(static_cast<size_t>(p) * p, 0.0);
    q.term0 = 0.5 * (hasM ? G(k, k) : 0.0) + cons[ci].c + (hasV ? cc.gv[k] : 0.0);
    for (int a = 0; a < p; ++a) q.term1[a] = (hasV ? cc.gv[a] : 0.0) + (hasM ? G(k, a) : 0.0);
    if (hasM)
      for (int a = 0; a < p; ++a)
        for (int b = 0; b < p; ++b) q.term2[static_cast<size_t>(a) * p + b] = 0.5 * G(a, b);
  }
}

// the host's wait for a step's reduction: its polled pinned slots, else ev_gram (recorded behind it)
static int con_step_wait(spis_context* c, const ConStep& cs) {
  if (cs.poll.empty()) return wait_event(c->ev_gram);
  const volatile uint64_t* w = reinterpret_cast<const volatile uint64_t*>(c->con_pinned);
  const double t0 = now_s();
  for (const auto& rg : cs.poll)
    for (size_t i = rg.first; i < rg.first + rg.second; ++i)
    for (unsigned spin = 0; __atomic_load_n(const_cast<const uint64_t*>(w + i), __ATOMIC_ACQUIRE) == kConSentinel;
         ++spin) {
      if ((spin & 4095) == 4095 && now_s() - t0 > 0.02) {  // a failed stream never writes them
        const hipError_t e = hipStreamQuery(cs.st);
        if (e != hipSuccess && e != hipErrorNotReady) return fail(SPIS_ERR_HIP, "stream: %s", hipGetErrorString(e));
        if (e == hipSuccess && __atomic_load_n(const_cast<const uint64_t*>(w + i), __ATOMIC_ACQUIRE) == kConSentinel)
          return fail(SPIS_ERR_STATE, "constraint increments: the stream drained without value %zu", i);
      }
      __builtin_ia32_pause();
    }
  return SPIS_OK;
}

// one constrained step's reduction, enqueued on the main stream with its results copied to
// c->con_pinned: the increments when every active constraint can take them, else the full
// reduction (which seeds the caches when they are eligible)
static int con_step_enqueue(spis_context* c, spis_workspace* ws, int m, const spis_constraint_desc* cons, int64_t n,
                            int p, const double* Z, int64_t pitch, const double* x0, ConStep* cs, bool side) {
  cs->p = p;
  cs->m = m;
  cs->inc = false;
  cs->gx_done = false;
  cs->poll.clear();
  cs->st = c->stream;
  cs->from.assign(m, 0);
  if (con_inc_eligible(c, ws, m, cons, p)) {
    bool fresh = false;  // a constraint without any cached column
    for (int ci = 0; ci < m; ++ci) {
      cs->from[ci] = std::max(0, std::min(ws->con[ci].gcols, p));
      fresh = fresh || ws->con[ci].gcols < 0;
    }
    cs->inc = !fresh || p <= kIncScratch;
  }
  if (cs->inc) {
    // side: the increments on stream2, beside the latency-bound MGS chain the host has just queued
    // (they read only z_0 .. z_{p-1}, finished by earlier chains, x0 and the constraint operators)
    if (side && !c->dist_on()) cs->st = c->stream2;
    con_inc_plan(m, cons, p, ws, *cs);
    return con_inc_enqueue(c, ws, cons, n, Z, pitch, x0, *cs);
  }
  ST_TRY(ensure_host_buf(&c->con_pinned, &c->con_pinned_len, con_result_len(m, p)));
  return con_gram_enqueue(c, ws, m, cons, n, p, Z, pitch, x0, c->stream, c->con_pinned, &cs->poll);
}

// after the wait: the step's terms (and the caches brought up to date)
static void con_step_assemble(spis_context* c, spis_workspace* ws, const spis_constraint_desc* cons,
                              const ConStep& cs, QuadCon* out) {
  if (cs.inc) {
    con_inc_take(ws, cs.m, cs, c->con_pinned);
    con_terms_from_cache(ws, cs.m, cons, cs.p, out);
    return;
  }
  con_terms_assemble(cs.m, cons, cs.p, c->con_pinned, out);
  if (con_inc_eligible(c, ws, cs.m, cons, cs.p)) con_full_take(ws, cs.m, cons, cs.p, c->con_pinned);
}

// fused path, synchronous: the step's launches (increments or the full reduction), then one wait
static int constraint_terms_fused(spis_context* c, spis_workspace* ws, int m, const spis_constraint_desc* cons,
                                  int64_t n, int p, const double* Z, int64_t pitch, const double* x0,
                                  QuadCon* out) {
  ConStep cs;
  ST_TRY(con_step_enqueue(c, ws, m, cons, n, p, Z, pitch, x0, &cs, false));
  if (cs.poll.empty()) HIP_TRY(hipEventRecord(c->ev_gram, c->stream));  // spin on it: a blocking
  ST_TRY(con_step_wait(c, cs));                                         // synchronize wakes up late
  con_step_assemble(c, ws, cons, cs, out);
  return SPIS_OK;
}

static int ensure_con_cache(spis_workspace* ws, size_t ncon, const spis_constraint_desc* cons) {
  if (ws->con.size() < ncon) ws->con.resize(ncon);
  for (size_t i = 0; i < ncon; ++i) {
    ConCache& cc = ws->con[i];
    cc.cols = 0;
    cc.mx0_done = false;
    cc.gcols = -1;
    cc.gc.assign(static_cast<size_t>(ws->k + 1) * (ws->k + 1), 0.0);
    cc.gv.assign(static_cast<size_t>(ws->k + 1), 0.0);
    const bool mzero = cons[i].M == nullptr || cons[i].M->all_zero;
    if (!mzero && !cc.MZ) {
      HIP_TRY(hipMalloc(&cc.MZ, sizeof(double) * ws->pitch_n * ws->k));
      HIP_TRY(hipMalloc(&cc.Mx0, sizeof(double) * ws->pitch_n));
    }
  }
  return SPIS_OK;
}

extern "C" int spis_constraint_terms(spis_context* c, const spis_constraint_desc* con, int64_t n, int32_t p,
                                     const double* Z, int64_t pitch, const double* x0, double* term0,
                                     double* term1, double* term2) {
  ABI_GUARD({
    if (!c || !con || !Z || !x0 || !term0 || !term1 || !term2 || p < 1 || n < 0 || pitch < n)
      return fail(SPIS_ERR_ARG, "bad argument");
    spis_workspace tmp;
    tmp.ctx = c;
    tmp.n = n;
    tmp.pitch_n = round_up(std::max<int64_t>(n, 1), 64);
    tmp.k = p;
    int st = ensure_con_cache(&tmp, 1, con);
    QuadCon q;
    if (st == SPIS_OK) st = constraint_terms_all(c, &tmp, 1, con, n, p, Z, pitch, x0, &q);
    (void)hipStreamSynchronize(c->stream);
    if (tmp.con[0].MZ) (void)hipFree(tmp.con[0].MZ);
    if (tmp.con[0].Mx0) (void)hipFree(tmp.con[0].Mx0);
    if (tmp.ext) (void)hipFree(tmp.ext);
    if (tmp.Ut) (void)hipFree(tmp.Ut);
    if (st != SPIS_OK) return st;
    *term0 = q.term0;
    std::copy(q.term1.begin(), q.term1.end(), term1);
    std::copy(q.term2.begin(), q.term2.end(), term2);
    return SPIS_OK;
  })
}

// ------------------------------------------------------------------------------------------------
// workspace
// ------------------------------------------------------------------------------------------------
static int get_workspace(spis_context* c, int64_t n, int64_t n_ext, int k, bool sep_z, spis_workspace** out) {
  const int64_t pitch = round_up(std::max<int64_t>(n_ext, 1), 64);
  for (size_t i = 0; i < c->pool.size(); ++i) {
    spis_workspace* ws = c->pool[i];
    if (ws->n == n && ws->pitch == pitch && ws->k == k && ws->sep_z == sep_z) {
      c->pool.erase(c->pool.begin() + i);
      *out = ws;
      return SPIS_OK;
    }
  }
  std::unique_ptr<spis_workspace> ws(new spis_workspace());
  ws->ctx = c;
  ws->n = n;
  ws->pitch = pitch;
  ws->pitch_n = round_up(std::max<int64_t>(n, 1), 64);
  ws->k = k;
  ws->sep_z = sep_z;
  const size_t basis = sizeof(double) * pitch * (k + 1);
  HIP_TRY(hipMalloc(&ws->Q, basis));
  HIP_TRY(hipMemsetAsync(ws->Q, 0, basis, c->stream));
  if (sep_z) {
    HIP_TRY(hipMalloc(&ws->Zb, basis));
    HIP_TRY(hipMemsetAsync(ws->Zb, 0, basis, c->stream));
  } else {
    ws->Zb = ws->Q;
  }
  for (double** p : {&ws->w, &ws->xj, &ws->xj2, &ws->r0, &ws->x0}) {
    HIP_TRY(hipMalloc(p, sizeof(double) * pitch));
    HIP_TRY(hipMemsetAsync(*p, 0, sizeof(double) * pitch, c->stream));
  }
  HIP_TRY(hipMalloc(&ws->ydev, sizeof(double) * (k + 1)));
  *out = ws.release();
  return SPIS_OK;
}

extern "C" int spis_workspace_release(spis_workspace* ws) {
  ABI_GUARD({
    if (!ws) return SPIS_OK;
    spis_context* c = ws->ctx;
    if (c->pool.size() >= 4) {
      (void)hipStreamSynchronize(c->stream);
      free_workspace(c->pool.front());
      c->pool.erase(c->pool.begin());
    }
    c->pool.push_back(ws);
    return SPIS_OK;
  })
}

extern "C" int spis_workspace_iterate(spis_workspace* ws, int32_t i, double* x_out) {
  ABI_GUARD({
    if (!ws || !x_out) return fail(SPIS_ERR_ARG, "null argument");
    spis_context* c = ws->ctx;
    if (i < 0 || i > ws->n_iter_y) return fail(SPIS_ERR_ARG, "iterate %d not available (have %d)", i, ws->n_iter_y);
    if (i == 0) {
      HIP_TRY(launch_copy(ws->n, ws->r0, x_out, c->stream));
    } else {
      const double* y = ws->y_all.data() + static_cast<size_t>(i - 1) * ws->k;
      if (i <= kYArg) {
        HIP_TRY(launch_gemv(ws->n, i, ws->Zb, ws->pitch, y, true, ws->x0, x_out, c->stream));
      } else {
        HIP_TRY(hipStreamSynchronize(c->stream));
        for (int a = 0; a < i; ++a) c->pinned[a] = y[a];
        HIP_TRY(hipMemcpyAsync(ws->ydev, c->pinned, sizeof(double) * i, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(launch_gemv(ws->n, i, ws->Zb, ws->pitch, ws->ydev, false, ws->x0, x_out, c->stream));
      }
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    return SPIS_OK;
  })
}

extern "C" int spis_workspace_basis(spis_workspace* ws, int32_t p, double* Z_host) {
  ABI_GUARD({
    if (!ws || !Z_host || p < 0 || p > ws->k + 1) return fail(SPIS_ERR_ARG, "bad argument");
    spis_context* c = ws->ctx;
    HIP_TRY(hipMemcpy2DAsync(Z_host, sizeof(double) * ws->n, ws->Zb, sizeof(double) * ws->pitch,
                             sizeof(double) * ws->n, p, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return SPIS_OK;
  })
}

extern "C" int spis_workspace_hessenberg(spis_workspace* ws, int32_t p, double* H_host) {
  ABI_GUARD({
    if (!ws || !H_host || p < 0) return fail(SPIS_ERR_ARG, "bad argument");
    if (p > ws->n_iter_y) return fail(SPIS_ERR_ARG, "H has %d columns (asked %d)", ws->n_iter_y, p);
    const int k = ws->k;
    for (int r = 0; r <= p; ++r)
      for (int cc = 0; cc < p; ++cc)
        H_host[static_cast<size_t>(r) * p + cc] = r <= cc + 1 ? ws->H[static_cast<size_t>(cc) * (k + 1) + r] : 0.0;
    return SPIS_OK;
  })
}

extern "C" int spis_workspace_constraint_terms(spis_workspace* ws, int32_t ci, int32_t* p_out, double* term0,
                                               double* term1, double* term2) {
  ABI_GUARD({
    if (!ws || !p_out || !term0 || !term1 || !term2) return fail(SPIS_ERR_ARG, "null argument");
    if (ws->last_con_p == 0 || ci < 0 || ci >= static_cast<int32_t>(ws->last_con.size()))
      return fail(SPIS_ERR_ARG, "no reduced constraint %d (the run had %zu at its last constrained step)", ci,
                  ws->last_con.size());
    const QuadCon& q = ws->last_con[ci];
    *p_out = ws->last_con_p;
    *term0 = q.term0;
    std::copy(q.term1.begin(), q.term1.end(), term1);
    std::copy(q.term2.begin(), q.term2.end(), term2);
    return SPIS_OK;
  })
}

// ------------------------------------------------------------------------------------------------
// the solver
// ------------------------------------------------------------------------------------------------
namespace {

enum Safety { kSafetyNone = -1, kSafetyFalse = 0, kSafetyTrue = 1 };

// Pipeline (one host wait per iteration, GPU never idle while the host solves the LS):
//   stream order  A_0, A_1, U_0, A_2, U_1, A_3, U_2, ...
//   A_j = Arnoldi step j (SpMV + MGS chain + normalise; h column j -> mapped pinned slot j)
//   U_j = update of step j (GEMV x_j = Z y_j + x0, true-residual SpMV; partials -> slot j%2)
// At iteration j the host waits for U_{j-1} (which also covers A_j), reads res_{j-1} (stop test
// of iteration j-1, as solvers.py:296) and h column j, solves LS_j, enqueues U_j and A_{j+2}.
// A_{j+1} was enqueued an iteration earlier, so the GPU works on it during LS_j; a stop or
// breakdown discards at most the speculative A_{j+1}, A_{j+2} (they never touch x / res).
struct Solver {
  spis_context* c;
  spis_matrix* A;
  const spis_solve_opts* o;
  spis_workspace* ws;
  const double* b;
  int64_t n;
  int k;
  int gs;  // SpMV partial count
  int gb;  // BLAS-1 partial count
  std::vector<double> hostq, hostz;
  // A/B switches (the context's, from the environment at its creation): the K2w fold, its
  // temporal window, K2s, and the small-N threshold for K2w at SPIS_OPT_MGS_CHAIN 3 (0: K2q at
  // every N; -1: where K2s fits)
  const bool k2w_fold = c->k2w_fold;
  const int k2w_tw = c->k2w_tw;
  const bool k2w_onepass = c->k2w_onepass;
  const int64_t k2w_small_n = c->k2w_small_n;

  double* Qv(int i) const { return ws->Q + static_cast<int64_t>(i) * ws->pitch; }
  double* Zv(int i) const { return ws->Zb + static_cast<int64_t>(i) * ws->pitch; }
  // mapped pinned layout: [k slots of (k+2) h values][2 residual-partial slots][y staging]
  size_t hoff(int j) const { return static_cast<size_t>(j) * (k + 2); }
  size_t roff(int j) const { return static_cast<size_t>(k) * (k + 2) + static_cast<size_t>(j & 1) * kSpmvGrid; }
  size_t yoff() const { return static_cast<size_t>(k) * (k + 2) + 2 * kSpmvGrid; }
  size_t flag_off() const { return yoff() + kMaxK + 8; }  // completion flag word (beta at +kMaxK)
  size_t seq_off(int j) const { return yoff() + kMaxK + 9 + (j & 1); }  // seq to publish for U_j
  size_t pinned_need() const { return yoff() + kMaxK + 16; }
  unsigned long long upd_seq[2] = {0, 0};  // completion sequence number of U_j (slot j & 1)
  unsigned long long* flag_dev() const { return reinterpret_cast<unsigned long long*>(c->pinned_dev + flag_off()); }
  const unsigned long long* seq_dev(int j) const {
    return reinterpret_cast<const unsigned long long*>(c->pinned_dev + seq_off(j));
  }
  void next_seq(int j) {  // before the launch that publishes U_j's residual: arm its slot
    upd_seq[j & 1] = ++c->seq;
    *reinterpret_cast<volatile unsigned long long*>(c->pinned + seq_off(j)) = upd_seq[j & 1];
    // the host read U_{j-2}'s residual from this slot before U_j's producer is enqueued
    *reinterpret_cast<volatile uint64_t*>(c->pinned + roff(j)) = kHSentinel;
  }

  double* xbuf(int j) const { return (j == k - 1 && x_last) ? x_last : (j & 1) ? ws->xj2 : ws->xj; }
  // one GPU: x_{k-1} (only ever a GEMV's output, n rows) goes straight to the caller's x[-1] buffer,
  // which its residual then reads: no copy at the solve's end
  double* x_last = nullptr;
  int launch_dual(int j, int ja, const double* bvec, const LaunchEv* le) {
    HIP_TRY(launch_spmv_dual(A->dual_view(), xbuf(j), bvec, c->partR, Zv(ja), ws->w, Qv(0), c->partA, gs, c->stream,
                             le));
    return SPIS_OK;
  }
  // rows the update GEMV computes.  Several GPUs: n + n_ghost.  Every basis vector z_l's ghost
  // rows hold its owners' values (exchanged before A_l's SpMV) and x0's were exchanged at the
  // start, so x_j's ghost rows come out bitwise equal to the owners' x_j (same y, same order):
  // no per-iteration halo exchange of x_j before its residual SpMV
  int64_t n_gx() const { return (c->dist_on() && !A->nbr.empty()) ? n + A->n_ghost : n; }

  // Speculative update (single GPU, K2q chains): K2q's gatherer writes H[:, j] with H[j+1, j]
  // last, behind a system-scope release, so the host can read the column as soon as A_j's chain
  // ends, instead of waiting for U_{j-1}'s residual (published at the start of A_{j+1}'s chain,
  // one dual SpMV later).  Where the branch of LS_j cannot depend on that residual except through
  // an unconstrained -> constrained switch, the unconstrained y_j is solved then and U_j's GEMV
  // enqueued at once on the side stream: it then runs beside the dual SpMV and A_{j+1}'s chain
  // instead of delaying the dual SpMV that reads x_j.  A constrained LS_j re-enqueues the GEMV
  // with its own y (stream order on the side stream); a stop at j-1 leaves x_j unused (x_j and
  // x_{j-1} live in separate buffers).  Results are identical to the unspeculated path.
  // basis streams nontemporal when the matrix and the k+1 basis vectors overflow the 256 MB
  // Infinity Cache (SPIS_OPT_NT_BASIS 2), so re-streaming the basis leaves the matrix resident
  bool nt_basis_on() const {
    const double ws_bytes = 12.0 * A->nnz + 4.0 * (A->n_rows + 1) + 8.0 * (k + 1) * static_cast<double>(n);
    return c->nt_basis == 1 || (c->nt_basis == 2 && ws_bytes > 256.0 * 1024 * 1024);
  }
  bool lag_chain() const { return (c->mgs_chain == 3 && !fixed_grid(c) && !c->cgs2 && k2q_fits()) || icwy_lag(); }
  // K2q pads an odd n's last pair: its capacity test counts (n + 1) / 2 pairs, as the launch does
  bool k2q_fits() const { return ((n + 1) >> 1) <= (kChainMaxWG - 1) * int64_t(kBlock) * 8; }
  // several GPUs: L mode on the one-reduce MGS (K2w) — every step of the solve takes it (k <=
  // kCgsMax), its coefficient kernel and normalise publish H[:, j] to pinned memory (the
  // normalise's system-scope store of H[j+1, j] last), and its update pass carries U_{j-1}'s GEMV
  bool icwy_lag() const { return icwy_on() && !c->cgs2 && k <= kCgsMax; }
  // K2w: several GPUs (SPIS_OPT_DIST_MGS 1), or one GPU with SPIS_OPT_MGS_CHAIN 4, or 3 beyond
  // K2q's capacity: two passes over the basis per step, the second carrying the update GEMV, in
  // place of K2b + a separate GEMV pass (C5: 826 -> 902 it/s; FX does not fit K2b's registers)
  bool icwy_on() const {
    return c->dist_on() ? c->dist_mgs == 1
                   : (c->mgs_chain == 4 || (c->mgs_chain == 3 && !c->cgs2 && !k2q_fits()) || k2w_small());
  }
  // small N: K2q's per-MGS-step exchanges are latency, not bandwidth; K2s (K2w in one launch over
  // register-resident basis slices) wins wherever it fits (lkdv, N = 100,002: MGS 29.1 -> 18.0 us,
  // 22,272 -> 26,485-28,246 it/s; 200,004: +3-7%; 250,002: +6.6%; gpurun_out/r04k2s), while
  // K2w's two launches lose to K2q from N = 250,000 on (gpurun_out/r04k2ws2): so K2w is taken at
  // small N only where K2s fits (icwy_onepass_max_n(): one resident chunk of 256 per workgroup up
  // to 262,144, two chunks, the second streamed, up to 524,288; C4's 300,006).  Every step must
  // take it (k <= kCgsMax): a later K2q step would read Gram entries (chain_gsub) it never wrote
  bool k2w_small() const {
    const int64_t cap = k2w_small_n >= 0 ? k2w_small_n : icwy_onepass_max_n();
    return c->mgs_chain == 3 && !c->cgs2 && k <= kCgsMax && n <= cap;
  }
  static constexpr uint64_t kHSentinel = 0x7FF4DEAD5EC0FFEEull;  // a signalling NaN no kernel writes
  void arm_hcol(int j) {  // before A_j's chain is enqueued: every slot of H[:, j] (pin_store)
    for (int i = 0; i <= j + 1; ++i) *reinterpret_cast<volatile uint64_t*>(c->pinned + hoff(j) + i) = kHSentinel;
  }
  // true once H[:, j] is complete; false if the stream drained without it (a failed chain)
  int wait_hcol(int j, bool* ok) const {
    // H[j+1, j] is written last in stream order; each entry is its own flag (no ordering between
    // the kernels' system-scope stores), so every slot is checked
    ST_TRY(wait_slot(reinterpret_cast<const uint64_t*>(c->pinned + hoff(j) + j + 1), ok));
    for (int i = 0; i <= j && *ok; ++i) ST_TRY(wait_slot(reinterpret_cast<const uint64_t*>(c->pinned + hoff(j) + i), ok));
    return SPIS_OK;
  }
  // spin until a pinned 8-B slot leaves kHSentinel; false if the stream drained first
  int wait_slot(const uint64_t* w, bool* ok) const {
    const double t0 = now_s();
    for (unsigned spin = 0;; ++spin) {
      if (__atomic_load_n(w, __ATOMIC_ACQUIRE) != kHSentinel) {
        *ok = true;
        return SPIS_OK;
      }
      if ((spin & 4095) == 4095 && now_s() - t0 > 0.02) {
        const hipError_t e = hipStreamQuery(c->stream);
        if (e != hipSuccess && e != hipErrorNotReady) return fail(SPIS_ERR_HIP, "stream: %s", hipGetErrorString(e));
        if (e == hipSuccess && __atomic_load_n(w, __ATOMIC_ACQUIRE) == kHSentinel) {
          *ok = false;
          return SPIS_OK;
        }
      }
      __builtin_ia32_pause();
    }
  }

  // A_j = arnoldi_pre (preconditioner + halo) -> Arnoldi SpMV -> arnoldi_post (MGS + normalise)
  int arnoldi_pre(int j) {  // solvers.py:190
    hipStream_t s = c->stream;
    double* zj = Zv(j);
    if (o->pre_matrix) {
      ST_TRY(spmv_local(c, ws, o->pre_matrix, Qv(j), zj));
    } else if (o->pre_ilu) {
      ST_TRY(ilu_enqueue(o->pre_ilu, Qv(j), zj, s));
    } else if (o->pre_fn) {
      hostq.resize(n);
      hostz.resize(n);
      HIP_TRY(hipMemcpyAsync(hostq.data(), Qv(j), sizeof(double) * n, hipMemcpyDeviceToHost, s));
      HIP_TRY(hipStreamSynchronize(s));
      if (o->pre_fn(o->pre_user, hostq.data(), hostz.data(), n) != 0)
        return fail(SPIS_ERR_CALLBACK, "preconditioner callback failed at iteration %d", j);
      HIP_TRY(hipMemcpyAsync(zj, hostz.data(), sizeof(double) * n, hipMemcpyHostToDevice, s));
    }
    return exchange(c, A, zj);
  }

  // with nontemporal basis loads, the first basis vectors (which every later step re-reads) and x0
  // keep ordinary loads while they fit the Infinity Cache beside the matrix and ~6 working vectors
  // (C3: 6 of them; chain mean 43.0 -> 42.4 us, the dual unchanged at 36.0 us; 10 evicted part of
  // the matrix: dual 38.4 us; gpurun_out/r04ab1)
  int chain_tw(bool nt) const {
    if (!nt) return 0;
    const double mat = 12.0 * A->nnz + 4.0 * (A->n_rows + 1), vec = 8.0 * static_cast<double>(n);
    const double room = 256.0 * 1024 * 1024 - mat - 6.0 * vec;
    return room <= 0.0 ? 0 : static_cast<int>(std::min(6.0, std::floor(room / vec)));
  }

  // (xpart, x_out, done): the first MGS step also reduces the previous update's residual partials
  // into host memory and carries that update's completion event (single GPU, fused path)
  // (yx, jx): K2q only — the chain also computes U_jx's GEMV x_jx = Z[:, :jx+1] yx + x0 (L mode)
  int arnoldi_post(int j, const double* xpart = nullptr, double* x_out = nullptr,
                   unsigned long long* flag = nullptr, const unsigned long long* seq = nullptr,
                   const double* yx = nullptr, int jx = -1) {
    if (c->cgs2 && j + 1 <= kCgsMax) return arnoldi_post_cgs2(j, xpart, x_out, flag, seq);
    if (icwy_on() && j + 1 <= kCgsMax) return arnoldi_post_icwy(j, xpart, x_out, flag, seq, yx, jx);
    hipStream_t s = c->stream;
    c->prof_iter = j;
    ST_TRY(allreduce(c, c->partA, gs));
    double* hcol = c->pinned_dev + hoff(j);  // the kernels write H[:, j] straight to host memory
    ProfEv pm(c, SPIS_PROF_MGS);  // start on the first MGS step, stop on the normalise
    const LaunchEv e_first = pm.first();
    const LaunchEv e_last = pm.last();
    const bool agg = c->mgs_chain >= 2;
    // K2q (mode 3): the pipelined chain, while it fits K2p's register slices (K2b beyond)
    // (never under CGS2: its steps j + 1 <= kCgsMax write no Gram entries G(m, m-1), G(m, m-2), so a
    // later K2q step would read stale ones; those steps take K2p with the aggregator instead)
    double* gsub = (c->mgs_chain == 3 && !c->cgs2) ? c->chain_gsub : nullptr;
    // nontemporal basis loads when the matrix and the basis overflow the 256 MB Infinity Cache:
    // the chain then leaves the matrix resident for the next SpMV (C3: dual SpMV 49 -> 42 us,
    // chain +1-2 us, +2.9%; C4, whose working set fits, measured 1% slower with them)
    const double ws_bytes = 12.0 * A->nnz + 4.0 * (A->n_rows + 1) + 8.0 * (k + 1) * static_cast<double>(n);
    const bool nt_chain = c->nt_basis == 1 || (c->nt_basis == 2 && ws_bytes > 256.0 * 1024 * 1024);
    if (!fixed_grid(c) && c->mgs_chain && mgs_chain_fits(n, agg)) {  // K2p: the chain in one launch
      const LaunchEv both{e_first.start, e_last.stop};
      if (lag_chain()) arm_hcol(j);
      const int px = (gsub && yx) ? jx + 1 : 0;
      HIP_TRY(launch_mgs_chain(n, ws->w, ws->Q, ws->pitch, j, c->partA, gs, hcol, c->chain_gran, c->chain_epoch,
                               c->chain_err_dev, s, &both, xpart, gs, x_out, flag, seq, agg, nt_chain, gsub, yx, px,
                               ws->x0, px > 0 ? xbuf(jx) : nullptr, chain_tw(nt_chain)));
      return SPIS_OK;
    }
    if (yx) return fail(SPIS_ERR_STATE, "fused update GEMV without the pipelined chain");
    double* src = c->partA;
    double* dst = c->partB;
    int n_in = gs;
    for (int i = 0; i <= j; ++i) {
      const double* qn = i < j ? Qv(i + 1) : nullptr;
      if (i == 0)
        HIP_TRY(launch_mgs_step(n, ws->w, Qv(i), qn, src, n_in, dst, hcol + i, gb, s, &e_first, xpart, gs, x_out,
                                flag, seq));
      else
        HIP_TRY(launch_mgs_step(n, ws->w, Qv(i), qn, src, n_in, dst, hcol + i, gb, s));
      ST_TRY(allreduce(c, dst, gb));
      std::swap(src, dst);
      n_in = gb;
    }
    HIP_TRY(launch_normalize(n, ws->w, Qv(j + 1), src, n_in, hcol + j + 1, s, gb, &e_last));
    return SPIS_OK;
  }

  // several GPUs, MGS (K2w, kernels.hip): the projections h_l = q_l . w - sum_{m<l} h_m G(l, m)
  // from one pass and one all-reduce (every q_l . w and the newest Gram row), then w -= Q h with
  // the ||w'||^2 partials (the second all-reduce) and the normalise.  Each rank reduces its own
  // partials in a fixed order first, so each all-reduce carries 2 j + 1 doubles (resp. one): the
  // latency of a few bytes, not of a kRedGrid-long partial array per dot.
  int arnoldi_post_icwy(int j, const double* xpart, double* x_out, unsigned long long* flag,
                        const unsigned long long* seq, const double* yx = nullptr, int jx = -1) {
    hipStream_t s = c->stream;
    c->prof_iter = j;
    if (icwy_lag()) arm_hcol(j);
    // U_{j-2}'s residual (L mode): partials all-reduced, then reduced and published.  On several
    // GPUs partR sits right behind the dot vector d, so one all-reduce carries both (3 collectives
    // per Arnoldi step instead of 4).  Either way the residual is reduced and published by the
    // update kernel's workgroup 0, after the dot pass (no finalize launch: the host's next need is
    // H[:, j], published at the end of this step; one rank takes the merged order, the all-reduce
    // being the identity: the self-halo test covers it)
    const bool merged = xpart != nullptr && xpart == c->partR && c->dist_on();
    if (xpart && !merged) ST_TRY(allreduce(c, const_cast<double*>(xpart), gs));
    const int nv = j + 1;
    double* hcol = c->pinned_dev + hoff(j);
    const int gc = fixed_grid(c) ? kRedGrid : static_cast<int>(std::min<int64_t>(kRedGrid, std::max<int64_t>(1, (n + 63) / 64)));
    ProfEv pm(c, SPIS_PROF_MGS);
    const LaunchEv e_first = pm.first(), e_last = pm.last();
    double* d = c->icwy_d;
    const bool nt = nt_basis_on();  // the matrix stays Infinity-Cache resident for the next SpMV
    const int px = (yx && ws->Zb == ws->Q) ? jx + 1 : 0;
    if (yx && px == 0) return fail(SPIS_ERR_STATE, "fused update GEMV needs Z = Q");
    // K2s: one GPU, small N: the whole step in one launch, the basis slices held in registers
    if (!c->dist_on() && k2w_onepass && !c->icwy_spin_off && n <= icwy_onepass_max_n() && n_gx() == n) {
      if (++c->icwy_tag == 0) c->icwy_tag = 1;
      const LaunchEv both{e_first.start, e_last.stop};
      HIP_TRY(launch_icwy_onepass(n, ws->w, Qv(0), ws->pitch, nv, c->icwy_G, hcol, c->icwy_slots, c->icwy_tag,
                                  c->chain_err_dev, s, &both, px, yx, ws->x0, px > 0 ? xbuf(jx) : nullptr, xpart, gs,
                                  x_out, flag, seq));
      return SPIS_OK;
    }
    const int tw = k2w_tw >= 0 ? k2w_tw : chain_tw(nt);
    // (merged: the slack between the dots and partR is zeroed, since the all-reduce sums it too)
    if (k2w_fold && !c->icwy_spin_off) {  // the dots reduced into d by the same launch (no finalize launch)
      if (++c->icwy_tag == 0) c->icwy_tag = 1;
      HIP_TRY(launch_icwy_dot(n, ws->w, Qv(0), ws->pitch, nv, nullptr, gc, s, &e_first, nt, tw, c->icwy_slots,
                              c->icwy_tag, d, merged ? kIcwyROff : 0, c->chain_err_dev));
    } else {
      HIP_TRY(launch_icwy_dot(n, ws->w, Qv(0), ws->pitch, nv, c->icwy_part, gc, s, &e_first, nt, tw));
      HIP_TRY(launch_cgs_finalize(c->icwy_part, gc, 2 * nv - 1, d, nullptr, nullptr, s, merged ? kIcwyROff : 0));
    }
    if (merged) {
      ST_TRY(allreduce(c, d, kIcwyROff + gs));  // [d | slack | partR]; partR reduced by the update
    } else {
      ST_TRY(allreduce(c, d, 2 * nv - 1));
    }
    // the coefficients h (and H[0..j, j]) in the update's prologue; L mode: U_jx's GEMV in the same
    // pass (x_jx = Z y + x0 over the local and ghost rows)
    HIP_TRY(launch_icwy_update(n, ws->w, Qv(0), ws->pitch, nv, d, c->icwy_G, hcol, c->partB, gc, s, nt, px, yx,
                               ws->x0, px > 0 ? xbuf(jx) : nullptr, n_gx(), xpart, gs, x_out, flag, seq, tw));
    // ||w'||^2: the gc partials all-reduced element-wise (8 KB, latency-bound like one double) and
    // summed in fixed order by every normalize workgroup: no finalize launch in between
    ST_TRY(allreduce(c, c->partB, gc));
    HIP_TRY(launch_normalize(n, ws->w, Qv(j + 1), c->partB, gc, hcol + j + 1, s, gb, &e_last));
    return SPIS_OK;
  }

  // opt-in CGS2 (SPIS_OPT_ORTHOG = 1): 3 reductions per step instead of j + 2 (kernels.hip K2c)
  int arnoldi_post_cgs2(int j, const double* xpart, double* x_out, unsigned long long* flag,
                        const unsigned long long* seq) {
    hipStream_t s = c->stream;
    c->prof_iter = j;
    if (xpart) HIP_TRY(launch_finalize(xpart, gs, x_out, 0, s, nullptr, flag, seq));  // U_{j-2}'s residual
    const int nv = j + 1;
    double* hcol = c->pinned_dev + hoff(j);
    double* c1 = c->cgs_c;
    double* c2 = c->cgs_c + kCgsMax;
    // 64-element chunks per workgroup iteration: up to kRedGrid workgroups (the partial slots);
    // fixed on several GPUs so every rank's partial arrays have the same length
    const int gc = fixed_grid(c) ? kRedGrid : static_cast<int>(std::min<int64_t>(kRedGrid, std::max<int64_t>(1, (n + 63) / 64)));
    ProfEv pm(c, SPIS_PROF_MGS);
    const LaunchEv e_first = pm.first(), e_last = pm.last();
    HIP_TRY(launch_cgs_dot(n, ws->w, Qv(0), ws->pitch, nv, c->cgs_part, gc, s, &e_first));
    ST_TRY(allreduce(c, c->cgs_part, static_cast<int64_t>(nv) * gc));
    HIP_TRY(launch_cgs_finalize(c->cgs_part, gc, nv, c1, nullptr, nullptr, s));
    HIP_TRY(launch_cgs_update(n, ws->w, Qv(0), ws->pitch, nv, c1, true, c->cgs_part, gc, s));
    ST_TRY(allreduce(c, c->cgs_part, static_cast<int64_t>(nv) * gc));
    HIP_TRY(launch_cgs_finalize(c->cgs_part, gc, nv, c2, c1, hcol, s));
    HIP_TRY(launch_cgs_update(n, ws->w, Qv(0), ws->pitch, nv, c2, false, c->partB, gc, s));
    ST_TRY(allreduce(c, c->partB, gc));
    HIP_TRY(launch_normalize(n, ws->w, Qv(j + 1), c->partB, gc, hcol + j + 1, s, gb, &e_last));
    return SPIS_OK;
  }

  int enqueue_arnoldi(int j, bool with_chain = true) {  // solvers.py:190-198
    c->prof_iter = j;
    ST_TRY(arnoldi_pre(j));
    {
      ProfEv ps(c, SPIS_PROF_SPMV);
      const LaunchEv le = ps.both();
      HIP_TRY(launch_spmv(A->dual_view(), kEpiDot, Zv(j), ws->w, Qv(0), c->partA, gs, c->stream, &le));
    }
    return with_chain ? arnoldi_post(j) : SPIS_OK;
  }

  // ---- L mode (lag_chain, see the solver loop): A_ja's chain is enqueued one iteration after its
  // SpMV, once H[:, ja-1] is on the host, so that it can carry U_{ja-1}'s GEMV
  // U_j's residual SpMV fused with A_ja's Arnoldi SpMV (the chain follows later: enqueue_chain)
  int enqueue_dual(int j, int ja) {
    ST_TRY(arnoldi_pre(ja));
    next_seq(j);
    c->prof_iter = j;
    ProfEv pd(c, SPIS_PROF_SPMV_DUAL);
    const LaunchEv le = pd.both();
    return launch_dual(j, ja, b, &le);
  }
  // A_ja's chain; jres >= 0: it also reduces U_jres's residual (the dual before it) and publishes
  // it; yx != nullptr: it also computes x_{ja-1} = Z y_{ja-1} + x0
  int enqueue_chain(int ja, int jres, const double* yx) {
    if (jres >= 0) return arnoldi_post(ja, c->partR, c->pinned_dev + roff(jres), flag_dev(), seq_dev(jres), yx, ja - 1);
    return arnoldi_post(ja, nullptr, nullptr, nullptr, nullptr, yx, ja - 1);
  }
  // U_j's GEMV: beside a running chain on the side stream (the main stream waits for it through a
  // stream write / wait on a device word: ~1.5% faster end to end than an event record + wait, and
  // equal to waiting on the GEMV dispatch's own completion event), or in stream order on the main
  // stream
  int enqueue_gemv(int j, int p, const double* y, bool overlap) {
    if (!overlap || p > kYArg) return update_gemv(j, p, y);
    ST_TRY(update_gemv(j, p, y, c->stream2));
    ++c->gemv_seq;
    HIP_TRY(hipStreamWriteValue64(c->stream2, c->gemv_flag, c->gemv_seq, 0));
    HIP_TRY(hipStreamWaitValue64(c->stream, c->gemv_flag, c->gemv_seq, hipStreamWaitValueGte, ~0ull));
    return SPIS_OK;
  }
  // U_j's residual partials (from [U_j res | a_{j+2}]) reduced and published without a chain
  int enqueue_finalize(int j) {
    ST_TRY(allreduce(c, c->partR, gs));
    HIP_TRY(launch_finalize(c->partR, gs, c->pinned_dev + roff(j), 0, c->stream, nullptr, flag_dev(), seq_dev(j)));
    return SPIS_OK;
  }
  // U_j's residual SpMV on its own (no A_{j+2} to pair with) and its host signal
  int enqueue_residual(int j) {
    {
      ProfEv ps(c, SPIS_PROF_SPMV_RES);
      const LaunchEv le = ps.both();
      HIP_TRY(launch_spmv(A->dual_view(), kEpiResNorm, xbuf(j), nullptr, b, c->partR, gs, c->stream, &le));
    }
    next_seq(j);
    ST_TRY(allreduce(c, c->partR, gs));
    HIP_TRY(launch_finalize(c->partR, gs, c->pinned_dev + roff(j), 0, c->stream, nullptr, flag_dev(), seq_dev(j)));
    return SPIS_OK;
  }

  // U_j1's and U_j2's true-residual SpMVs in one launch (the matrix read once; the last two
  // iterates of a solve, which have no Arnoldi SpMV to pair with), both published
  bool res2_ok() const { return !c->dist_on() && A->dual_view().blk_meta != nullptr; }
  int enqueue_residual2(int j1, int j2) {
    {
      ProfEv ps(c, SPIS_PROF_SPMV_RES);
      const LaunchEv le = ps.both();
      HIP_TRY(launch_spmv_pipe(A->dual_view(), 6, xbuf(j1), b, nullptr, c->partR, xbuf(j2), b, nullptr, c->partB, gs,
                               c->stream, &le));
    }
    next_seq(j1);
    next_seq(j2);
    HIP_TRY(launch_finalize2(c->partR, c->partB, gs, c->pinned_dev + roff(j1), c->pinned_dev + roff(j2), c->stream,
                             flag_dev()));
    return SPIS_OK;
  }

  // U_j = update_gemv (x_j = Z y + x0, halo) -> true-residual SpMV -> update_finish (host signal)
  int update_gemv(int j, int p, const double* y, hipStream_t s_gemv = nullptr) {  // :287
    hipStream_t s = s_gemv ? s_gemv : c->stream;
    c->prof_iter = j;
    {
      ProfEv pg(c, SPIS_PROF_GEMV);
      const LaunchEv le = pg.both();
      // several GPUs: over the ghost rows too (n_gx), so x_j's halo needs no exchange
      if (p <= kYArg) {
        // several GPUs: the GEMV runs every iteration beside the distributed MGS; nontemporal basis
        // loads keep the matrix resident there (single GPU: the GEMV rides in K2q, FX)
        HIP_TRY(launch_gemv(n_gx(), p, ws->Zb, ws->pitch, y, true, ws->x0, xbuf(j), s, &le, c->dist_on() && nt_basis_on()));
      } else {
        double* yh = c->pinned + yoff();
        for (int a = 0; a < p; ++a) yh[a] = y[a];
        HIP_TRY(hipMemcpyAsync(ws->ydev, yh, sizeof(double) * p, hipMemcpyHostToDevice, s));
        HIP_TRY(launch_gemv(n_gx(), p, ws->Zb, ws->pitch, ws->ydev, false, ws->x0, xbuf(j), s, &le));
      }
    }
    return SPIS_OK;
  }

  // U_j's true-residual partials go to device memory (partR).  Single GPU: one workgroup reduces
  // them into the host slot roff(j) and publishes upd_seq[j & 1] to the host flag after a
  // system-scope release (the first MGS step of A_{j+2} when fused, else a finalize kernel): no
  // event, marker or completion signal on the stream (each costs 4-7 us, tools/kbench sig).
  // Multi-GPU: the partials all-reduced element-wise (identical on every rank), then the same
  // finalize kernel publishes the sum (no copy-engine blit, 3.7 us, and no event marker)
  int update_comm_finish(int j) {
    ST_TRY(allreduce(c, c->partR, gs));
    next_seq(j);
    HIP_TRY(launch_finalize(c->partR, gs, c->pinned_dev + roff(j), 0, c->stream, nullptr, flag_dev(), seq_dev(j)));
    return SPIS_OK;
  }

  int enqueue_update(int j, int p, const double* y) {  // solvers.py:287,290
    ST_TRY(update_gemv(j, p, y));
    {
      ProfEv ps(c, SPIS_PROF_SPMV_RES);
      const LaunchEv le = ps.both();
      HIP_TRY(launch_spmv(A->dual_view(), kEpiResNorm, xbuf(j), nullptr, b, c->partR, gs, c->stream, &le));
    }
    if (c->dist_on()) return update_comm_finish(j);
    next_seq(j);
    HIP_TRY(launch_finalize(c->partR, gs, c->pinned_dev + roff(j), 0, c->stream, nullptr, flag_dev(), seq_dev(j)));
    return SPIS_OK;
  }

  // U_j and A_ja (ja = j + 2, adjacent in stream order) with their two SpMVs in one launch: U_j's
  // GEMV on the side stream, next to A_{j+1}'s MGS chain (latency-bound, little HBM traffic;
  // multi-GPU: its per-step all-reduces) still running on the main stream; the dual SpMV
  // (multi-GPU: x_j's halo exchange before it) waits for it.  Safe: every reader of x_j's previous
  // contents (the dual of U_{j-1}) finished before the chain that published U_{j-1}'s residual
  // started, and the GEMV's inputs were written before that.
  int enqueue_update_arnoldi(int j, int p, const double* y, int ja) {
    ST_TRY(enqueue_gemv(j, p, y, true));
    ST_TRY(arnoldi_pre(ja));
    if (!c->dist_on()) next_seq(j);
    c->prof_iter = j;
    {
      ProfEv pd(c, SPIS_PROF_SPMV_DUAL);
      const LaunchEv le = pd.both();
      ST_TRY(launch_dual(j, ja, b, &le));
    }
    if (c->dist_on()) {
      ST_TRY(update_comm_finish(j));
      return arnoldi_post(ja);
    }
    return arnoldi_post(ja, c->partR, c->pinned_dev + roff(j), flag_dev(), seq_dev(j));
  }

  // host wait for U_j's residual (which also covers every earlier launch on the stream: its
  // producer starts after them).  The slot was armed by next_seq(j) and is written whole by one
  // system-scope store (kernels.hip pin_store)
  int wait_update(int j) const {
    bool ok = false;
    ST_TRY(wait_slot(reinterpret_cast<const uint64_t*>(c->pinned + roff(j)), &ok));
    if (!ok) return fail(SPIS_ERR_STATE, "update %d drained without publishing its residual", j);
    return SPIS_OK;
  }

  double residual(int j) const {  // ||A x_j - b||, reduced on the device
    return std::sqrt(c->pinned[roff(j)]);
  }
};

}  // namespace

// tools/host_phases.py: a build with -DSPIS_HOST_PHASES (make phases) prints the mean host time
// of spis_solve's phases every 40 calls (the product build compiles the marks away)
#ifdef SPIS_HOST_PHASES
static double g_phase_t[40], g_phase_acc[40];
static int g_phase_calls = 0;
// the iteration marks 20-27 record (SPIS_PHASE_ITER, default 10; marks 30-35: the start-up launches)
static const int g_phase_iter = [] {
  const char* e = std::getenv("SPIS_PHASE_ITER");
  return e ? std::atoi(e) : 10;
}();
#define PHASE(i) (g_phase_t[i] = now_s())
#define PHASE_IF(cond, i) ((cond) ? (void)(g_phase_t[i] = now_s()) : (void)0)
extern "C" double spis_debug_phase_t(int i) { return g_phase_t[i]; }  // the last call's marks
static void phase_report(int np) {  // the first 10 calls (allocations, warm-up) are not counted
  if (++g_phase_calls <= 10) return;
  for (int i = 1; i < np; ++i) g_phase_acc[i] += g_phase_t[i] - g_phase_t[i - 1];
  if (g_phase_calls % 40 == 10) {
    std::fprintf(stderr, "spis_solve phases (us):");
    for (int i = 1; i < np; ++i) std::fprintf(stderr, " %d:%.1f", i, 1e6 * g_phase_acc[i] / (g_phase_calls - 10));
    std::fprintf(stderr, "\n");
  }
}
#define PHASE_ITER g_phase_iter
#else
#define PHASE(i) ((void)0)
#define PHASE_IF(cond, i) ((void)0)
#define PHASE_ITER 10
static void phase_report(int) {}
#endif

extern "C" int spis_solve(spis_context* c, spis_matrix* A, const double* b, const double* x0,
                          const spis_solve_opts* o, spis_solve_out* out, spis_workspace** ws_out) {
  ABI_GUARD({
    PHASE(0);
    if (!c || !A || !b || !x0 || !o || !out || !ws_out) return fail(SPIS_ERR_ARG, "null argument");
    const int k = o->k;
    if (k < 1 || k > kMaxK) return fail(SPIS_ERR_ARG, "k=%d out of range [1,%d]", k, kMaxK);
    if (o->method < SPIS_CGMRES || o->method > SPIS_CGMRES_P) return fail(SPIS_ERR_ARG, "bad method");
    if (o->n_constraints < 0 || (o->n_constraints > 0 && !o->constraints && !o->conls_fn))
      return fail(SPIS_ERR_ARG, "constraints missing");
    if (!out->res_host || !out->y_host || !out->branch_host || !out->events_host || !out->msg_host)
      return fail(SPIS_ERR_ARG, "output arrays missing");
    const int64_t n = A->n_rows;
    if (c->prof) ++c->prof_phase;
    if (o->pre_matrix && o->pre_matrix->n_rows != n) return fail(SPIS_ERR_ARG, "preconditioner size mismatch");
    if (o->pre_ilu && o->pre_ilu->n != n) return fail(SPIS_ERR_ARG, "ILU preconditioner size mismatch");
    if (o->pre_ilu && c->dist_on()) return fail(SPIS_ERR_ARG, "the device ILU preconditioner is single-GPU");
    if (o->pre_ilu && o->pre_ilu->ctx != c) return fail(SPIS_ERR_ARG, "ILU preconditioner of another context");
    if (!!o->pre_matrix + !!o->pre_ilu + !!o->pre_fn > 1) return fail(SPIS_ERR_ARG, "more than one preconditioner");
    for (int i = 0; i < (o->conls_fn ? 0 : o->n_constraints); ++i)
      if (o->constraints[i].M && o->constraints[i].M->n_rows != n)
        return fail(SPIS_ERR_ARG, "constraint %d matrix size mismatch", i);
    HIP_TRY(hipSetDevice(c->device));
    PHASE(1);
    const bool sep_z = o->pre_matrix != nullptr || o->pre_fn != nullptr || o->pre_ilu != nullptr;
    spis_workspace* ws = nullptr;
    ST_TRY(get_workspace(c, n, n + A->n_ghost, k, sep_z, &ws));
    PHASE(2);
    std::unique_ptr<spis_workspace, int (*)(spis_workspace*)> guard(ws, spis_workspace_release);
    // side-stream work (a constrained step's increments beside the chain, a GEMV) reads the
    // workspace and x0 and writes the constraint caches and the pinned slots the next solve arms:
    // it completes before the solve returns on every path, the early exits included (destroyed
    // before the guard hands the workspace back)
    struct SideJoin {
      hipStream_t st;
      ~SideJoin() {
        if (hipStreamQuery(st) == hipErrorNotReady) (void)hipStreamSynchronize(st);
      }
    } side_join{c->stream2};
    ws->steps = 0;
    ws->n_iter_y = 0;
    ws->broke_at_start = false;
    ws->y_all.assign(static_cast<size_t>(k) * k, 0.0);
    ws->H.assign(static_cast<size_t>(k + 1) * k, 0.0);
    ws->last_con.clear();
    ws->last_con_p = 0;
    const bool use_cb = o->conls_fn != nullptr;
    if (!use_cb && o->n_constraints > 0) ST_TRY(ensure_con_cache(ws, o->n_constraints, o->constraints));
    PHASE(3);

    // every solver SpMV runs on the kDualCap row blocks, so the fused and the single launches
    // group their partial sums identically (bit-identical results either way)
    Solver S{c, A, o, ws, b, n, k, spmv_grid(A->dual_view(), fixed_grid(c)), blas_grid(n, fixed_grid(c)), {}, {}};
    ST_TRY(ensure_pinned(c, S.pinned_need()));
    hipStream_t s = c->stream;
    if (!c->dist_on() && out->x_final_dev && out->x_final_dev != b && out->x_final_dev != x0)
      S.x_last = out->x_final_dev;  // (a caller buffer aliasing b or x0 keeps the copy at the end)
    double* stamps = out->stamps_host;  // [0,k) iter start, [k,2k) iter end, [2k,3k) con start, [3k,4k) con end
    const double t_start = now_s();
    PHASE(4);
    for (int i = 0; i < k; ++i) {
      out->branch_host[i] = SPIS_BRANCH_UNCON;
      out->events_host[i] = 0;
      out->msg_host[i] = SPIS_MSG_SUCCESS;
    }

    // r0 = b - A x0 ; beta = ||r0|| ; q0 = r0 / beta      (solvers.py:167-177)
    // copies: x0 into the workspace (zero padding for K2q's pairs, one buffer for every x0 use);
    // x0 into a halo'd buffer only when the SpMV reads ghost entries
    // x0 = 0 (the copy sees no nonzero) on a finite single-rank matrix: the r0 SpMV skips the
    // matrix, r0 = b bit for bit (spmv_pipe_kernel MODE 3)
    // (SPIS_OPT_X0_ZERO_TEST 0: always the full SpMV, the A/B of test_x0_zero_fast_path_bit_identical)
    const bool x0_test = !c->dist_on() && A->n_ghost == 0 && A->all_finite && A->dual_view().blk_meta != nullptr &&
                         c->x0_zero_test;
    if (x0_test) {
      if (!c->x0_flag) {
        HIP_TRY(hipMalloc(&c->x0_flag, sizeof(unsigned)));
        HIP_TRY(hipMemsetAsync(c->x0_flag, 0, sizeof(unsigned), s));
      }
      if (++c->x0_gen == 0) ++c->x0_gen;  // a stale word never equals a new generation
      HIP_TRY(launch_copy_flag(n, x0, ws->x0, c->x0_flag, c->x0_gen, s));
      PHASE(30);
    } else {
      HIP_TRY(launch_copy(n, x0, ws->x0, s));
    }
    const double* xr0 = ws->x0;
    if (A->n_ghost > 0 || c->dist_on()) {
      HIP_TRY(launch_copy(n, x0, ws->xj, s));
      ST_TRY(exchange(c, A, ws->xj));
      xr0 = ws->xj;
      // x0's ghost rows for the update GEMV over n_gx() rows
      if (S.n_gx() > n) HIP_TRY(launch_copy(S.n_gx() - n, ws->xj + n, ws->x0 + n, s));
    }
    HIP_TRY(launch_spmv(A->dual_view(), kEpiR0, xr0, ws->r0, b, c->partA, S.gs, s, nullptr,
                        x0_test ? c->x0_flag : nullptr, c->x0_gen));
    PHASE(31);
    ST_TRY(allreduce(c, c->partA, S.gs));
    double* beta_slot = c->pinned + S.yoff() + kMaxK;
    // beta: the normalize kernel's one system-scope store into pinned memory; the host spins
    // until the slot leaves its sentinel (an event marker here cost ~6 us of GPU idle per solve);
    // several GPUs keep the event (the slot is written after an all-reduce)
    const bool beta_spin = !c->dist_on();
    if (beta_spin) *reinterpret_cast<volatile uint64_t*>(beta_slot) = Solver::kHSentinel;
    HIP_TRY(launch_normalize(n, ws->r0, S.Qv(0), c->partA, S.gs, c->pinned_dev + S.yoff() + kMaxK, s, S.gb));
    if (!beta_spin) HIP_TRY(hipEventRecord(c->ev_gram, s));  // beta in pinned memory (system-scope event)
    PHASE(32);
    // A_0 and A_1 are queued before beta is read: the GPU goes straight on while the host waits.
    // On beta == 0 they ran on q0 = 0 (normalize writes zeros) and are discarded unread.
    // L mode: the solver loop below (lag_chain: K2q chains publish H[:, j] to the host themselves)
    const bool L = S.lag_chain() && c->fuse_spmv;
    if (stamps) stamps[0] = now_s();
    ST_TRY(S.enqueue_arnoldi(0));
    PHASE(33);
    if (!L) HIP_TRY(hipEventRecord(c->ev_arn, s));  // L mode waits for H[:, 0] itself
    if (k > 1) {
      if (stamps) stamps[1] = now_s();
      ST_TRY(S.enqueue_arnoldi(1, !L));  // L: A_1's chain is enqueued at iteration 0
    }
    PHASE(34);
    if (beta_spin) {
      bool ok = false;
      ST_TRY(S.wait_slot(reinterpret_cast<const uint64_t*>(beta_slot), &ok));
      if (!ok) return fail(SPIS_ERR_STATE, "r0 normalisation drained without publishing beta");
    } else {
      ST_TRY(wait_event(c->ev_gram));
    }
    const double beta = *beta_slot;
    PHASE(5);
    int n_res = 0;
    out->res_host[n_res++] = beta;
    int steps = 0;
    int safety = kSafetyNone;
    const double ctol = 1e-12;  // solvers.py:138
    GivensQR qr;
    qr.reset(k, beta);
    std::vector<double> y(k + 1, 0.0), yk(k + 1, 0.0), y0(k + 1, 0.0), ycon(k + 1, 0.0), hcol(k + 2, 0.0);
    std::vector<QuadCon> cons(std::max(o->n_constraints, 0));
    bool have_x = false;   // ws->xj holds x[-1] (else x[-1] = r0)
    int pending = -1;      // iteration whose update U_j is in flight and not yet read
    if (beta == 0.0) {  // x0 solves the system: q0 would be 0/0 (reference: NaNs); report breakdown
      out->events_host[0] |= SPIS_EV_BREAKDOWN;
      ws->broke_at_start = true;
    }
    // L mode.  Stream order  A_0, a_1, [c_1 + U_0 gemv], [U_0 res | a_2], [c_2 + U_1 gemv],
    // [U_1 res | a_3], ...  with a_j = A_j's preconditioner + Arnoldi SpMV, c_j = its MGS chain (K2q).
    // At iteration j the host waits for H[:, j] (c_j's gatherer publishes it: one chain, not one
    // chain plus a dual SpMV, after LS_{j-1}), then enqueues c_{j+1}; when LS_j's branch can
    // depend on res_{j-1} only through the unconstrained -> constrained switch (GMRES: never;
    // CGMRES while safety is None and j < k - 1) y_j is solved first and c_{j+1} computes U_j's
    // GEMV as it streams q_0 .. q_j (no second pass over the basis).  Then it waits for res_{j-1}
    // (reduced and published by c_{j+1}), decides LS_j as the reference does (a constrained LS_j
    // recomputes x_j after c_{j+1}), and enqueues [U_j res | a_{j+2}] (res + finalize at the end).
    std::vector<double> yspec(k);
    int last_x = -1;  // iteration whose x_j is x[-1]
    bool x_host_spec = false;  // x_{k-1} is on its way to out->x_final_host (stream2, ev_xd2)
    out->x_host_ready = 0;
    // L mode: U_{k-2}'s residual held back and read with U_{k-1}'s in one SpMV (the matrix read
    // once) when it cannot stop the run: CGMRES with safety not True at k-2 (solvers.py:296-297)
    // or CGMRES_P; the record order stays res_{k-2}, res_{k-1}
    int deferred = -1;
    bool deferred_queued = false;
    int gram_queued = -1;  // iteration whose constraint reduction is already on the stream
    ConStep gram_step;     // ... and what it enqueued (increments or the full reduction)
    int spec_kkt = -1;     // iteration whose KKT solve already ran (ycon, spec_kr)
    KKTResult spec_kr;
    // L mode: a forced constrained step's reduction (class-form constraints, fused path) is
    // queued ahead of the residual of the iterate before it (queue_gram)
    // the constraints step jc enforces: all of them (CGMRES), clist[:jc] (CGMRES_P, solvers.py:412)
    auto m_of = [&](int jc) { return o->method == SPIS_CGMRES_P ? std::min(jc, o->n_constraints) : o->n_constraints; };
    auto gram_early_ok = [&](int jc) {
      return (o->method == SPIS_CGMRES || o->method == SPIS_CGMRES_P) && !use_cb && m_of(jc) > 0 &&
             fused_con_ok(c, jc + 1, m_of(jc), o->constraints);
    };
    auto queue_gram = [&](int jc, bool side = false) -> int {
      ST_TRY(con_step_enqueue(c, ws, m_of(jc), o->constraints, n, jc + 1, ws->Zb, ws->pitch, ws->x0, &gram_step,
                              side));
      gram_step.gx_p = 0;  // a GEMV request holds for one enqueue
      if (gram_step.poll.empty()) HIP_TRY(hipEventRecord(c->ev_gram, gram_step.st));
      gram_queued = jc;
      return SPIS_OK;
    };
    for (int j = 0; j < k && !ws->broke_at_start; ++j) {
      bool fused = false, col_added = false;
      if (L) {
        bool ok = false;
        PHASE_IF(j == PHASE_ITER, 20);
        ST_TRY(S.wait_hcol(j, &ok));
        PHASE_IF(j == k - 1, 10);
        PHASE_IF(j == PHASE_ITER, 21);
        if (!ok) {  // the chain failed (c->chain_err): reported at the end of the solve
          (void)hipStreamSynchronize(s);
          break;
        }
        const double* hp = c->pinned + S.hoff(j);
        const bool brk = hp[j + 1] == 0.0 && o->method != SPIS_CGMRES_P;  // the run ends below
        if (!brk && j + 1 < k) {
          const double prev = out->res_host[n_res - 1];  // beta at j = 0; res_{j-1} arrives later
          const bool uncon = o->method == SPIS_GMRES ||
                             (o->method == SPIS_CGMRES && safety == kSafetyNone && j < k - 1 &&
                              (j >= 1 || prev > o->contol * o->tol));
          if (uncon && j + 1 <= kYArg && ws->Zb == ws->Q) {
            for (int i = 0; i < j + 2; ++i) hcol[i] = hp[i];
            qr.add_column(j, hcol.data());
            col_added = true;
            qr.solve(j + 1, yspec.data());
            fused = true;
          }
          PHASE_IF(j == PHASE_ITER, 22);
          ST_TRY(S.enqueue_chain(j + 1, j >= 1 ? j - 1 : -1, fused ? yspec.data() : nullptr));
          PHASE_IF(j == PHASE_ITER, 23);
        } else if (brk && j >= 1 && j + 1 < k) {  // no c_{j+1}: U_{j-1}'s residual on its own
          ST_TRY(S.enqueue_finalize(j - 1));
        }
      }
      // L mode, a step that is constrained whatever res_{j-1} says (the forced last step, or
      // safety set, :230): its reduction goes on the stream now, behind c_{j+1} / U_{j-1}'s
      // residual, not after the host has waited for that residual (C3: a 20 us gap before it)
      // (CGMRES_P: every step from j = 1 is constrained, solvers.py:396-401; its increments go beside
      // the chain just queued)
      if (L && gram_queued != j && (o->method == SPIS_CGMRES_P || j == k - 1 || safety != kSafetyNone) &&
          gram_early_ok(j))
        ST_TRY(queue_gram(j, true));
      // ... and when U_{j-1}'s residual cannot stop the run (safety is not True) and the step
      // is not timed, LS_j's KKT solve runs now, while the GPU still works on that residual
      // (it was queued behind this reduction, see the end of the iteration); the result is
      // used unchanged by the constrained branch below
      if (L && gram_queued == j && safety != kSafetyTrue && !o->timing && spec_kkt != j) {
        const double* hp = c->pinned + S.hoff(j);
        if (hp[j + 1] != 0.0) {
          PHASE_IF(j == k - 1, 11);
          ST_TRY(con_step_wait(c, gram_step));
          PHASE_IF(j == k - 1, 12);
          con_step_assemble(c, ws, o->constraints, gram_step, cons.data());  // (gram_step.m constraints)
          PHASE_IF(j == k - 1, 13);
          if (!col_added) {
            for (int i = 0; i < j + 2; ++i) hcol[i] = hp[i];
            qr.add_column(j, hcol.data());
            col_added = true;
          }
          std::fill(y0.begin(), y0.end(), 0.0);
          for (int a = 0; a < j; ++a) y0[a] = yk[a];
          spec_kr = kkt_newton(j + 1, qr.R(), qr.ld(), qr.g(), gram_step.m, cons.data(), y0.data(), ycon.data());
          spec_kkt = j;
          PHASE_IF(j == k - 1, 14);
        }
      }
      PHASE_IF(j == PHASE_ITER, 24);
      ST_TRY(j == 0 ? (L ? SPIS_OK : wait_event(c->ev_arn)) : (deferred == j - 1 ? SPIS_OK : S.wait_update(j - 1)));
      PHASE_IF(j == PHASE_ITER, 25);
      prof_drain(c);
      if (pending >= 0 && pending != deferred) {  // finish iteration j-1: true residual + stop test (:290-297)
        out->res_host[n_res++] = S.residual(pending);
        if (stamps) stamps[k + pending] = now_s();
        pending = -1;
        const double r = out->res_host[n_res - 1];
        const bool stop = o->method == SPIS_GMRES ? (r < o->tol)
                          : o->method == SPIS_CGMRES ? (r < o->tol && safety == kSafetyTrue)
                                                     : false;
        if (stop) break;
      }
      steps = j + 1;  // solvers.py:189
      const double* hp = c->pinned + S.hoff(j);
      for (int i = 0; i < j + 2; ++i) hcol[i] = hp[i];
      for (int i = 0; i < j + 2; ++i) ws->H[static_cast<size_t>(j) * (k + 1) + i] = hcol[i];
      if (hcol[j + 1] == 0.0 && o->method != SPIS_CGMRES_P) {  // :197-202
        out->events_host[j] |= SPIS_EV_BREAKDOWN;
        break;
      }
      if (!col_added) qr.add_column(j, hcol.data());
      const int p = j + 1;
      std::fill(y0.begin(), y0.end(), 0.0);
      for (int a = 0; a < j; ++a) y0[a] = yk[a];  // warm start (:225-227)
      int branch = SPIS_BRANCH_UNCON, ev = 0, msg = SPIS_MSG_SUCCESS;

      bool constrained = false;
      int m_active = 0;
      if (o->method == SPIS_CGMRES) {
        const double prev = out->res_host[n_res - 1];
        constrained = !(prev > o->contol * o->tol && j < k - 1 && safety == kSafetyNone);  // :230
        m_active = o->n_constraints;
      } else if (o->method == SPIS_CGMRES_P) {
        constrained = true;
        m_active = std::min(j, o->n_constraints);  // clist[:j] (:412)
      }

      if (!constrained) {
        if (fused) std::copy(yspec.begin(), yspec.begin() + p, y.begin());  // the same solve
        else qr.solve(p, y.data());
      } else if (use_cb && m_active > 0) {
        // dict-form constraints: the host callback runs the constrained LS (and its fallback)
        std::vector<double> Hc(static_cast<size_t>(p + 1) * p);
        for (int cc = 0; cc < p; ++cc)
          for (int r = 0; r <= p; ++r) Hc[static_cast<size_t>(cc) * (p + 1) + r] = ws->H[static_cast<size_t>(cc) * (k + 1) + r];
        HIP_TRY(hipStreamSynchronize(s));
        if (stamps) stamps[2 * k + j] = now_s();
        int32_t br = SPIS_BRANCH_CON, evc = 0, msc = SPIS_MSG_SUCCESS;
        if (o->conls_fn(o->conls_user, ws, j, p, Hc.data(), beta, y0.data(), y.data(), &br, &evc, &msc) != 0)
          return fail(SPIS_ERR_CALLBACK, "constraint callback failed at iteration %d", j);
        if (stamps) stamps[3 * k + j] = now_s();
        branch = br;
        ev = evc;
        msg = msc;
        if (o->method == SPIS_CGMRES) {
          if (branch == SPIS_BRANCH_CON) safety = kSafetyTrue;
          else if (ev & SPIS_EV_VIOLATION) safety = kSafetyFalse;
        }
        if (branch == SPIS_BRANCH_FALLBACK) qr.solve(p, y.data());
      } else {
        // class-form constraints reduced on the device (:242-247), KKT on the host (:251-255)
        if (stamps) stamps[2 * k + j] = now_s();
        if (m_active > 0 && spec_kkt == j && m_active == gram_step.m) {
          // terms assembled and the KKT solved before res_{j-1} was waited for (above)
        } else if (m_active > 0 && gram_queued == j && m_active == gram_step.m) {
          ST_TRY(con_step_wait(c, gram_step));  // queued before res_{j-1} was waited for (L mode)
          con_step_assemble(c, ws, o->constraints, gram_step, cons.data());
        } else if (m_active > 0) {
          ST_TRY(constraint_terms_all(c, ws, m_active, o->constraints, n, p, ws->Zb, ws->pitch, ws->x0,
                                      cons.data()));
        }
        if (stamps) stamps[3 * k + j] = now_s();
        bool failed = false;
        if (m_active == 0) {
          qr.solve(p, ycon.data());
        } else {
          const KKTResult kr = (spec_kkt == j && m_active == gram_step.m)
                                   ? spec_kr
                                   : kkt_newton(p, qr.R(), qr.ld(), qr.g(), m_active, cons.data(), y0.data(), ycon.data());
          msg = kr.message;
          ws->last_con.assign(cons.begin(), cons.begin() + m_active);
          ws->last_con_p = p;
        }
        bool has_nan = false;
        for (int a = 0; a < p; ++a) has_nan = has_nan || std::isnan(ycon[a]);
        if (o->method == SPIS_CGMRES) {
          if (!o->timing && has_nan) {  // :259-260
            failed = true;
            ev |= SPIS_EV_NAN;
          } else {
            safety = kSafetyTrue;  // :262
            if (!o->timing) {
              double dev = 0.0;  // constraint_checker: signed max from 0 (:14-18)
              for (int i = 0; i < m_active; ++i) dev = std::max(dev, con_value(cons[i], p, ycon.data()));
              if (dev > ctol) {  // :267-269 (the warning there raises AttributeError -> except)
                safety = kSafetyFalse;
                failed = true;
                ev |= SPIS_EV_VIOLATION;
              }
            }
          }
        } else if (has_nan) {  // cgmres_p (:418-424)
          failed = true;
          ev |= SPIS_EV_NAN;
        }
        if (failed) {  // :271-278
          ev |= SPIS_EV_FALLBACK;
          branch = SPIS_BRANCH_FALLBACK;
          msg = SPIS_MSG_SUCCESS;
          qr.solve(p, y.data());
        } else {
          branch = SPIS_BRANCH_CON;
          for (int a = 0; a < p; ++a) y[a] = ycon[a];
        }
      }
      if (msg != SPIS_MSG_SUCCESS) ev |= SPIS_EV_LS_MESSAGE;  // :280-284
      out->branch_host[j] = branch;
      out->events_host[j] |= ev;
      out->msg_host[j] = msg;
      for (int a = 0; a < p; ++a) {
        yk[a] = y[a];
        ws->y_all[static_cast<size_t>(j) * k + a] = y[a];
        out->y_host[static_cast<size_t>(j) * k + a] = y[a];
      }
      ws->n_iter_y = j + 1;
      if (L) {
        // step j+1 constrained whatever res_j says (CGMRES_P; CGMRES once safety is set, :230):
        // its reduction reads z_0 .. z_{j+1}, complete when c_{j+1} (queued above) ends, so it
        // goes on the main stream right behind that chain, ahead of U_j's GEMV and a_{j+2}: it
        // runs while the host solves LS_j and is done when the host reaches LS_{j+1} (beside the
        // chain on stream2 it was starved by the persistent SpMV and chain kernels)
        // U_j's GEMV rides in its multidot (the increments read z_0 .. z_{j+1}): no GEMV launch and
        // no side-stream hand-off before [U_j res | a_{j+2}]
        const bool need_gemv = !fused || constrained;
        bool gemv_done = false;
        if (j + 2 < k && gram_queued != j + 1 && (o->method == SPIS_CGMRES_P || safety != kSafetyNone) &&
            gram_early_ok(j + 1)) {
          gram_step.gx_p = need_gemv && p <= kYArg ? p : 0;
          gram_step.gx_y = y.data();
          gram_step.gx_out = S.xbuf(j);
          ST_TRY(queue_gram(j + 1));
          gemv_done = gram_step.gx_done;
        }
        // x_j: from c_{j+1} (fused), else a GEMV beside c_{j+1} on the side stream, or after it
        // on the main stream when c_{j+1} computed x_j from the speculative unconstrained y_j
        PHASE_IF(j == k - 1, 15);
        if (need_gemv && !gemv_done) ST_TRY(S.enqueue_gemv(j, p, y.data(), !fused && j + 1 < k));
        PHASE_IF(j == k - 1, 16);
        // x_{k-1} (the caller's buffer) to the caller's host buffer on the side stream, under the
        // last residual SpMV; used when x_{k-1} is x[-1] (below)
        if (j == k - 1 && need_gemv && !gemv_done && out->x_final_host && S.x_last && !c->dist_on()) {
          HIP_TRY(hipEventRecord(c->ev_xd, s));
          HIP_TRY(hipStreamWaitEvent(c->stream2, c->ev_xd, 0));
          HIP_TRY(hipMemcpyAsync(out->x_final_host, S.x_last, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream2));
          HIP_TRY(hipEventRecord(c->ev_xd2, c->stream2));
          x_host_spec = true;
        }
        if (j + 2 < k) {
          if (stamps) stamps[j + 2] = now_s();
          PHASE_IF(j == PHASE_ITER, 26);
          ST_TRY(S.enqueue_dual(j, j + 2));
          PHASE_IF(j == PHASE_ITER, 27);
        } else {
          // the forced constrained last step's reduction first (its inputs, q_0 .. q_{k-1} and
          // x0, are complete): the host's KKT then runs while the GPU computes this residual
          if (j + 1 == k - 1 && gram_early_ok(j + 1)) ST_TRY(queue_gram(j + 1));
          const bool may_stop = o->method == SPIS_GMRES || (o->method == SPIS_CGMRES && safety == kSafetyTrue);
          if (j == k - 2 && !may_stop && !o->timing && S.res2_ok()) {
            deferred = j;  // paired with U_{k-1}'s below
          } else if (deferred == j - 1 && deferred >= 0) {
            ST_TRY(S.enqueue_residual2(j - 1, j));
            deferred_queued = true;
          } else {
            ST_TRY(S.enqueue_residual(j));
          }
        }
      } else if (j + 2 < k && c->fuse_spmv) {
        if (stamps) stamps[j + 2] = now_s();
        ST_TRY(S.enqueue_update_arnoldi(j, p, y.data(), j + 2));
      } else {
        ST_TRY(S.enqueue_update(j, p, y.data()));
        if (j + 2 < k) {
          if (stamps) stamps[j + 2] = now_s();
          ST_TRY(S.enqueue_arnoldi(j + 2));
        }
      }
      have_x = true;
      last_x = j;
      pending = j;
    }
    PHASE(6);
    // the run reached its last iteration, whose residual is the last work queued (below)
    bool tail_launch = pending != k - 1;
    // x[-1] -> caller's buffer, stream-ordered after the last update (and any speculative
    // Arnoldi step, which never touches xj / r0), then one synchronisation
    // the side-stream copy of x_{k-1} is x[-1] when x_{k-1} is the last iterate and stays in the
    // caller's buffer (no copy below)
    const bool x_host_ok = x_host_spec && !ws->broke_at_start && have_x && last_x == k - 1 &&
                           out->x_final_dev && S.xbuf(last_x) == out->x_final_dev;
    if (out->x_final_dev) {
      if (ws->broke_at_start) {
        HIP_TRY(launch_copy(n, x0, out->x_final_dev, s));
        tail_launch = true;
      } else if (!have_x || S.xbuf(last_x) != out->x_final_dev) {
        HIP_TRY(launch_copy(n, have_x ? S.xbuf(last_x) : ws->r0, out->x_final_dev, s));
        tail_launch = true;
      }
    }
    if (deferred >= 0) {  // U_{k-2}'s residual, on its own if the run ended before U_{k-1}
      if (!deferred_queued) {
        ST_TRY(S.enqueue_residual(deferred));
        tail_launch = true;
      }
      ST_TRY(S.wait_update(deferred));
      out->res_host[n_res++] = S.residual(deferred);
      if (stamps) stamps[k + deferred] = now_s();
    }
    if (pending >= 0 && pending != deferred) {
      ST_TRY(S.wait_update(pending));
      out->res_host[n_res++] = S.residual(pending);
      if (stamps) stamps[k + pending] = now_s();
    }
    PHASE(7);
    // speculative Arnoldi steps finish before x / ws are used
    // (event spin: a blocking synchronize wakes the host up tens of us late, per solve).
    // Not needed when the residual the host has just read was published by the last kernel on
    // the stream and the side stream is idle: every kernel before it has completed (in-order
    // stream), so no H column or residual of this solve can still land in a pinned slot the next
    // solve arms, and everything the caller may read later is stream-ordered (C3: 12 us of GPU
    // idle per solve)
    const bool drained = !tail_launch && !c->dist_on() && !o->pre_ilu && hipStreamQuery(c->stream2) == hipSuccess;
    if (!drained) {
      // a side-stream reduction the run never consumed (queue_gram(j, true), then a stop or a
      // breakdown) still reads ws->Zb / x0 and writes the context's pinned slots: join it as well
      if (hipStreamQuery(c->stream2) != hipSuccess) {  // event spin, as below
        HIP_TRY(hipEventRecord(c->ev_side, c->stream2));
        HIP_TRY(hipStreamWaitEvent(s, c->ev_side, 0));
      }
      HIP_TRY(hipEventRecord(c->ev_gram, s));
      ST_TRY(wait_event(c->ev_gram));
    }
    PHASE(8);
    if (x_host_spec) {  // the side-stream copy has finished (the caller may read or reuse the buffer)
      ST_TRY(wait_event(c->ev_xd2));
      out->x_host_ready = x_host_ok ? 1 : 0;
    }
    prof_drain(c);
    if (o->pre_ilu) ST_TRY(ilu_check(o->pre_ilu));
    if (const unsigned ce = *reinterpret_cast<volatile unsigned*>(c->chain_err)) {  // never on a healthy device
      *c->chain_err = 0;
      // bit 0: a persistent MGS chain (K2p / K2b / K2q); bit 1: a one-reduce hand-off (the K2w
      // dot pass's folded reduction, or K2s).  Each disables the kernels that spin on its own
      // protocol, so the rerun takes launch boundaries instead (K2 launches; K2w's finalize)
      if (ce & 1u) c->mgs_chain = 0;
      if (ce & 2u) c->icwy_spin_off = true;
      return fail(SPIS_ERR_STATE, (ce & 1u) ? "persistent MGS chain: a workgroup never reached an exchange (the chain "
                                              "is now disabled on this context; rerun the solve)"
                                            : "one-reduce MGS (K2w fold / K2s): a workgroup never reached a hand-off "
                                              "(both are now disabled on this context; rerun the solve)");
    }
    if (stamps) {
      stamps[4 * k] = t_start;
      stamps[4 * k + 1] = now_s();
    }
    ws->steps = steps;
    out->steps = steps;
    out->n_res = n_res;
    *ws_out = guard.release();
    PHASE(9);
    phase_report(10);
    return SPIS_OK;
  })
}
