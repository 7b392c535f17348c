/*
 * spis.h — C-ABI of libspis.so, the MI355X-native CGMRES/FGMRES inner loop.
 *
 * This is the drop-in boundary for the hot path of the reference
 * (JamesJackaman/StructurePreservingIterativeSolvers, /root/reference):
 *
 *   spis_solve (method SPIS_CGMRES)   replaces solvers.cgmres    solvers.py:131-323
 *   spis_solve (method SPIS_GMRES)    replaces solvers.gmres     solvers.py:58-127
 *   spis_solve (method SPIS_CGMRES_P) replaces solvers.cgmres_p  solvers.py:328-445
 *   spis_constraint_terms             replaces constraint_container.__init__
 *                                     (class form)               solvers.py:21-40
 *   spis_csr_upload                   replaces the CSR the wrappers hand over
 *                                     (csr_matrix of getValuesCSR, e.g. swe/swe.py:90-91)
 *   spis_spmv / spis_residual_norm    A @ z (solvers.py:191), ||A x - b|| (:290)
 *   spis_dot / spis_nrm2 / spis_axpy  np.dot / norm / y - h q (:194-198)
 *   spis_gemv                         Z @ yk + x0 (solvers.py:287)
 *
 * Conventions:
 *   - every export returns int status (SPIS_OK = 0) and never throws;
 *     spis_last_error() returns a thread-local message for the last failure;
 *   - "_dev" pointers are device (HBM) pointers on the context's device,
 *     "_host" pointers are host memory; sizes are element counts;
 *   - all arithmetic is fp64; CSR indices are int32 (PETSc AIJ via SciPy);
 *   - every call is ordered on the context's HIP stream and returns after the
 *     results it reports are complete (host outputs are valid on return);
 *   - handles are not re-entrant: one host thread per context.
 *
 * Multi-GPU: one process per GPU.  Each process uploads its local rows with
 * columns renumbered [0, n_local) owned, [n_local, n_local + n_ghost) ghosts,
 * plus a halo plan (spis_halo_desc).  After spis_comm_init, dots/norms are
 * all-reduced with RCCL over xGMI and ghosts are exchanged with grouped
 * ncclSend/ncclRecv before every SpMV.
 */
#ifndef SPIS_H
#define SPIS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPIS_ABI_VERSION 1

enum spis_status {
  SPIS_OK = 0,
  SPIS_ERR_ARG = 1,      /* bad argument (shape, null pointer, range)        */
  SPIS_ERR_HIP = 2,      /* HIP runtime error                                */
  SPIS_ERR_RCCL = 3,     /* RCCL error                                       */
  SPIS_ERR_ALLOC = 4,    /* device/host allocation failed                    */
  SPIS_ERR_CALLBACK = 5, /* a host callback (preconditioner/constraint) failed */
  SPIS_ERR_STATE = 6     /* handle used in the wrong state                   */
};

enum spis_method { SPIS_CGMRES = 0, SPIS_GMRES = 1, SPIS_CGMRES_P = 2 };

/* what the least-squares step of iteration j did (solvers.py:230-278) */
enum spis_branch {
  SPIS_BRANCH_UNCON = 0,    /* unconstrained LS (solvers.py:230-235)          */
  SPIS_BRANCH_CON = 1,      /* constrained LS kept (:236-270)                 */
  SPIS_BRANCH_FALLBACK = 2  /* constrained LS failed -> unconstrained (:271-278) */
};

/* per-iteration event bits (the reference's warnings, replayed by the host) */
enum spis_event {
  SPIS_EV_BREAKDOWN = 1 << 0,    /* h[j+1,j] == 0 -> warn + break (:197-202)      */
  SPIS_EV_LS_MESSAGE = 1 << 1,   /* LS exit message not accepted (:280-284); code in msg[] */
  SPIS_EV_NAN = 1 << 2,          /* NaN in constrained solution (:259-260)        */
  SPIS_EV_VIOLATION = 1 << 3,    /* constraint_checker > ctol (:267-269)          */
  SPIS_EV_FALLBACK = 1 << 4      /* fallback warning emitted (:272-273 / :419)    */
};

/* exit-message codes (numbering of scipy SLSQP exit modes, which the
 * reference compares against in solvers.py:280-282) */
enum spis_ls_message {
  SPIS_MSG_SUCCESS = 0,          /* "Optimization terminated successfully"           */
  SPIS_MSG_MORE_EQ = 2,          /* "More equality constraints than independent variables" */
  SPIS_MSG_SINGULAR_C = 6,       /* "Singular matrix C in LSQ subproblem"            */
  SPIS_MSG_ITER_LIMIT = 9        /* "Iteration limit reached"                        */
};

typedef struct spis_context spis_context;
typedef struct spis_matrix spis_matrix;
typedef struct spis_workspace spis_workspace;
typedef struct spis_ilu spis_ilu;

/* ---- library / context ---------------------------------------------------- */
int spis_abi_version(void);
const char* spis_last_error(void);
int spis_device_count(int32_t* count);
int spis_context_create(int32_t device, spis_context** out);
int spis_context_destroy(spis_context* ctx);
int spis_context_synchronize(spis_context* ctx);
/* HIP stream (hipStream_t) the context orders its work on */
int spis_context_stream(spis_context* ctx, void** stream_out);

/* Content digest of a host array (no device needed): the drop-in's upload cache (device.py)
 * re-verifies a cached SciPy matrix's data / indices / indptr with it on every solver call, on
 * a second host thread beside spis_solve.  The bytes are hashed in 1 MiB pieces on up to
 * `threads` threads; the digest does not depend on the thread count. */
int spis_host_hash(const void* data, int64_t bytes, int32_t threads, uint64_t* out);
/* 1 when the host CPU runs the x86-64-v3 code the host least squares is built as (AVX2, FMA,
 * BMI2: Makefile LSQFLAGS), else 0; the Python loader refuses the library on 0 with a rebuild
 * hint instead of an illegal instruction at the first constrained step. */
int spis_host_isa_ok(void);
/* Whether any of `count` host fp64 entries is nonzero: in numpy's truthiness when `bitwise` is 0
 * (-0.0 is zero, NaN is not: the wrappers drop an all-zero constraint vector), any bit set when 1
 * (an x0 of +0.0 entries needs no upload).  Stops at the first nonzero entry; up to `threads`
 * threads. */
int spis_host_nonzero(const double* data, int64_t count, int32_t bitwise, int32_t threads, int32_t* any_out);
/* dst[0 .. bytes) = src[0 .. bytes) on up to `threads` host threads (1 MiB pieces): the drop-in
 * stages a caller's right-hand side into its own page-locked buffer with it, then uploads that
 * buffer asynchronously (device.py: callers' memory is never page-locked). */
int spis_host_copy(void* dst, const void* src, int64_t bytes, int32_t threads);

/* ---- live kernel timing ------------------------------------------------------
 * spis_profile_enable(ctx, period): period > 0 makes spis_solve record HIP
 * events on the context stream around the Arnoldi SpMV, the MGS chain
 * (+ normalise), the GEMV and the true-residual SpMV of every period-th
 * iteration (an event pair costs a few us of queue time, so bench.py samples);
 * totals (ms) and launch counts accumulate until the next call.  period <= 0
 * disables. */
enum spis_prof_kind {
  SPIS_PROF_SPMV = 0,       /* Arnoldi SpMV, solvers.py:191 (standalone launches)          */
  SPIS_PROF_MGS = 1,        /* MGS chain + normalise, :193-198                             */
  SPIS_PROF_GEMV = 2,       /* Z y + x0, :287                                              */
  SPIS_PROF_SPMV_RES = 3,   /* true-residual SpMV + norm, :290 (standalone launches)       */
  SPIS_PROF_SPMV_DUAL = 4,  /* fused: residual SpMV of x_j + Arnoldi SpMV of z_{j+2}       */
  SPIS_PROF_KINDS = 5
};
int spis_profile_enable(spis_context* ctx, int32_t on);
int spis_profile_read(spis_context* ctx, double ms_out[SPIS_PROF_KINDS], int64_t count_out[SPIS_PROF_KINDS]);
/* Standalone timing of the solver's own SpMV launch (its table, walk and grid) for roofline
 * reporting: kind 0 = the Arnoldi SpMV (w = A z + q0.w partials, solvers.py:191), 1 = the fused
 * dual (||A x_j - b||^2 with A z_{j+2}, :290 + :191).  cold = 1 evicts L2 and the 256 MB Infinity
 * Cache (a 1 GiB streaming read) before every launch; *us_out = mean launch time (us) over reps
 * launches, from events carried by the launch itself.  Single GPU, square matrices. */
int spis_spmv_bench(spis_context* ctx, spis_matrix* A, int32_t kind, int32_t cold, int32_t reps, double* us_out);

/* ---- options -------------------------------------------------------------------
 * SPIS_OPT_FUSE_SPMV (default 1): the true-residual SpMV of update j and the Arnoldi SpMV of
 *   step j+2 (adjacent in the pipelined stream) run as one launch reading the matrix once;
 *   results are bit-identical either way.
 * SPIS_OPT_ORTHOG (default 0): 0 = modified Gram-Schmidt (the reference's, solvers.py:193-195);
 *   1 = CGS2, classical Gram-Schmidt with one re-orthogonalisation pass (3 reductions per
 *   Arnoldi step instead of j + 2; the low-synchronisation option of SURVEY §8e; steps with
 *   more than 32 basis vectors fall back to MGS).  Not MGS's arithmetic: opt-in only.
 * SPIS_OPT_CON_GRAM (default 2): how the constraint terms (solvers.py:33-36) are reduced.  2 = the
 *   fused reduction on the f64 matrix cores (p + 1 <= 32): a symmetric constraint matrix from a
 *   slot table of its upper triangle (K7t: G = H + H^T, half the gathers), any other from its CSR
 *   (K7m); 3 = K7m for every matrix; 1 = the fused reduction on the CSR without matrix cores (K7,
 *   also the kernel for 32 < p + 1 <= 64); 0 = the generic path (one SpMM M Z, then a tiled Gram).
 *   C3 (swe energy matrix, p = 30): K7t 122 us, K7m 232 us.
 * SPIS_OPT_MGS_CHAIN (default 3): each Arnoldi step's MGS chain + normalise runs as one persistent
 *   launch exchanging partial dots between workgroups in-launch (single GPU, N <= 2^20); 2 = the
 *   partials are gathered by a dedicated workgroup that holds no slice (beyond 2^20, K2b: only w
 *   in registers, N <= 10.4 M), 1 = by workgroup 0; 0 = one launch per MGS step.  MGS's
 *   arithmetic either way; the partial sums are grouped differently, so results differ from the
 *   per-step launches at roundoff level.  3 = the pipelined chain (K2q): MGS's projections and
 *   updates, each dot product evaluated two steps early by the distributive law (h_m = q_m.w^(m-2)
 *   - h_{m-2} q_m.q_{m-2} - h_{m-1} q_m.q_{m-1}), so three exchanges overlap; roundoff differs
 *   from MGS's.  Beyond K2q's capacity (N > 2^20 - 4096) mode 3 takes mode 4: the one-reduce
 *   two-pass MGS (K2w, the several-GPU kernels: every q_l.w and the newest Gram row in one pass,
 *   the projections by the distributive law, then the update pass, which also forms the previous
 *   iteration's update GEMV); MGS in exact arithmetic, not its rounding; k <= 32.
 * SPIS_OPT_SPMV_PIPE (default 5): the solver's SpMVs (and spis_spmv / spis_residual_norm) run the
 *   software-pipelined row-block kernels (K1p / K1dp); 2 = each XCD's workgroups walk a contiguous
 *   eighth of the row blocks (its share of the gathered vectors stays in its own L2), in slab
 *   order when the upload found one (square matrices whose DoF groups are numbered one after
 *   another: slab_order.h), 7 = 2 on the blocks' natural order, 1 = grid-stride walk, 0 = the
 *   unpipelined kernels (K1 / K1d); 5 = 2 when the table has a slab order or the matrix's val/col
 *   fit the 256 MB Infinity Cache, else 1.  Rows are bit-identical in every mode; the reduction
 *   partials are grouped per workgroup, so scalars (h, residuals) differ between modes at roundoff.
 * SPIS_OPT_NT_BASIS (default 2): the MGS kernels load basis vectors with nontemporal loads, so
 *   re-streaming the basis every Arnoldi step does not evict the matrix from the 256 MB Infinity
 *   Cache before the next SpMV; 2 = when the matrix and the k+1 basis vectors exceed 256 MB,
 *   1 = always, 0 = never.  Results identical.
 * SPIS_OPT_COL16 (default 1): the pipelined SpMV reads the matrix's columns from a 16-bit copy made
 *   at upload when every row block spans <= 4 ranges of 2^14 columns (csrc/col16.h: a 2-bit base
 *   index + 14-bit offset per nonzero, 4 base columns per block): 10 instead of 12 bytes per
 *   nonzero.  1 = when val/col exceed the 256 MB Infinity Cache (C5: dual 470 vs 494 us; a
 *   cache-resident C3 matrix is faster on 32-bit columns, 37.6 vs 39.5 us), 2 = always, 0 = never.
 *   Rows bit-identical.
 * SPIS_OPT_DIST_MGS (default 1): several GPUs (after spis_comm_init), Arnoldi steps with at most
 *   32 basis vectors: MGS's projections in inverse-compact-WY form, h_l = q_l.w - sum_{m<l} h_m
 *   q_l.q_m, from one pass and one all-reduce (every q_l.w and the newest Gram row), then the
 *   update with ||w'||^2 and a second all-reduce: 2 all-reduces per Arnoldi step instead of
 *   MGS's j + 2.  MGS in exact arithmetic (the pipelined single-GPU chain's correction terms with
 *   an unbounded lag); roundoff differs.  0 = one MGS step launch and all-reduce per projection.
 * SPIS_OPT_SLAB_KEY (default 1): read at spis_csr_upload.  1 = within a slab the row blocks
 *   follow their rows' mean position in the slab's dominant DoF group (slab_order.h), so the
 *   slab's DoF groups are walked side by side and each XCD gathers an x line about once; 0 = the
 *   groups one after another inside a slab (round 2's order).  Rows bit-identical; reduction
 *   partials grouped differently (roundoff).
 * Variants measured slower and removed from the library (round 4): hipGraph replay of the Arnoldi
 *   step, the early constraint reduction on a third stream, the nontemporal / 4-waves-per-SIMD /
 *   buffer-descriptor / thread-major-column / two-deep / SELL-64 SpMV kernels (now
 *   tools/spmv_variants.hip), 32-slot K7t blocks, the sliced-ELL and chunk-staged K7 Gram kernels;
 *   DESIGN.md §3 keeps their measurements. */
enum spis_option {
  SPIS_OPT_FUSE_SPMV = 1,
  SPIS_OPT_ORTHOG = 4,
  SPIS_OPT_CON_GRAM = 5,
  SPIS_OPT_MGS_CHAIN = 6,
  SPIS_OPT_SPMV_PIPE = 8,
  SPIS_OPT_NT_BASIS = 10,
  SPIS_OPT_COL16 = 11,
  SPIS_OPT_DIST_MGS = 12,
  SPIS_OPT_SLAB_KEY = 16,
  /* A/B switches of parity tests (each is bitwise-neutral; the default 1 is the fast form): the
   * constraint terms from cached increments (0 = the full reduction at every constrained step),
   * the x0 = 0 test that skips the r0 SpMV's matrix read (0 = always the full SpMV), and the
   * pipelined basis transpose of K7t (0 = the one-tile-at-a-time kernel).  Each starts from the
   * environment variable of the same name (SPIS_GRAM_INC, SPIS_X0_ZERO_TEST,
   * SPIS_TRANSPOSE_PIPE) read once when the context is created. */
  SPIS_OPT_GRAM_INC = 17,
  SPIS_OPT_X0_ZERO_TEST = 18,
  SPIS_OPT_TRANSPOSE_PIPE = 19,
  /* A/B switches of the one-reduce MGS (K2w / K2s; each from its environment variable at context
   * creation, SPIS_K2W_*): the small-N threshold below which mode 3 takes K2s (-1 = where K2s
   * fits, 0 = K2q at every N), the dots' fold into the dot pass (1 = on), the nontemporal window
   * (-1 = auto) and the one-launch K2s (1 = on). */
  SPIS_OPT_K2W_SMALL_N = 20,
  SPIS_OPT_K2W_FOLD = 21,
  SPIS_OPT_K2W_TW = 22,
  SPIS_OPT_K2W_ONEPASS = 23,
  /* Output stores (bitwise-neutral; PROCESS-WIDE, every context): a mask of the kernels that store
   * their output vectors write-through (sc1) rather than write-back, so a kernel boundary has
   * fewer dirty L2 lines to write back: 1 the MGS chain K2q (default), 2 the SpMVs, 4 the
   * constraint transpose / update GEMV / x0 copy, 8 the one-reduce MGS update pass and the
   * normalise.  Starts from SPIS_STORE_WT when the first context is created. */
  SPIS_OPT_STORE_WT = 24
};
int spis_set_option(spis_context* ctx, int32_t option, int64_t value);

/* ---- multi-GPU (RCCL over xGMI) ----------------------------------------------
 * rank 0 creates the id (128 bytes), the host side broadcasts it (e.g. over
 * torch.distributed), every rank calls spis_comm_init. */
int spis_comm_unique_id(uint8_t id_out[128]);
int spis_comm_init(spis_context* ctx, int32_t nranks, int32_t rank, const uint8_t id[128]);
int spis_comm_allreduce_sum(spis_context* ctx, double* buf_dev, int64_t count);
int spis_comm_barrier(spis_context* ctx);
/* The rank count of the context's communicator as the transport itself reports it: RCCL's
 * ncclCommCount for spis_comm_init, the count given to spis_comm_init_host for the host
 * transport (*transport_out 1 = RCCL, 2 = host), 0 ranks / transport 0 with no communicator. */
int spis_comm_size(spis_context* ctx, int32_t* nranks_out, int32_t* transport_out);

/* The same several-rank code path with the collectives done by a host callback instead of RCCL
 * (operands staged through host memory, the stream drained first).  For rehearsing several ranks
 * on one GPU, which RCCL refuses; not a production transport.  The callback returns 0 on success.
 *   SPIS_COLL_ALLREDUCE: buf[0 .. count) summed element-wise over the ranks, in place;
 *   SPIS_COLL_EXCHANGE:  buf[0 .. count) holds send_counts[i] doubles for neighbors[i] (i in
 *                        order, concatenated); recv receives recv_counts[i] doubles from each, in
 *                        the same order. */
enum { SPIS_COLL_ALLREDUCE = 0, SPIS_COLL_EXCHANGE = 1 };
typedef int (*spis_host_coll_fn)(void* user, int32_t op, double* buf, int64_t count, int32_t n_neighbors,
                                 const int32_t* neighbors, const int64_t* send_counts, const int64_t* recv_counts,
                                 double* recv);
int spis_comm_init_host(spis_context* ctx, int32_t nranks, int32_t rank, spis_host_coll_fn fn, void* user);

/* ---- matrices ----------------------------------------------------------------
 * Local CSR rows (n_rows x (n_rows + n_ghost)), host arrays, copied to HBM.
 * The matrix is partitioned into row blocks of <= 2048 merge items (rows +
 * nnz) here (SpMV schedule). */
typedef struct spis_halo_desc {
  int32_t n_ghost;            /* ghost columns appended after the owned ones     */
  int32_t n_neighbors;        /* peer ranks exchanged with                       */
  const int32_t* neighbors;   /* [n_neighbors] peer ranks                        */
  const int32_t* send_counts; /* [n_neighbors] owned entries sent to each peer   */
  const int32_t* send_idx;    /* [sum send_counts] local row ids, grouped by peer */
  const int32_t* recv_counts; /* [n_neighbors] ghosts received from each peer;
                                 ghosts of one peer are contiguous, peers in order */
} spis_halo_desc;

int spis_csr_upload(spis_context* ctx, int64_t n_rows, int64_t n_cols, int64_t nnz,
                    const int32_t* indptr_host, const int32_t* indices_host,
                    const double* data_host, const spis_halo_desc* halo /* NULL = 1 GPU */,
                    spis_matrix** out);
int spis_matrix_destroy(spis_matrix* A);
/* info[0]=n_rows info[1]=n_cols info[2]=nnz info[3]=row blocks info[4]=long-row blocks
 * info[5]=n_ghost info[6]=all values zero (1/0) */
int spis_matrix_info(spis_matrix* A, int64_t info[8]);
/* Several GPUs: declares A (a rank's rows, as uploaded with a halo plan) a row block of a global
 * matrix: col_gid[n_cols] is the global index of each local column (the owned columns first, in
 * the rows' order, then the ghosts) and symmetric != 0 says the global matrix equals its transpose
 * exactly.  The constraint Gram then pairs (r, c) with (c, r) by global index (K7t) on every rank
 * instead of gathering both (K7m).  Replaces nothing in the reference: the global matrix of
 * constraint_container (solvers.py:22-36) is one object there. */
int spis_matrix_set_global(spis_matrix* A, const int64_t* col_gid, int32_t symmetric);

/* ---- device ILU preconditioner (pre.solve of a SuperLU spilu object) -------- */
/* Replaces the host call pre.solve(vec) of solvers.py:152-154 (used at :190) for
 * pre = scipy.sparse.linalg.spilu(A, ...) (swe/TimedSolve.py:23, lkdvRK/Evolve.py:51,
 * lkdvRK/SingleSolve.py:19).  Takes SuperLU's factors Pr A Pc = L U as scipy exposes them
 * (pre.L, pre.U as CSR with sorted columns, pre.perm_r, pre.perm_c) and applies
 *   z = Pc U^{-1} L^{-1} Pr q   (y[perm_r[i]] = q[i]; L y' = y; U v = y'; z[i] = v[perm_c[i]])
 * on the device.  L must be unit lower triangular (a stored diagonal must be 1), U upper
 * triangular with a non-zero diagonal.  Single GPU.  The factorisation itself stays with SuperLU
 * on the host (once per operator, as in the reference). */
int spis_ilu_create(spis_context* ctx, int64_t n, const int32_t* l_rowptr, const int32_t* l_col,
                    const double* l_val, const int32_t* u_rowptr, const int32_t* u_col, const double* u_val,
                    const int32_t* perm_r, const int32_t* perm_c, spis_ilu** out);
/* z = P^{-1} q (device pointers, must not alias); synchronises the context stream */
int spis_ilu_apply(spis_ilu* ilu, const double* q_dev, double* z_dev);
/* info: levels(L), levels(U), blocks(L), blocks(U), steps(L), steps(U), nnz(L strict), nnz(U strict) */
int spis_ilu_info(spis_ilu* ilu, int64_t info[8]);
int spis_ilu_destroy(spis_ilu* ilu);

/* ---- vectors / BLAS-1 primitives (device pointers, n = local length) -------- */
/* spis_malloc: zero-filled block, ordered on the context stream (no host wait); blocks come from
 * a per-context stream-ordered cache.  spis_free returns a block to that cache (it must come
 * from spis_malloc of the same context); blocks are released at spis_context_destroy. */
int spis_malloc(spis_context* ctx, int64_t bytes, void** dev_out);
int spis_free(spis_context* ctx, void* dev);
int spis_memcpy_h2d(spis_context* ctx, void* dst_dev, const void* src_host, int64_t bytes);
int spis_memcpy_d2h(spis_context* ctx, void* dst_host, const void* src_dev, int64_t bytes);
/* Page-locked host memory (hipHostMalloc): the drop-in returns x[-1] in such a buffer (device.py
 * keeps a few per length and recycles them when the caller drops the array), so its download is
 * one DMA at the link's rate instead of a staged pageable copy. */
int spis_host_alloc(int64_t bytes, void** host_out);
int spis_host_free(void* host);
/* Page-lock an existing host range (hipHostRegister) and undo it.  The caller owns the lifetime:
 * unregister before the memory is freed, and never register ranges that share a page with another
 * registration.  (The drop-in does not use it: registering callers' arrays led to intermittent
 * illegal-address faults in later copies through the same pages; it stages through
 * spis_host_alloc buffers with spis_host_copy instead.) */
int spis_host_register(void* host, int64_t bytes);
int spis_host_unregister(void* host);
/* Host -> device copy enqueued on the context stream without waiting (the source must be
 * page-locked: spis_host_alloc or spis_host_register); later work on the stream is ordered
 * after it, and the source must not change until it has run (the next spis_* call that waits). */
int spis_memcpy_h2d_async(spis_context* ctx, void* dst_dev, const void* src_host, int64_t bytes);
/* dst_host[0 .. n) = src_dev[0 .. n) by a copy kernel storing straight into page-locked host
 * memory (spis_host_alloc / spis_host_register: mapped into the device's address space), then an
 * event spin; any other destination falls back to spis_memcpy_d2h. */
int spis_copy_to_host(spis_context* ctx, double* dst_host, const double* src_dev, int64_t n);

/* y = A x (x must hold n_rows + n_ghost entries; ghosts are exchanged first) */
int spis_spmv(spis_context* ctx, spis_matrix* A, double* x_dev, double* y_dev);
/* out = ||A x - b||_2 (global) */
int spis_residual_norm(spis_context* ctx, spis_matrix* A, double* x_dev, const double* b_dev,
                       double* out_host);
int spis_dot(spis_context* ctx, int64_t n, const double* x_dev, const double* y_dev, double* out_host);
int spis_nrm2(spis_context* ctx, int64_t n, const double* x_dev, double* out_host);
/* y = y - h x  (numpy's y - h*x: product rounded, then subtracted) */
int spis_axpy(spis_context* ctx, int64_t n, double h, const double* x_dev, double* y_dev);
/* x = Z[:, :p] y + x0, Z row-major (p, pitch) */
int spis_gemv(spis_context* ctx, int64_t n, int32_t p, const double* Z_dev, int64_t pitch,
              const double* y_host, const double* x0_dev, double* x_dev);
/* Gram: G (nu x nv, row-major, host) = U^T V for lists of device vectors */
int spis_gram(spis_context* ctx, int64_t n, int32_t nu, const double* const* U_dev_host_list,
              int32_t nv, const double* const* V_dev_host_list, double* G_host);

/* ---- constraints (class form: 1/2 X'MX + v.X + c with X = x0 + Z y) --------- */
typedef struct spis_constraint_desc {
  spis_matrix* M;       /* NULL or all-zero matrix: skipped (mass constraint 0*A) */
  const double* v_dev;  /* [n] or NULL (= 0) */
  double c;
} spis_constraint_desc;

/* term0 (scalar), term1 (p), term2 (p x p row-major) of solvers.py:33-36 for the
 * basis Z[:, :p] (row-major (p, pitch)) */
int spis_constraint_terms(spis_context* ctx, const spis_constraint_desc* con, int64_t n, int32_t p,
                          const double* Z_dev, int64_t pitch, const double* x0_dev,
                          double* term0_host, double* term1_host, double* term2_host);

/* ---- the solver ------------------------------------------------------------ */
/* host preconditioner callback (objects with .solve, solvers.py:152-154):
 * z = P^{-1} q on host arrays of the local length; return 0 on success */
typedef int (*spis_precond_fn)(void* user, const double* q_host, double* z_host, int64_t n);
/* host constrained-LS callback for constraints the library cannot reduce
 * (dict form: solvers.py:27-28,38-40,46,52).  H is (p+1) x p column-major,
 * y0 the warm start (solvers.py:225-227).  The callback writes y_out and
 * *branch_out (SPIS_BRANCH_CON / SPIS_BRANCH_FALLBACK) and *events_out. */
typedef int (*spis_conls_fn)(void* user, spis_workspace* ws, int32_t j, int32_t p, const double* H,
                             double beta, const double* y0, double* y_out, int32_t* branch_out,
                             int32_t* events_out, int32_t* msg_out);

typedef struct spis_solve_opts {
  int32_t method;            /* spis_method                                      */
  int32_t k;                 /* max iterations (Krylov dimension)                */
  double tol;                /* solvers.py:132 (cgmres), :58 (gmres)             */
  double contol;             /* solvers.py:133                                   */
  int32_t timing;            /* solvers.py:136: skip NaN/checker, record stamps  */
  int32_t n_constraints;
  const spis_constraint_desc* constraints;
  spis_matrix* pre_matrix;   /* device preconditioner (pre @ vec, :156-161)       */
  spis_precond_fn pre_fn;    /* host preconditioner (pre.solve, :152-154)         */
  void* pre_user;
  spis_conls_fn conls_fn;    /* dict-form constraints                              */
  void* conls_user;
  spis_ilu* pre_ilu;         /* device ILU apply of pre.solve (spilu), single GPU  */
} spis_solve_opts;

typedef struct spis_solve_out {
  int32_t steps;     /* iterations run (solvers.py:189)                          */
  int32_t n_res;     /* residual norms written: res[0] = ||r0||, then one per step */
  double* res_host;          /* capacity k+1                                    */
  double* y_host;            /* capacity k*k: y of iteration j at y_host + j*k   */
  int32_t* branch_host;      /* capacity k                                      */
  int32_t* events_host;      /* capacity k                                      */
  int32_t* msg_host;         /* capacity k: spis_ls_message of iteration j       */
  double* stamps_host;       /* capacity 4k+2 or NULL: iter start/end, constraint
                                build start/end (seconds), then run start/end   */
  double* x_final_dev;       /* [n] receives x[-1] (device), or NULL             */
  /* [n] page-locked host buffer (spis_host_alloc) or NULL: when the run reaches its last step,
   * x_{k-1} is copied there by DMA on the side stream while the last residual SpMV runs, and
   * x_host_ready is set to 1 when that copy is x[-1]; 0 otherwise (the caller downloads
   * x_final_dev itself) */
  double* x_final_host;
  int32_t x_host_ready;
} spis_solve_out;

/* Runs the solver; *ws_out receives a workspace holding the Krylov basis so
 * that the iterate list x[i] (solvers.py:169,287) can be materialised lazily
 * with spis_workspace_iterate.  Release it with spis_workspace_release. */
int spis_solve(spis_context* ctx, spis_matrix* A, const double* b_dev, const double* x0_dev,
               const spis_solve_opts* opts, spis_solve_out* out, spis_workspace** ws_out);
/* x[i]: i = 0 -> r0 = b - A x0 ; i >= 1 -> Z[:, :i] y_i + x0 */
int spis_workspace_iterate(spis_workspace* ws, int32_t i, double* x_dev_out);
/* Z[:, :p] to host, row-major (p, n) */
int spis_workspace_basis(spis_workspace* ws, int32_t p, double* Z_host);
/* H[:p+1, :p] of the run (solvers.py:181,193-196) to host, row-major (p+1, p);
 * p <= the number of LS steps taken.  With res_host[0] = beta it is the exact
 * small least-squares problem every step j < p solved (diagnostics, parity). */
int spis_workspace_hessenberg(spis_workspace* ws, int32_t p, double* H_host);
/* The reduced class-form constraint ci (solvers.py:33-36) of the run's last
 * constrained step, as the host KKT solve received it: *p_out = that step's p;
 * term1 capacity k, term2 capacity k*k (row-major p x p).  SPIS_ERR_ARG if the
 * run had no such step (dict-form constraints go through the callback). */
int spis_workspace_constraint_terms(spis_workspace* ws, int32_t ci, int32_t* p_out, double* term0,
                                    double* term1, double* term2);
int spis_workspace_release(spis_workspace* ws);

#ifdef __cplusplus
}
#endif
#endif /* SPIS_H */
