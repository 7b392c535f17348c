// kernels.hip — gfx950 (MI355X, CDNA4) kernels of the CGMRES/FGMRES inner loop.
//
// The SpMV, MGS chain, norms and GEMV are HBM-bandwidth bound fp64 work (SpMV
// ~0.17 flop/B, BLAS-1 <= 0.125 flop/B): their levers are coalesced 8/16-B-per-lane
// streams, LDS staging of the irregular SpMV products, enough waves in flight, and
// deterministic reductions whose partials never leave the device.  The one place
// with matrix-shaped work, the constraint Gram U^T M U of the terminal projection
// (K7t / K7m, the default), runs on f64 MFMA (v_mfma_f64_16x16x4).  See DESIGN.md §3.
//
// Reference call sites (solvers.py): SpMV :191 / :167 / :290, MGS :193-195,
// norm + normalise :196-198, GEMV :287, constraint Gram :33-36.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdlib>
#include <type_traits>

#include "kernels.h"

namespace spis {

// ---------------------------------------------------------------------------------------------
// deterministic reductions: wave butterfly (all lanes get the bitwise-same total by
// commutativity of IEEE addition), then a fixed-order sum of the 4 wave totals.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ double block_sum(double v, double* s_wave) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) s_wave[w] = v;
  __syncthreads();
  const double t = ((s_wave[0] + s_wave[1]) + s_wave[2]) + s_wave[3];
  __syncthreads();
  return t;
}

// One 8-B system-scope store into mapped host memory: a host spinning on the slot sees the value
// whole, and needs no fence or separate flag.  The host arms every such slot with a
// signalling-NaN sentinel no kernel writes before the launch that fills it (spis.cpp kHSentinel),
// so the value is its own flag.  (Round 3 stored the value, released with __threadfence_system()
// and then stored a sequence flag: the fence's L2 write-back stalled the publishing wave by
// microseconds, on the critical path of every chain and K2w update that carries a residual.)
__device__ __forceinline__ void pin_store(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), static_cast<unsigned long long>(__double_as_longlong(v)),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// a residual handed to the host: flag != nullptr marks a host-spun slot (pin_store; flag and seq
// are no longer written); without a flag, a plain store (the caller synchronises through an event)
__device__ __forceinline__ void publish(double* out, double v, unsigned long long* flag,
                                        const unsigned long long* seq) {
  (void)seq;
  if (flag != nullptr)
    pin_store(out, v);
  else
    *out = v;
}

// every workgroup reduces the same partial array in the same order -> the same scalar
__device__ __forceinline__ double sum_partials(const double* __restrict__ part, int n, double* s_wave) {
  double v = 0.0;
  for (int i = threadIdx.x; i < n; i += kBlock) v += part[i];
  return block_sum(v, s_wave);
}

// launch with events carried by the dispatch itself when requested (see LaunchEv)
template <typename F, typename... Args>
static void launch_k(F kernel, dim3 g, dim3 b, uint32_t shm, hipStream_t s, const LaunchEv* ev, Args... args) {
  if (ev != nullptr && (ev->start != nullptr || ev->stop != nullptr))
    hipExtLaunchKernelGGL(kernel, g, b, shm, s, ev->start, ev->stop, 0, args...);
  else
    hipLaunchKernelGGL(kernel, g, b, shm, s, args...);
}

// basis-vector loads of the MGS chain: optionally nontemporal, so that re-streaming the basis at
// every Arnoldi step does not evict the matrix from the 256 MB Infinity Cache between two SpMVs
__device__ __forceinline__ double2 ld_basis(const double2* p, bool nt) {
  if (nt) {
    typedef double v2d __attribute__((ext_vector_type(2)));
    const v2d v = __builtin_nontemporal_load(reinterpret_cast<const v2d*>(p));
    return make_double2(v.x, v.y);
  }
  return *p;
}

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
// buffer-descriptor loads / stores: one 32-bit lane offset shared by every element of a thread,
// the element's distance in the scalar offset (no per-element address registers).  The hardware
// range check does not cover the scalar offset: callers predicate every access themselves.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t vec_rsrc(const double* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(p), 0, static_cast<int>(bytes), 0x00020000);
}
__device__ __forceinline__ double2 buf_ld2(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
  return make_double2(__hiloint2double(static_cast<int>(v.y), static_cast<int>(v.x)),
                      __hiloint2double(static_cast<int>(v.w), static_cast<int>(v.z)));
}
__device__ __forceinline__ void buf_st2(__amdgpu_buffer_rsrc_t r, int voff, int soff, double2 d) {
  u32x4_t v;
  v.x = static_cast<unsigned>(__double2loint(d.x));
  v.y = static_cast<unsigned>(__double2hiint(d.x));
  v.z = static_cast<unsigned>(__double2loint(d.y));
  v.w = static_cast<unsigned>(__double2hiint(d.y));
  __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, soff, 0);
}

// Write-through (sc1) stores for a kernel's output vectors.  A kernel boundary writes back every
// line its kernel left dirty in the XCD L2s (≈ B / 6 TB/s, MI355X_MICROARCH.md "boundary"); a
// write-through line is already in memory (and stays cached, clean), so the boundary has nothing
// to write back.  The data and every later read are unchanged.
__device__ __forceinline__ void st_wt(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), static_cast<unsigned long long>(__double_as_longlong(v)),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_out(double* p, double v, bool wt) {
  if (wt)
    st_wt(p, v);
  else
    *p = v;
}
__device__ __forceinline__ void buf_st2_wt(__amdgpu_buffer_rsrc_t r, int voff, double2 d) {
  u32x4_t v;
  v.x = static_cast<unsigned>(__double2loint(d.x));
  v.y = static_cast<unsigned>(__double2hiint(d.x));
  v.z = static_cast<unsigned>(__double2loint(d.y));
  v.w = static_cast<unsigned>(__double2hiint(d.y));
  __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, 0, 16);  // aux 16 = sc1 (write-through)
}

// the store form of the output vectors, a mask (SPIS_STORE_WT): 1 K2q's q_{j+1} and x_j, 2 the
// SpMVs' w, 4 the rest (the transpose's Ut, the GEMV's x, the x0 copy), 8 K2w's update pass and the
// normalise; a set bit = sc1.  Default 1: at C3 K2q 39.9 -> 38.5 us, C3 +1.5%; bits 2 and 4 measured
// no better (the dual SpMV's 8-B sc1 stores cost it 0.3-0.5 us); bit 8 costs K2w's step 62 -> 66 us
// at one rank and 491 -> 526 us at C5 (a streaming pass: its write-back overlaps at the boundary
// anyway), and K2s's 8-B sc1 stores cost it 1.5-1.8 us at C4 (profiles/r06_store_wt_ab.txt)
static int g_store_wt = 1;
void set_store_wt(int mask) { g_store_wt = mask & 15; }
static inline int wt_mgs() { return g_store_wt & 1; }
static inline int wt_k2w() { return (g_store_wt >> 3) & 1; }
static inline int wt_spmv() { return (g_store_wt >> 1) & 1; }
static inline int wt_other() { return (g_store_wt >> 2) & 1; }

// a descriptor over [p, p + 2^31 B) with a wave-uniform base (callers index it with valid offsets)
template <typename T>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t span_rsrc(const T* p) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint64_t u = (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(a >> 32)))) << 32) |
                     static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(a & 0xffffffffu)));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(u), 0, 0x7fffffff, 0x00020000);
}

// ---------------------------------------------------------------------------------------------
// K1: CSR SpMV, row blocks of <= kItemCap merge items (rows + nnz), products staged in LDS.
//
// Phase 1 streams the block's contiguous nnz range [indptr[r0], indptr[r1]) with fully
// coalesced val/col loads (lane i -> element i), gathers x, and writes the ROUNDED product to
// LDS.  Phase 2 gives each row to one thread, which sums its products left to right from 0 —
// exactly SciPy's csr_matvec arithmetic, so y is bit-identical to ``A @ x`` (solvers.py:191).
// A row longer than kNnzCap forms a block of its own and is reduced by the whole workgroup
// (strided partials + fixed-order tree: deterministic, not SciPy's order).
// Workgroups loop over row blocks (grid-stride) so the epilogue leaves <= kSpmvGrid partials.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int swizzled_block(bool swz) {
  const int G = gridDim.x;
  return (swz && (G & 7) == 0) ? (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3) : blockIdx.x;
}

template <int EPI>
__global__ __launch_bounds__(kBlock) void spmv_rowblock_kernel(
    const int32_t* __restrict__ rp, const int32_t* __restrict__ ci, const double* __restrict__ va,
    const int32_t* __restrict__ blk_row, int n_blk, const double* __restrict__ x,
    double* __restrict__ y, const double* __restrict__ aux, double* __restrict__ partials, bool swz) {
  __shared__ double s_prod[kNnzCap];
  __shared__ double s_wave[4];
  double part = 0.0;
  for (int blk = swizzled_block(swz); blk < n_blk; blk += gridDim.x) {
    const int r0 = blk_row[blk];
    const int r1 = blk_row[blk + 1];
    const int nz0 = rp[r0];
    const int nnz = rp[r1] - nz0;
    if (nnz > kNnzCap) {  // one long row (r1 == r0 + 1)
      double acc = 0.0;
      for (int i = nz0 + threadIdx.x; i < nz0 + nnz; i += kBlock) acc += va[i] * x[ci[i]];
      const double sum = block_sum(acc, s_wave);
      if (threadIdx.x == 0) {
        if (EPI == kEpiPlain) y[r0] = sum;
        if (EPI == kEpiDot) { y[r0] = sum; part += aux[r0] * sum; }
        if (EPI == kEpiResNorm) { const double t = sum - aux[r0]; part += t * t; }
        if (EPI == kEpiR0) { const double t = aux[r0] - sum; y[r0] = t; part += t * t; }
      }
      continue;
    }
    // all of the block's val/col loads first (kNnzCap / kBlock per lane, coalesced), then the
    // x gathers, then the rounded products to LDS: maximal loads in flight per lane
    constexpr int kPer = kNnzCap / kBlock;
    int cols[kPer];
    double vals[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int i = threadIdx.x + u * kBlock;
      cols[u] = i < nnz ? ci[nz0 + i] : 0;
      vals[u] = i < nnz ? va[nz0 + i] : 0.0;
    }
    double xs[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) xs[u] = x[cols[u]];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int i = threadIdx.x + u * kBlock;
      if (i < nnz) s_prod[i] = vals[u] * xs[u];
    }
    __syncthreads();
    const int r = r0 + threadIdx.x;
    if (r < r1) {
      const int s = rp[r] - nz0;
      const int e = rp[r + 1] - nz0;
      double sum = 0.0;
      for (int t = s; t < e; ++t) sum += s_prod[t];
      if (EPI == kEpiPlain) y[r] = sum;
      if (EPI == kEpiDot) { y[r] = sum; part += aux[r] * sum; }
      if (EPI == kEpiResNorm) { const double t = sum - aux[r]; part += t * t; }
      if (EPI == kEpiR0) { const double t = aux[r] - sum; y[r] = t; part += t * t; }
    }
    __syncthreads();
  }
  if (EPI != kEpiPlain) {
    const double tot = block_sum(part, s_wave);
    if (threadIdx.x == 0) partials[blockIdx.x] = tot;
  }
}

// ---------------------------------------------------------------------------------------------
// K1d: two SpMVs with the same matrix in one pass — the true residual of update U_j (x1 = x_j:
// ||A x1 - b||^2 partials, solvers.py:290) and the Arnoldi SpMV of step j+2 (x2 = z_{j+2}:
// w = A x2 and q0.w partials, solvers.py:191), adjacent in the pipelined stream order.  val/col
// are read once; each product array and each row sum is exactly K1's (bit-identical rows).  It
// runs on row blocks of <= CAP nnz (kDualCap: two CAP-long product arrays in LDS).
// ---------------------------------------------------------------------------------------------
template <int CAP, int SWZ = 0>
__global__ __launch_bounds__(kBlock) void spmv_dual_kernel(
    const int32_t* __restrict__ rp, const int32_t* __restrict__ ci, const double* __restrict__ va,
    const int32_t* __restrict__ blk_row, int n_blk, const double* __restrict__ x1,
    const double* __restrict__ b, double* __restrict__ part1, const double* __restrict__ x2,
    double* __restrict__ w, const double* __restrict__ q0, double* __restrict__ part2) {
  __shared__ double2 s_p[CAP];  // (residual, Arnoldi) products: one 16-B LDS access each way
  __shared__ double s_wave[4];   // (two separate arrays: 52.8 vs 46.7 us at C3, tools/kbench)
  double pt1 = 0.0, pt2 = 0.0;
  // SWZ (tuning): 1 = XCD-swizzled logical workgroup id, grid-stride; 2 = swizzled id, one
  // contiguous chunk of row blocks per workgroup (each XCD then owns an eighth of the rows)
  const int G = gridDim.x;
  int L = blockIdx.x;
  if (SWZ && (G & 7) == 0) L = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  int b0 = L, b1 = n_blk, bs = G;
  if (SWZ == 2) {
    const int c = (n_blk + G - 1) / G;
    b0 = L * c;
    b1 = min(n_blk, b0 + c);
    bs = 1;
  }
  for (int blk = b0; blk < b1; blk += bs) {
    const int r0 = blk_row[blk];
    const int r1 = blk_row[blk + 1];
    const int nz0 = rp[r0];
    const int nnz = rp[r1] - nz0;
    if (nnz > CAP) {  // one long row (r1 == r0 + 1): K1's workgroup reduction, twice
      double a1 = 0.0, a2 = 0.0;
      for (int i = nz0 + threadIdx.x; i < nz0 + nnz; i += kBlock) {
        a1 += va[i] * x1[ci[i]];
        a2 += va[i] * x2[ci[i]];
      }
      const double s1 = block_sum(a1, s_wave);
      const double s2 = block_sum(a2, s_wave);
      if (threadIdx.x == 0) {
        const double t = s1 - b[r0];
        pt1 += t * t;
        w[r0] = s2;
        pt2 += q0[r0] * s2;
      }
      continue;
    }
    constexpr int kPer = CAP / kBlock;
    int cols[kPer];
    double vals[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int i = threadIdx.x + u * kBlock;
      cols[u] = i < nnz ? ci[nz0 + i] : 0;
      vals[u] = i < nnz ? va[nz0 + i] : 0.0;
    }
    double g1[kPer], g2[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      g1[u] = x1[cols[u]];
      g2[u] = x2[cols[u]];
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int i = threadIdx.x + u * kBlock;
      if (i < nnz) s_p[i] = make_double2(vals[u] * g1[u], vals[u] * g2[u]);
    }
    __syncthreads();
    const int r = r0 + threadIdx.x;
    if (r < r1) {
      const int s = rp[r] - nz0;
      const int e = rp[r + 1] - nz0;
      double s1 = 0.0, s2 = 0.0;
      for (int t = s; t < e; ++t) {
        const double2 pp = s_p[t];
        s1 += pp.x;
        s2 += pp.y;
      }
      const double t = s1 - b[r];
      pt1 += t * t;
      w[r] = s2;
      pt2 += q0[r] * s2;
    }
    __syncthreads();
  }
  const double tot1 = block_sum(pt1, s_wave);
  const double tot2 = block_sum(pt2, s_wave);
  if (threadIdx.x == 0) {
    part1[blockIdx.x] = tot1;
    part2[blockIdx.x] = tot2;
  }
}

// ---------------------------------------------------------------------------------------------
// K1p / K1dp: software-pipelined SpMV on row blocks of <= CAP nnz with a (row start, nz start)
// table.  Per block the unpipelined kernels pay ~5 dependent memory round trips (block table ->
// indptr -> val/col -> x gathers -> indptr/aux of the rows); here the block table is scalar,
// and block i+1's val/col, row bounds and row aux values are loaded while block i's gathers are in
// flight, so a workgroup waits about one memory latency per block.  Each row sum is K1's (left
// to right over the rounded products): rows are bit-identical to K1 / K1d.  MODE 0-3 = a single
// SpMV with K1's epilogue of that number; MODE 4 = K1d's dual (residual of x1, Arnoldi of x2).
// ---------------------------------------------------------------------------------------------
template <int CAP>
struct PipeStage {
  static constexpr int kPer = CAP / kBlock;
  int r0, r1, nz0, nnz;
  int cols[kPer];
  double vals[kPer];
  int rs, re;     // this thread's row bounds relative to nz0 (rows r0 + threadIdx.x)
  double a1, a2;  // the row's aux values (b / q0 / aux)
  int bs0, bs1, bs2, bs3;  // C16: the block's base columns (col16.h; plain ints: the stage must
                          // stay in registers)
};

// C16: column = base[k] + offset of a 16-bit entry (k = the top 2 bits)
__device__ __forceinline__ int col16_decode(unsigned v, int b0, int b1, int b2, int b3) {
  const unsigned k = v >> 14;
  const int base = (k & 2u) ? ((k & 1u) ? b3 : b2) : ((k & 1u) ? b1 : b0);
  return base + static_cast<int>(v & 0x3fffu);
}

// block lb of the table (entries lb * ms, lb * ms + 1: ms = 1 consecutive starts, 2 (start, end)
// pairs); C16: the columns from the 16-bit copy and the block's bases base[lb]
template <int CAP, int MODE, bool C16 = false>
__device__ __forceinline__ void pipe_load(PipeStage<CAP>& st, const int2* __restrict__ meta, int lb, int ms,
                                          const int32_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                          const uint16_t* __restrict__ c16, const int4* __restrict__ base,
                                          const double* __restrict__ va, const double* __restrict__ aux1,
                                          const double* __restrict__ aux2) {
  const int2 m0 = meta[lb * ms];
  const int2 m1 = meta[lb * ms + 1];
  if (C16) {
    const int* bp = reinterpret_cast<const int*>(base) + 4 * lb;
    st.bs0 = bp[0];
    st.bs1 = bp[1];
    st.bs2 = bp[2];
    st.bs3 = bp[3];
  }
  st.r0 = m0.x;
  st.r1 = m1.x;
  st.nz0 = m0.y;
  st.nnz = m1.y - m0.y;
  if (st.nnz > CAP) return;  // long row: read directly by the workgroup-wide path
#pragma unroll
  for (int u = 0; u < PipeStage<CAP>::kPer; ++u) {
    const int i = threadIdx.x + u * kBlock;
    if (C16) {
      st.cols[u] = i < st.nnz ? c16[st.nz0 + i] : 0;  // raw: decoded at the gathers, so the prefetch
                                                      // stays in flight (0 decodes to a column of the block)
      st.vals[u] = i < st.nnz ? va[st.nz0 + i] : 0.0;
    } else {
      st.cols[u] = i < st.nnz ? ci[st.nz0 + i] : 0;
      st.vals[u] = i < st.nnz ? va[st.nz0 + i] : 0.0;
    }
  }
  const int r = st.r0 + threadIdx.x;
  if (r < st.r1) {
    st.rs = rp[r] - st.nz0;
    st.re = rp[r + 1] - st.nz0;
    if (MODE != kEpiPlain) st.a1 = aux1[r];
    if (MODE >= 4) st.a2 = aux2[r];
  } else {
    st.rs = st.re = 0;
  }
}

__device__ __forceinline__ void block_walk(int n_blk, int walk, int& b0, int& b1, int& bs) {
  const int G = gridDim.x;
  if (walk >= 1 && (G & 7) == 0) {
    const int x = blockIdx.x & 7;
    b0 = static_cast<int>((static_cast<int64_t>(n_blk) * x) >> 3) + (blockIdx.x >> 3);
    b1 = static_cast<int>((static_cast<int64_t>(n_blk) * (x + 1)) >> 3);
    bs = G >> 3;
  } else {
    b0 = blockIdx.x;
    b1 = n_blk;
    bs = G;
  }
}

// x1/aux1/y1/part1: the single SpMV (MODE 0-3) or the residual half of the dual (aux1 = b);
// x2/aux2 (= q0)/y2 (= w)/part2: the dual's Arnoldi half (MODE 4); MODE 6: two true residuals
// (x1 and x2 against aux1 = aux2 = b, ||.||^2 partials to part1 / part2, nothing stored)
// C16: columns from the 16-bit copy (c16, per-block bases; col16.h)
// (variants measured and not adopted — nontemporal stream, 4 waves per SIMD, buffer descriptors,
// thread-major columns, two-deep pipeline, SELL-64 — live in tools/spmv_variants.hip)
template <int CAP, int MODE, bool C16 = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, C16 ? 3 : 8))) void spmv_pipe_kernel(
    const int32_t* __restrict__ rp, const int32_t* __restrict__ ci, const double* __restrict__ va,
    const int2* __restrict__ meta, int n_blk, int walk, const double* __restrict__ x1,
    const double* __restrict__ aux1, double* __restrict__ y1, double* __restrict__ part1,
    const double* __restrict__ x2, const double* __restrict__ aux2, double* __restrict__ y2,
    double* __restrict__ part2, const uint16_t* __restrict__ c16, const int4* __restrict__ base,
    const unsigned* __restrict__ zf, unsigned gen, int wt) {
  constexpr bool DUAL = MODE == 4 || MODE == 6;
  constexpr int kPer = PipeStage<CAP>::kPer;
  // products at padded index i + i/16: one thread per row reads its row left to right, and rows
  // of 16 entries (swe's edge rows) would otherwise put a wave's lanes 256 B apart, all in one
  // LDS bank group; the pad staggers them
  __shared__ typename std::conditional<DUAL, double2, double>::type s_p[CAP + CAP / 16];
  __shared__ double s_wave[4];
  double pt1 = 0.0, pt2 = 0.0;
  int b0, b1, bs;
  block_walk(n_blk, walk, b0, b1, bs);
  const int ms = walk == 2 ? 2 : 1;  // walk 2: (start, end) pair per block (an ordered table)
  if (MODE == kEpiR0 && zf != nullptr && *zf != gen) {
    // r0 = b - A x0 with x0 all zeros (copy_flag_kernel saw no nonzero) and A finite (the host
    // checked at upload): every product is +-0, every row sum +0 (0.0 + (-0.0) = +0.0), so
    // r = b - 0.0 = b bit for bit; the same walk and row -> thread mapping as below, so the
    // ||r||^2 partials are the full path's too.  Skips the matrix and the gathers.
    for (int blk = b0; blk < b1; blk += bs) {
      const int2 m0 = meta[blk * ms];
      const int2 m1 = meta[blk * ms + 1];
      if (m1.y - m0.y > CAP) {  // one long row: thread 0, as the full path (block_sum of zeros = +0)
        if (threadIdx.x == 0) {
          const double t = aux1[m0.x] - 0.0;
          y1[m0.x] = t;
          pt1 += t * t;
        }
        continue;
      }
      const int r = m0.x + threadIdx.x;
      if (r < m1.x) {
        const double t = aux1[r] - 0.0;
        y1[r] = t;
        pt1 += t * t;
      }
    }
    const double tot1 = block_sum(pt1, s_wave);
    if (threadIdx.x == 0) part1[blockIdx.x] = tot1;
    return;
  }
  // one block: cur's products and row sums, nxt (block nb) loaded meanwhile.  The loop below
  // alternates two stages (no stage copy at the back edge: the copy's register moves spilled)
  auto step = [&](PipeStage<CAP>& cur, PipeStage<CAP>& nxt, int blk) __attribute__((always_inline)) {
    const int nb = blk + bs;
    if (cur.nnz > CAP) {  // one long row (r1 == r0 + 1): K1's workgroup reduction
      double s1 = 0.0, s2 = 0.0;
      {
        double acc1 = 0.0, acc2 = 0.0;
        for (int i = cur.nz0 + threadIdx.x; i < cur.nz0 + cur.nnz; i += kBlock) {
          const int c = C16 ? col16_decode(c16[i], cur.bs0, cur.bs1, cur.bs2, cur.bs3) : ci[i];
          acc1 += va[i] * x1[c];
          if (DUAL) acc2 += va[i] * x2[c];
        }
        s1 = block_sum(acc1, s_wave);
        if (DUAL) s2 = block_sum(acc2, s_wave);
      }
      if (threadIdx.x == 0) {
        const int r0 = cur.r0;
        if (DUAL) {
          const double t = s1 - aux1[r0];
          pt1 += t * t;
          if (MODE == 6) {
            const double t2 = s2 - aux2[r0];
            pt2 += t2 * t2;
          } else {
            y2[r0] = s2;
            pt2 += aux2[r0] * s2;
          }
        }
        if (MODE == kEpiPlain) y1[r0] = s1;
        if (MODE == kEpiDot) { y1[r0] = s1; pt1 += aux1[r0] * s1; }
        if (MODE == kEpiResNorm) { const double t = s1 - aux1[r0]; pt1 += t * t; }
        if (MODE == kEpiR0) { const double t = aux1[r0] - s1; y1[r0] = t; pt1 += t * t; }
      }
      nxt.nnz = 0;
      if (nb < b1) pipe_load<CAP, MODE, C16>(nxt, meta, nb, ms, rp, ci, c16, base, va, aux1, aux2);
      return;
    }
    // this block's gathers first, then the next block's loads: the gathers' vmcnt wait does not
    // include the prefetch, and the prefetch is in flight through the LDS phase below
    double g1[kPer], g2[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int c = C16 ? col16_decode(cur.cols[u], cur.bs0, cur.bs1, cur.bs2, cur.bs3) : cur.cols[u];
      g1[u] = x1[c];
      if (DUAL) g2[u] = x2[c];
    }
    nxt.nnz = 0;
    if (nb < b1) pipe_load<CAP, MODE, C16>(nxt, meta, nb, ms, rp, ci, c16, base, va, aux1, aux2);
    // entry i = tid + u kBlock sits at i + i/16 = (tid + tid/16) + u (kBlock + kBlock/16): one base
    // register and an immediate offset per u (the compiler's own form of i + i/16 kept 8 addresses
    // live)
    const int pbase = threadIdx.x + (threadIdx.x >> 4);
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int i = threadIdx.x + u * kBlock;
      if (i < cur.nnz) {
        if constexpr (DUAL)
          s_p[pbase + u * (kBlock + kBlock / 16)] = make_double2(cur.vals[u] * g1[u], cur.vals[u] * g2[u]);
        else
          s_p[pbase + u * (kBlock + kBlock / 16)] = cur.vals[u] * g1[u];
      }
    }
    __syncthreads();
    const int r = cur.r0 + threadIdx.x;
    if (r < cur.r1) {
      double s1 = 0.0, s2 = 0.0;
      // LDS reads in flight in groups, then the adds in row order (the sum is still left to right)
      int t = cur.rs;
      for (; t + 8 <= cur.re; t += 8) {
        if constexpr (DUAL) {
          double2 pp[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) pp[u] = s_p[t + u + ((t + u) >> 4)];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            s1 += pp[u].x;
            s2 += pp[u].y;
          }
        } else {
          double pp[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) pp[u] = s_p[t + u + ((t + u) >> 4)];
#pragma unroll
          for (int u = 0; u < 8; ++u) s1 += pp[u];
        }
      }
      for (; t + 4 <= cur.re; t += 4) {
        if constexpr (DUAL) {
          const double2 p0 = s_p[t + (t >> 4)], p1 = s_p[t + 1 + ((t + 1) >> 4)];
          const double2 p2 = s_p[t + 2 + ((t + 2) >> 4)], p3 = s_p[t + 3 + ((t + 3) >> 4)];
          s1 += p0.x;
          s2 += p0.y;
          s1 += p1.x;
          s2 += p1.y;
          s1 += p2.x;
          s2 += p2.y;
          s1 += p3.x;
          s2 += p3.y;
        } else {
          const double p0 = s_p[t + (t >> 4)], p1 = s_p[t + 1 + ((t + 1) >> 4)];
          const double p2 = s_p[t + 2 + ((t + 2) >> 4)], p3 = s_p[t + 3 + ((t + 3) >> 4)];
          s1 += p0;
          s1 += p1;
          s1 += p2;
          s1 += p3;
        }
      }
      for (; t < cur.re; ++t) {
        if constexpr (DUAL) {
          const double2 pp = s_p[t + (t >> 4)];
          s1 += pp.x;
          s2 += pp.y;
        } else {
          s1 += s_p[t + (t >> 4)];
        }
      }
      if (DUAL) {
        const double t = s1 - cur.a1;
        pt1 += t * t;
        if (MODE == 6) {
          const double t2 = s2 - cur.a2;
          pt2 += t2 * t2;
        } else {
          st_out(y2 + r, s2, wt);
          pt2 += cur.a2 * s2;
        }
      }
      if (MODE == kEpiPlain) st_out(y1 + r, s1, wt);
      if (MODE == kEpiDot) { st_out(y1 + r, s1, wt); pt1 += cur.a1 * s1; }
      if (MODE == kEpiResNorm) { const double t = s1 - cur.a1; pt1 += t * t; }
      if (MODE == kEpiR0) { const double t = cur.a1 - s1; y1[r] = t; pt1 += t * t; }
    }
    __syncthreads();
  };
  PipeStage<CAP> sa, sb;
  if (b0 < b1) pipe_load<CAP, MODE, C16>(sa, meta, b0, ms, rp, ci, c16, base, va, aux1, aux2);
  for (int blk = b0; blk < b1; blk += 2 * bs) {
    step(sa, sb, blk);
    if (blk + bs >= b1) break;
    step(sb, sa, blk + bs);
  }
  if (MODE != kEpiPlain) {
    const double tot1 = block_sum(pt1, s_wave);
    double tot2 = 0.0;
    if (DUAL) tot2 = block_sum(pt2, s_wave);
    if (threadIdx.x == 0) {
      part1[blockIdx.x] = tot1;
      if (DUAL) part2[blockIdx.x] = tot2;
    }
  }
}

hipError_t launch_spmv_pipe(const CsrView& A, int mode, const double* x1, const double* aux1, double* y1,
                            double* part1, const double* x2, const double* aux2, double* y2, double* part2,
                            int grid, hipStream_t s, const LaunchEv* ev, const unsigned* zf, unsigned gen) {
  dim3 g(grid), b(kBlock);
  if (mode == kEpiR0 && zf != nullptr) {  // r0 with the x0 = 0 test
    if (A.col16 != nullptr)
      launch_k(spmv_pipe_kernel<kPipeCap, kEpiR0, true>, g, b, 0, s, ev, A.indptr, A.indices, A.vals, A.blk_meta,
               A.n_blk, A.walk, x1, aux1, y1, part1, x2, aux2, y2, part2, A.col16, A.blk_base, zf, gen, wt_spmv());
    else
      launch_k(spmv_pipe_kernel<kPipeCap, kEpiR0>, g, b, 0, s, ev, A.indptr, A.indices, A.vals, A.blk_meta, A.n_blk,
               A.walk, x1, aux1, y1, part1, x2, aux2, y2, part2, nullptr, nullptr, zf, gen, wt_spmv());
    return hipGetLastError();
  }
#define SPIS_PIPE(M)                                                                                            \
  if (A.col16 != nullptr)                                                                                       \
    launch_k(spmv_pipe_kernel<kPipeCap, M, true>, g, b, 0, s, ev, A.indptr, A.indices, A.vals, A.blk_meta,      \
             A.n_blk, A.walk, x1, aux1, y1, part1, x2, aux2, y2, part2, A.col16, A.blk_base,                  \
             static_cast<const unsigned*>(nullptr), 0u, wt_spmv());                                           \
  else                                                                                                          \
    launch_k(spmv_pipe_kernel<kPipeCap, M>, g, b, 0, s, ev, A.indptr, A.indices, A.vals, A.blk_meta, A.n_blk,  \
             A.walk, x1, aux1, y1, part1, x2, aux2, y2, part2, nullptr, nullptr,                                \
             static_cast<const unsigned*>(nullptr), 0u, wt_spmv())
  switch (mode) {
    case 0: SPIS_PIPE(0); break;
    case 1: SPIS_PIPE(1); break;
    case 2: SPIS_PIPE(2); break;
    case 3: SPIS_PIPE(3); break;
    case 4: SPIS_PIPE(4); break;
    default: SPIS_PIPE(6); break;
  }
#undef SPIS_PIPE
  return hipGetLastError();
}

hipError_t launch_spmv_dual(const CsrView& A, const double* x1, const double* b, double* part1,
                            const double* x2, double* w, const double* q0, double* part2, int grid,
                            hipStream_t s, const LaunchEv* ev) {
  if (A.blk_meta != nullptr)
    return launch_spmv_pipe(A, 4, x1, b, nullptr, part1, x2, q0, w, part2, grid, s, ev);
  if (A.swz)
    launch_k(spmv_dual_kernel<kDualCap, 1>, dim3(grid), dim3(kBlock), 0, s, ev, A.indptr, A.indices, A.vals,
             A.blk_row, A.n_blk, x1, b, part1, x2, w, q0, part2);
  else
    launch_k(spmv_dual_kernel<kDualCap, 0>, dim3(grid), dim3(kBlock), 0, s, ev, A.indptr, A.indices, A.vals,
             A.blk_row, A.n_blk, x1, b, part1, x2, w, q0, part2);
  return hipGetLastError();
}

// resident workgroups of the pipelined kernels (all of them fit at once: each walks its blocks)
template <typename F>
static int resident_grid(F kernel) {
  int dev = 0, cus = 256, per = 1;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, kBlock, 0) != hipSuccess || per < 1) per = 1;
  const int t = (cus * per) & ~7;
  return t < 8 ? 8 : (t > kSpmvGrid ? kSpmvGrid : t);
}

static int pipe_grid_max(bool c16) {
  static const int g1 = resident_grid(spmv_pipe_kernel<kPipeCap, 4>);
  static const int g1c = resident_grid(spmv_pipe_kernel<kPipeCap, 4, true>);
  return c16 ? g1c : g1;
}

int spmv_grid(const CsrView& A, bool fixed) {
  // fixed (multi-GPU: partial arrays all-reduced element-wise) = the same count on every rank
  if (fixed) return A.blk_meta != nullptr ? kPipeGridFixed : kSpmvGrid;
  const int cap = A.blk_meta != nullptr ? pipe_grid_max(A.col16 != nullptr) : kSpmvGrid;
  int g = A.n_blk < cap ? A.n_blk : cap;
  if (A.blk_meta != nullptr && g > 8) g &= ~7;  // the XCD-local walk deals workgroups 8 at a time
  return g < 1 ? 1 : g;
}

int blas_grid(int64_t n, bool fixed) {
  if (fixed) return kRedGrid;
  int64_t g = (n / 2 + kBlock * kMgsPer - 1) / (kBlock * kMgsPer);  // kMgsPer 16-B pairs per lane
  if (g > kRedGrid) g = kRedGrid;
  return g < 1 ? 1 : static_cast<int>(g);
}

hipError_t launch_spmv(const CsrView& A, int epi, const double* x, double* y, const double* aux,
                       double* partials, int grid, hipStream_t s, const LaunchEv* ev, const unsigned* zf,
                       unsigned gen) {
  if (A.blk_meta != nullptr)
    return launch_spmv_pipe(A, epi, x, aux, y, partials, nullptr, nullptr, nullptr, nullptr, grid, s, ev, zf, gen);
  dim3 g(grid), b(kBlock);
  switch (epi) {
    case kEpiPlain:
      launch_k(spmv_rowblock_kernel<kEpiPlain>, g, b, 0, s, ev, A.indptr, A.indices, A.vals, A.blk_row, A.n_blk,
               x, y, aux, partials, A.swz);
      break;
    case kEpiDot:
      launch_k(spmv_rowblock_kernel<kEpiDot>, g, b, 0, s, ev, A.indptr, A.indices, A.vals, A.blk_row, A.n_blk,
               x, y, aux, partials, A.swz);
      break;
    case kEpiResNorm:
      launch_k(spmv_rowblock_kernel<kEpiResNorm>, g, b, 0, s, ev, A.indptr, A.indices, A.vals, A.blk_row,
               A.n_blk, x, y, aux, partials, A.swz);
      break;
    default:
      launch_k(spmv_rowblock_kernel<kEpiR0>, g, b, 0, s, ev, A.indptr, A.indices, A.vals, A.blk_row, A.n_blk,
               x, y, aux, partials, A.swz);
      break;
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K2: one modified Gram-Schmidt step (solvers.py:194-195), fused with the NEXT dot.
//   h_i = sum(part_in)            (every workgroup, same order -> same h_i)
//   y   = y - h_i q_i             (numpy: product rounded, then subtracted — no FMA)
//   part_out = q_{i+1} . y        (or y . y when this is the last step: the norm of :196)
// 16-B accesses (double2) when all streams are 16-B aligned; the odd tail element belongs to
// workgroup 0 / lane 0 so the partial layout is fixed.
// ---------------------------------------------------------------------------------------------
template <bool VEC>
__global__ __launch_bounds__(kBlock) void mgs_step_kernel(int64_t n, double* __restrict__ y,
                                                          const double* __restrict__ qi,
                                                          const double* __restrict__ qn,
                                                          const double* __restrict__ part_in,
                                                          int n_in, double* __restrict__ part_out,
                                                          double* __restrict__ h_out,
                                                          const double* __restrict__ xpart, int n_x,
                                                          double* __restrict__ x_out,
                                                          unsigned long long* __restrict__ flag,
                                                          const unsigned long long* __restrict__ seq) {
#pragma clang fp contract(off)
  __shared__ double s_wave[4];
  double part = 0.0;
  if (VEC) {
    const int64_t npair = n >> 1;
    double2* y2 = reinterpret_cast<double2*>(y);
    const double2* q2 = reinterpret_cast<const double2*>(qi);
    const double2* n2 = reinterpret_cast<const double2*>(qn);
    const int64_t round = static_cast<int64_t>(gridDim.x) * kBlock * kMgsPer;
    int64_t base = static_cast<int64_t>(blockIdx.x) * kBlock * kMgsPer + threadIdx.x;
    double2 yv[kMgsPer], qv[kMgsPer], nv[kMgsPer];
    auto load = [&](int64_t b0) {
#pragma unroll
      for (int u = 0; u < kMgsPer; ++u) {
        const int64_t p = b0 + u * kBlock;
        if (p < npair) {
          qv[u] = q2[p];
          yv[u] = y2[p];
          if (qn) nv[u] = n2[p];
        }
      }
    };
    // the first round's loads are in flight while h_i is formed (barrier + partial reads)
    load(base);
    const double h = sum_partials(part_in, n_in, s_wave);
    if (blockIdx.x == 0 && threadIdx.x == 0) *h_out = h;
    for (;;) {
#pragma unroll
      for (int u = 0; u < kMgsPer; ++u) {
        const int64_t p = base + u * kBlock;
        if (p < npair) {
          const double a0 = h * qv[u].x, a1 = h * qv[u].y;
          yv[u].x = yv[u].x - a0;
          yv[u].y = yv[u].y - a1;
          y2[p] = yv[u];
          if (qn) {
            part += nv[u].x * yv[u].x;
            part += nv[u].y * yv[u].y;
          } else {
            part += yv[u].x * yv[u].x;
            part += yv[u].y * yv[u].y;
          }
        }
      }
      base += round;
      if (base - threadIdx.x >= npair) break;
      load(base);
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
      const int64_t e = n - 1;
      const double a = h * qi[e];
      const double yv1 = y[e] - a;
      y[e] = yv1;
      part += qn ? qn[e] * yv1 : yv1 * yv1;
    }
  } else {
    const double h = sum_partials(part_in, n_in, s_wave);
    if (blockIdx.x == 0 && threadIdx.x == 0) *h_out = h;
    const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
    for (int64_t e = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; e < n; e += stride) {
      const double a = h * qi[e];
      const double yv1 = y[e] - a;
      y[e] = yv1;
      part += qn ? qn[e] * yv1 : yv1 * yv1;
    }
  }
  const double tot = block_sum(part, s_wave);
  if (threadIdx.x == 0) part_out[blockIdx.x] = tot;
  if (xpart != nullptr && blockIdx.x == 0) {  // piggybacked reduction (e.g. a residual's partials)
    const double t = sum_partials(xpart, n_x, s_wave);
    if (threadIdx.x == 0) publish(x_out, t, flag, seq);
  }
}

static inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

hipError_t launch_mgs_step(int64_t n, double* y, const double* qi, const double* qnext,
                           const double* part_in, int n_in, double* part_out, double* h_out,
                           int grid, hipStream_t s, const LaunchEv* ev, const double* xpart, int n_x,
                           double* x_out, unsigned long long* flag, const unsigned long long* seq) {
  const bool vec = aligned16(y) && aligned16(qi) && (qnext == nullptr || aligned16(qnext));
  if (vec)
    launch_k(mgs_step_kernel<true>, dim3(grid), dim3(kBlock), 0, s, ev, n, y, qi, qnext, part_in, n_in, part_out,
             h_out, xpart, n_x, x_out, flag, seq);
  else
    launch_k(mgs_step_kernel<false>, dim3(grid), dim3(kBlock), 0, s, ev, n, y, qi, qnext, part_in, n_in, part_out,
             h_out, xpart, n_x, x_out, flag, seq);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K2p: persistent MGS chain (kernels.h).  Workgroup g owns pairs [g*256*PER, (g+1)*256*PER); data
// thread t (waves 0-3) holds pairs t + 256 k in registers; wave 4 runs the exchange.  Per step i
// (h_i known everywhere):
//   y -= h_i q_i ; part = q_{i+1}.y (or y.y at the last step) — MGS's arithmetic, contraction off
//   DPP wave sums + fixed combine -> the workgroup's partial -> two granules {tag, lo32} {tag,
//   hi32} in slot parity i&1 (sc1 stores, from a data wave)
//   workgroup 0's exchange wave sweeps all partials' granules until every tag matches, sums them
//   in a fixed order and publishes h_{i+1} as two granules; the other workgroups' exchange waves
//   poll those two (256 workgroups sweeping 512 granules each cost 15% of the chain in polling
//   traffic); q_{i+2} loads of the data waves are in flight meanwhile
// Tags are base + i + 1 with base read from a device counter the previous chain advanced, so no
// per-call reset is needed and a replayed graph stays valid.  A slot parity is rewritten two steps
// later, after every workgroup has read it (it cannot publish step i+2 before step i+1's exchange
// completed).  Spins are bounded (0.5 s of s_memrealtime): a missing workgroup sets *err, the
// launch drains, and the host reports the failure.
// ---------------------------------------------------------------------------------------------
typedef __attribute__((address_space(1))) unsigned long long chain_gu64;
constexpr unsigned long long kChainWaitTicks = 50000000ull;  // 0.5 s at 100 MHz
// SPIS_CHAIN_TRACE (tools/chainbench only, never in libspis): K2q phase timestamps (100 MHz
// s_memrealtime) of data workgroup 0, the last data workgroup and the gatherer
#ifdef SPIS_CHAIN_TRACE
__device__ unsigned long long g_chain_trace[3][48];
#define CHAIN_TR(row, idx) (g_chain_trace[row][idx] = __builtin_amdgcn_s_memrealtime())
#else
#define CHAIN_TR(row, idx) ((void)0)
#endif

__device__ __forceinline__ void chain_store(unsigned long long* p, unsigned tag, unsigned half) {
  __hip_atomic_store((chain_gu64*)p, (static_cast<unsigned long long>(tag) << 32) | half, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long chain_load(const unsigned long long* p) {
  return __hip_atomic_load((chain_gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// wave sum on DPP moves only (ALU latency; __shfl_xor is ds_bpermute, LDS latency): xor 1, xor 2,
// half-row and row mirrors make each 16-lane row uniform, row_bcast15/31 fold the rows into lane
// 63, s_readlane broadcasts it.  A fixed order: every workgroup gets the same bits for the same
// inputs (the chain relies on that for h).
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROW_MASK, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROW_MASK, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wave_sum_dpp(double v) {
  v += dpp_f64<0xB1>(v);        // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);        // quad_perm [2,3,0,1]
  v += dpp_f64<0x141>(v);       // row_half_mirror
  v += dpp_f64<0x140>(v);       // row_mirror: every lane of a row holds the row's sum
  v += dpp_f64<0x142, 0xA>(v);  // row_bcast15 into rows 1, 3 (rows 0, 2 add 0)
  v += dpp_f64<0x143, 0xC>(v);  // row_bcast31 into rows 2, 3: lane 63 holds the total
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), 63);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), 63);
  return __hiloint2double(hi, lo);
}

constexpr int kChainThreads = kBlock + 64;  // 4 data waves + 1 exchange wave

// sum_partials' exact arithmetic (same per-thread loop, same shuffle wave sums, same combine) on
// the 4 data waves, with the exchange wave joining the barriers: the first h and the piggybacked
// residual get the same bits as from the per-step kernels and finalize_kernel
// s_waitcnt vmcnt(0) alone (gfx9 encoding: vmcnt [3:0] + [15:14] = 0, expcnt and lgkmcnt at
// their max): every load of the wave, LDS DMA (global_load_lds) included, has completed
__device__ __forceinline__ void vm_drain() { __builtin_amdgcn_s_waitcnt((0x7 << 4) | (0xF << 8)); }

__device__ __forceinline__ double chain_sum_partials(const double* __restrict__ part, int n, double* s_wave) {
  const int tid = threadIdx.x;
  double v = 0.0;
  if (tid < kBlock)
    for (int i = tid; i < n; i += kBlock) v += part[i];
  v = wave_sum(v);
  if (tid < kBlock && (tid & 63) == 0) s_wave[tid >> 6] = v;
  __syncthreads();
  const double t = ((s_wave[0] + s_wave[1]) + s_wave[2]) + s_wave[3];
  __syncthreads();
  return t;
}

template <int PER>
__global__ __launch_bounds__(kChainThreads, 1) void mgs_chain_kernel(
    int64_t n, const double* __restrict__ w, double* __restrict__ Q, int64_t pitch, int j,
    const double* __restrict__ part_in, int n_in, double* __restrict__ hcol, unsigned long long* gran,
    unsigned* epoch, unsigned* err, const double* __restrict__ xpart, int n_x, double* __restrict__ x_out,
    unsigned long long* __restrict__ flag, const unsigned long long* __restrict__ seq, int agg_wg, bool nt) {
#pragma clang fp contract(off)
  __shared__ double s_wave[4];
  __shared__ double s_h;
  __shared__ int s_fail;
  // agg_wg >= 0: that workgroup (the last) holds no slice and only gathers the partials of the
  // others (its polls never queue behind q loads of its own CU); else workgroup 0 gathers
  const int G = gridDim.x;
  const int tid = threadIdx.x;
  const bool agg = static_cast<int>(blockIdx.x) == agg_wg;
  const int gat = agg_wg >= 0 ? agg_wg : 0;          // the gathering workgroup
  const int GD = agg_wg >= 0 ? G - 1 : G;            // workgroups publishing partials
  const bool data = tid < kBlock && !agg;  // waves 0-3 hold the slices; wave 4 runs the exchange
  const int64_t npair = n >> 1;
  const int64_t p0 = static_cast<int64_t>(blockIdx.x) * kBlock * PER + tid;
  // U = q_i (update), D = q_{i+1} (dot), P = q_{i+2} (in flight behind the exchange; a second
  // vector of lead time measured no faster)
  double2 y[PER], U[PER], D[PER], P[PER];
  auto load = [&](double2 (&r)[PER], const double* v) {
    const double2* v2 = reinterpret_cast<const double2*>(v);
#pragma unroll
    for (int k = 0; k < PER; ++k)
      if (data && p0 + k * kBlock < npair) r[k] = ld_basis(v2 + p0 + k * kBlock, nt);
  };
  const unsigned base = *epoch;
  load(y, w);
  load(U, Q);
  if (j >= 1) load(D, Q + pitch);
  const bool tail = (n & 1) && blockIdx.x == 0 && tid == 0;  // odd element: workgroup 0, lane 0
  double yt = 0.0, ut = 0.0, dt = 0.0, pt = 0.0;
  if (tail) {
    yt = w[n - 1];
    ut = Q[n - 1];
    if (j >= 1) dt = Q[pitch + n - 1];
  }
  if (tid == 0) s_fail = 0;
  double h = chain_sum_partials(part_in, n_in, s_wave);
  if (blockIdx.x == 0 && tid == 0) pin_store(hcol, h);
  if (xpart != nullptr && blockIdx.x == 0) {  // piggybacked reduction (the previous update's residual)
    const double t = chain_sum_partials(xpart, n_x, s_wave);
    if (tid == 0) publish(x_out, t, flag, seq);
  }
  for (int i = 0; i <= j; ++i) {
    const bool last = i == j;
    double part = 0.0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      if (data && p0 + k * kBlock < npair) {
        const double a0 = h * U[k].x, a1 = h * U[k].y;
        y[k].x = y[k].x - a0;
        y[k].y = y[k].y - a1;
        if (!last) {
          part += D[k].x * y[k].x;
          part += D[k].y * y[k].y;
        } else {
          part += y[k].x * y[k].x;
          part += y[k].y * y[k].y;
        }
      }
    }
    if (tail) {
      const double a = h * ut;
      yt = yt - a;
      part += last ? yt * yt : dt * yt;
    }
    if (i + 2 <= j) {  // q_{i+2}: in flight behind the exchange (the exchange wave holds no loads)
      load(P, Q + static_cast<int64_t>(i + 2) * pitch);
      if (tail) pt = Q[static_cast<int64_t>(i + 2) * pitch + n - 1];
    }
    {  // workgroup partial: DPP wave sums of the data waves, fixed combine
      const double wv = wave_sum_dpp(part);
      if (data && (tid & 63) == 0) s_wave[tid >> 6] = wv;
    }
    __syncthreads();
    const unsigned tag = base + static_cast<unsigned>(i) + 1u;
    unsigned long long* slots = gran + static_cast<size_t>(i & 1) * 2 * kChainMaxWG;
    if (tid == 0 && !agg) {  // publish from a data wave: the exchange wave's polls never wait on these stores
      const double tot = ((s_wave[0] + s_wave[1]) + s_wave[2]) + s_wave[3];
      const unsigned long long bits = static_cast<unsigned long long>(__double_as_longlong(tot));
      chain_store(slots + 2 * blockIdx.x, tag, static_cast<unsigned>(bits));
      chain_store(slots + 2 * blockIdx.x + 1, tag, static_cast<unsigned>(bits >> 32));
    }
    if (tid >= kBlock) {  // exchange wave
      const int lane = tid - kBlock;
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      bool all_ok = false;
      double acc = 0.0;
      if (static_cast<int>(blockIdx.x) == gat) {  // gathers every data workgroup's partial (granule 2g = lo, 2g+1 = hi)
        unsigned long long g[8];
        for (unsigned spins = 0;; ++spins) {
          bool ok = true;
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int idx = lane + 64 * k;
            g[k] = idx < 2 * GD ? chain_load(slots + idx) : (static_cast<unsigned long long>(tag) << 32);
            ok &= static_cast<unsigned>(g[k] >> 32) == tag;
          }
          if (__all(ok)) {
            all_ok = true;
            break;
          }
          if ((spins & 63) == 63 && __builtin_amdgcn_s_memrealtime() - t0 > kChainWaitTicks) break;
        }
        // fixed order: lane pairs (2m, 2m+1) of round k hold partial (64 k + 2 m) / 2; k-major
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const unsigned lo = static_cast<unsigned>(g[k]);
          const unsigned hi =
              static_cast<unsigned>(__shfl_xor(static_cast<int>(static_cast<unsigned>(g[k])), 1, 64));
          const double v =
              __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo));
          if ((lane & 1) == 0 && lane + 64 * k < 2 * GD) acc += v;
        }
        acc = wave_sum_dpp(acc);
        if (lane == 0) {  // and hands the sum to every other workgroup
          const unsigned long long bits = static_cast<unsigned long long>(__double_as_longlong(acc));
          unsigned long long* hs = gran + 4 * kChainMaxWG + 2 * (i & 1);
          chain_store(hs, tag, static_cast<unsigned>(bits));
          chain_store(hs + 1, tag, static_cast<unsigned>(bits >> 32));
        }
      } else {  // the others poll the gatherer's two granules (few pollers: the q stream keeps its bandwidth)
        const unsigned long long* hs = gran + 4 * kChainMaxWG + 2 * (i & 1);
        unsigned long long g = 0;
        for (unsigned spins = 0;; ++spins) {
          g = lane < 2 ? chain_load(hs + lane) : (static_cast<unsigned long long>(tag) << 32);
          if (__all(static_cast<unsigned>(g >> 32) == tag)) {
            all_ok = true;
            break;
          }
          if ((spins & 63) == 63 && __builtin_amdgcn_s_memrealtime() - t0 > kChainWaitTicks) break;
        }
        const unsigned lo = static_cast<unsigned>(__shfl(static_cast<int>(static_cast<unsigned>(g)), 0, 64));
        const unsigned hi = static_cast<unsigned>(__shfl(static_cast<int>(static_cast<unsigned>(g)), 1, 64));
        acc = __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo));
      }
      if (lane == 0) {
        s_h = acc;
        if (!all_ok) {
          s_fail = 1;
          atomicOr(err, 1u);
        }
      }
    }
    __syncthreads();
    const double hn = s_h;
    if (s_fail) break;  // uniform: a workgroup never arrived; the host reports it
    if (!last) {
      h = hn;
      if (blockIdx.x == 0 && tid == 0) pin_store(hcol + i + 1, hn);
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        U[k] = D[k];
        D[k] = P[k];
      }
      ut = dt;
      dt = pt;
    } else {  // K3: h_{j+1,j} = ||y||, q_{j+1} = y / h (zeros on breakdown, as normalize_kernel)
      const double hh = sqrt(hn);
      if (blockIdx.x == 0 && tid == 0) pin_store(hcol + j + 1, hh);
      double2* q2 = reinterpret_cast<double2*>(Q + static_cast<int64_t>(j + 1) * pitch);
#pragma unroll
      for (int k = 0; k < PER; ++k)
        if (data && p0 + k * kBlock < npair)
          q2[p0 + k * kBlock] = hh == 0.0 ? make_double2(0.0, 0.0) : make_double2(y[k].x / hh, y[k].y / hh);
      if (tail) Q[static_cast<int64_t>(j + 1) * pitch + n - 1] = hh == 0.0 ? 0.0 : yt / hh;
    }
  }
  if (blockIdx.x == 0 && tid == 0) *epoch = base + static_cast<unsigned>(j) + 2u;
}

// ---------------------------------------------------------------------------------------------
// K2q: pipelined MGS chain (SPIS_OPT_MGS_CHAIN = 3, the default).  MGS's projections and updates,
// with each dot product evaluated LAG steps early by the distributive law:
//     h_m = q_m . w^{(m)} = q_m . w^{(m-LAG)} - sum_{l = m-LAG}^{m-1} h_l (q_m . q_l),
// w^{(i+1)} = w^{(i)} - h_i q_i (the update itself is MGS's, in registers, contraction off; for
// m < LAG the dot is taken against w^{(0)} and every earlier h_l is subtracted).  The partial of
// q_m . w^{(m-LAG)} needs h_{m-LAG-1} only, so LAG + 1 exchanges are in flight and an Arnoldi
// step waits for about 1 / (LAG + 1) of a round trip per MGS step instead of a whole one.  The
// Gram entries G(m, l) = q_m . q_l, l = m-LAG .. m-1, do not change once q_m exists: chain j
// computes the new ones, G(j, j-LAG .. j-1) (partials published beside those of h_j), and keeps
// them in gsub for the later chains of the same basis.  The dedicated gathering workgroup (the
// last) sums each step's partials in a fixed order, forms h_m (the correction terms in l order;
// every workgroup gets the same bits), publishes it and writes H[:, j] to the host.
// Exact arithmetic: the identity above, no orthogonality assumed.  Rounding: the error of h_m is
// eps |w^{(m-LAG)}| instead of MGS's eps |w^{(m)}|.
// Basis slices rotate through NS register slots without moves (vector q_m in slot m % NS; the
// step body is instantiated per ring position): q_{i+NS-1} is loaded into q_{i-1}'s slot right
// after the update that consumed it, NS - LAG - 1 steps before it is dotted.
// Vectors are handled as ceil(n / 2) pairs: an odd n's last pair reaches into the basis' zero
// padding (pitch > n; the padding of Q, w and x0 is zeroed at allocation and never written
// nonzero), so no thread has a scalar tail.
// Slots: E_m (the exchange producing h_m, m = 1..j; E_{j+1} = ||w||^2) uses tag base + m, partial
// ring m % 4, h ring m % 4; G(j, .)'s partials have their own granules.  Ring safety (LAG <= 2):
// a workgroup publishes E_m once it has read h_{m-LAG-1}, which the gatherer published after
// reading E_{m-4}'s partials; the gatherer publishes h_m after reading E_m, which every workgroup
// publishes after it read h_{m-LAG-1} >= h_{m-3}, the last reader of h slot m % 4 before.
// FX: the update GEMV x = Q[:, :px] yx + x0 of the previous LS step rides along (K4's
// arithmetic: the sum in basis order, then + x0), accumulated in LDS as each q_i passes (each
// thread its own entries: no barrier; in registers it spilled); x = acc + x0 is stored after the
// chain's last exchange.
// ---------------------------------------------------------------------------------------------
// DW data waves hold the slices (DW * 64 threads x PER pairs each); wave DW runs the exchange.
template <int DW, int PER, int NS, int LAG, bool FX, bool NT>
__global__ __launch_bounds__(DW * 64 + 64, 1) void mgs_chain_lag_kernel(
    int64_t n, const double* __restrict__ w, double* __restrict__ Q, int64_t pitch, int j,
    const double* __restrict__ part_in, int n_in, double* __restrict__ hcol, unsigned long long* gran,
    unsigned* epoch, unsigned* err, const double* __restrict__ xpart, int n_x, double* __restrict__ x_out,
    unsigned long long* __restrict__ flag, const unsigned long long* __restrict__ seq, double* __restrict__ gsub,
    YArg yx, int px, const double* __restrict__ x0, double* __restrict__ xo, int tw, int wt) {
#pragma clang fp contract(off)
  static_assert(LAG >= 1 && LAG <= 2 && NS >= LAG + 3, "ring: q_{i-1}, the dotted q_{i+LAG}, one loading");
  // NT: nontemporal basis loads, except q_0 .. q_{tw-1} and x0 when tw > 0 (a window every chain
  // re-reads, left to stay Infinity-Cache resident beside the matrix)
  constexpr int DT = DW * 64;  // data threads
  constexpr int NV = 1 + LAG;  // values a workgroup may publish per exchange (a_m, G(m, m-LAG..m-1))
  __shared__ double2 s_acc[FX ? PER * DT : 1];
  __shared__ double2 s_x0[FX ? PER * DT : 1];
  __shared__ double s_wave[2 * NV * DW];  // publish_m's wave sums by m's parity: step 0 publishes E_1
                                         // and E_2 back to back (E_2's sums are written while E_1's
                                         // may still be read); chain_sum_partials uses the first 4
  __shared__ double s_h;
  __shared__ int s_fail;
  const int G = gridDim.x;
  const int GD = G - 1;  // data workgroups; the last one gathers
  const int tid = threadIdx.x;
  const bool agg = static_cast<int>(blockIdx.x) == GD;
  const bool data = tid < DT && !agg;
  const int64_t npair = (n + 1) >> 1;  // the last pair of an odd n reaches into the zero padding
  const int64_t p0 = static_cast<int64_t>(blockIdx.x) * DT * PER + tid;
  unsigned long long* aslots = gran;                       // 4 x 2 kChainMaxWG
  unsigned long long* gslots = gran + 8 * kChainMaxWG;     // LAG x 2 kChainMaxWG (G(j, .))
  unsigned long long* hslots = gran + 12 * kChainMaxWG;    // 4 x 2
  double* gs1 = gsub;          // G(m, m-1)
  double* gs2 = gsub + kMaxK;  // G(m, m-2)
  const unsigned base = *epoch;
  double2 y[PER];
  double2 S[NS][PER];
  auto load = [&](double2 (&r)[PER], const double* v, bool nt) {
    const double2* v2 = reinterpret_cast<const double2*>(v);
#pragma unroll
    for (int k = 0; k < PER; ++k)
      if (data && p0 + k * DT < npair) r[k] = ld_basis(v2 + p0 + k * DT, nt);
  };
  // start-up: the data workgroups issue their loads in the order of need (loads complete in issue
  // order): w and q_1, q_2 (step 0's dots), q_0 (step 1's update), the rest of the ring, then x0
  // by LDS DMA (read at the last step only).  h_0 = q_0 . w (the SpMV's
  // partials) and the piggybacked residual are summed by the gatherer, which has no basis loads to
  // queue behind; h_0 reaches the data workgroups through the exchange slots (E_0) when step 1's
  // update needs it.  The first exchange then starts after four vectors have arrived, not after
  // six vectors and two partial sums behind them.
  if (!agg) {
    if (FX && data) {
#pragma unroll
      for (int k = 0; k < PER; ++k) s_acc[k * DT + tid] = make_double2(0.0, 0.0);
    }
    load(y, w, NT);
#pragma unroll
    for (int m = 1; m < NS - 1; ++m)
      if (m <= j) load(S[m], Q + static_cast<int64_t>(m) * pitch, NT && m >= tw);
    load(S[0], Q, NT && 0 >= tw);
    if (FX && data) {  // x0 straight into LDS (global_load_lds: no registers, nothing waits on it
                       // before the last step, which drains it: vm_drain)
      const double2* x02 = reinterpret_cast<const double2*>(x0);
#pragma unroll
      for (int k = 0; k < PER; ++k)
        if (p0 + k * DT < npair)
          __builtin_amdgcn_global_load_lds(x02 + p0 + k * DT,
                                           (__attribute__((address_space(3))) void*)(s_x0 + k * DT + (tid & ~63)), 16,
                                           0, 0);
    }
  }
  if (tid == 0) s_fail = 0;
  const int tr_row = blockIdx.x == 0 ? 0 : agg ? 2 : static_cast<int>(blockIdx.x) == GD - 1 ? 1 : -1;
  if (tid == 0 && tr_row >= 0) CHAIN_TR(tr_row, 0);
  double h0 = 0.0;  // data workgroups: from E_0 (wait_h(0)) at their first update
  if (agg) {
    h0 = chain_sum_partials(part_in, n_in, s_wave);
    if (xpart != nullptr) {  // piggybacked reduction (the previous update's residual)
      const double t = chain_sum_partials(xpart, n_x, s_wave);
      if (tid == 0) publish(x_out, t, flag, seq);
    }
    if (tid == 0) {  // E_0: h_0 in h slot 0 under tag base (slot 0's next use, E_4, is published
                     // after every workgroup has read h_0 at its step 1, before its E_4 partials;
                     // the caller's tag base is never 0, the zero-initialised slots' tag)
      const unsigned long long bits = static_cast<unsigned long long>(__double_as_longlong(h0));
      chain_store(hslots, base, static_cast<unsigned>(bits));
      chain_store(hslots + 1, base, static_cast<unsigned>(bits >> 32));
    }
  }
  if (tid == 0 && tr_row >= 0) CHAIN_TR(tr_row, 1);

  if (agg) {  // ---- the gatherer: one wave sums, forms h_m and publishes it
    if (tid >= 64) return;
    const int lane = tid;
    // the whole column H[:, j] is written by this lane, each entry one system-scope store into a
    // slot the host armed (the solver's L mode, spis.cpp, waits for every slot of the column)
    if (lane == 0) pin_store(hcol, h0);
    double hl[LAG];  // h_{m-LAG} .. h_{m-1} (hl[LAG-1] = h_{m-1})
#pragma unroll
    for (int l = 0; l < LAG; ++l) hl[l] = 0.0;
    hl[LAG - 1] = h0;
    for (int m = 1; m <= j + 1; ++m) {
      const unsigned tag = base + static_cast<unsigned>(m);
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      auto sweep = [&](const unsigned long long* slots, double* out) -> bool {
        unsigned long long g[8];
        bool all_ok = false;
        for (unsigned spins = 0;; ++spins) {
          bool ok = true;
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int idx = lane + 64 * k;
            g[k] = idx < 2 * GD ? chain_load(slots + idx) : (static_cast<unsigned long long>(tag) << 32);
            ok &= static_cast<unsigned>(g[k] >> 32) == tag;
          }
          if (__all(ok)) {
            all_ok = true;
            break;
          }
          if ((spins & 63) == 63 && __builtin_amdgcn_s_memrealtime() - t0 > kChainWaitTicks) break;
        }
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {  // lane pairs (2m, 2m+1) of round k hold partial (64 k + 2 m) / 2
          const unsigned lo = static_cast<unsigned>(g[k]);
          const unsigned hi =
              static_cast<unsigned>(__shfl_xor(static_cast<int>(static_cast<unsigned>(g[k])), 1, 64));
          const double v =
              __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo));
          if ((lane & 1) == 0 && lane + 64 * k < 2 * GD) acc += v;
        }
        *out = wave_sum_dpp(acc);
        return all_ok;
      };
      double hm = 0.0;
      bool ok = sweep(aslots + static_cast<size_t>(m & 3) * 2 * kChainMaxWG, &hm);
      if (m <= j) {
        // h_m = a_m - sum_{l = max(0, m-LAG)}^{m-1} h_l G(m, l), l ascending
        double gv[LAG];
#pragma unroll
        for (int d = 0; d < LAG; ++d) {  // gv[d] = G(m, m - LAG + d)
          gv[d] = 0.0;
          const int l = m - LAG + d;
          if (l < 0) continue;
          if (m == j) {
            ok = ok && sweep(gslots + static_cast<size_t>(LAG - 1 - d) * 2 * kChainMaxWG, &gv[d]);
            if (lane == 0) (LAG - d == 1 ? gs1 : gs2)[j] = gv[d];
          } else {
            gv[d] = (LAG - d == 1 ? gs1 : gs2)[m];
          }
        }
#pragma unroll
        for (int d = 0; d < LAG; ++d) {
          if (m - LAG + d < 0) continue;
          const double t = hl[d] * gv[d];
          hm = hm - t;
        }
      }  // else E_{j+1}: ||w^{(j+1)}||^2, square-rooted by every workgroup
      if (!ok) {
        if (lane == 0) atomicOr(err, 1u);
        hm = 0.0;  // the data workgroups time out as well and report the failure
      }
      if (lane == 0) {
        const unsigned long long bits = static_cast<unsigned long long>(__double_as_longlong(hm));
        unsigned long long* hs = hslots + 2 * (m & 3);
        chain_store(hs, tag, static_cast<unsigned>(bits));
        chain_store(hs + 1, tag, static_cast<unsigned>(bits >> 32));
        pin_store(hcol + m, m <= j ? hm : sqrt(hm));  // every slot armed: no order needed
      }
      if (lane == 0) CHAIN_TR(2, 2 + m);
      if (!ok) return;
#pragma unroll
      for (int l = 0; l + 1 < LAG; ++l) hl[l] = hl[l + 1];
      hl[LAG - 1] = hm;
    }
    if (lane == 0) *epoch = base + static_cast<unsigned>(j) + 2u;
    return;
  }

  // ---- data workgroups
  // h_m from the gatherer (exchange wave polls, every wave joins the barrier); false on timeout
  auto wait_h = [&](int m, double* out) -> bool {
    const unsigned tag = base + static_cast<unsigned>(m);
    if (tid >= DT) {
      const int lane = tid - DT;
      const unsigned long long* hs = hslots + 2 * (m & 3);
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      unsigned long long g = 0;
      bool ok = false;
      for (unsigned spins = 0;; ++spins) {
        g = lane < 2 ? chain_load(hs + lane) : (static_cast<unsigned long long>(tag) << 32);
        if (__all(static_cast<unsigned>(g >> 32) == tag)) {
          ok = true;
          break;
        }
        if ((spins & 63) == 63 && __builtin_amdgcn_s_memrealtime() - t0 > kChainWaitTicks) break;
      }
      const unsigned lo = static_cast<unsigned>(__shfl(static_cast<int>(static_cast<unsigned>(g)), 0, 64));
      const unsigned hi = static_cast<unsigned>(__shfl(static_cast<int>(static_cast<unsigned>(g)), 1, 64));
      if (lane == 0) {
        s_h = __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo));
        if (!ok) {
          s_fail = 1;
          atomicOr(err, 1u);
        }
      }
    }
    __syncthreads();
    *out = s_h;
    if (tid == 0 && tr_row >= 0) CHAIN_TR(tr_row, 2 + m);
    const bool failed = s_fail != 0;
    __syncthreads();  // s_h is rewritten by the next wait
    return !failed;
  };
  // the workgroup's partials of E_m: v[0] = a_m, v[1 + d] = G(m, m - LAG + d) when ng > 0
  // (granules {tag, half}, sc1 stores from a data wave)
  auto publish_m = [&](const double (&v)[NV], bool with_g, int m) {
    double* sw = s_wave + (m & 1) * (NV * DW);
    double wv[NV];
#pragma unroll
    for (int c = 0; c < NV; ++c) wv[c] = (c == 0 || with_g) ? wave_sum_dpp(v[c]) : 0.0;
    if (data && (tid & 63) == 0) {
#pragma unroll
      for (int c = 0; c < NV; ++c) sw[c * DW + (tid >> 6)] = wv[c];
    }
    __syncthreads();
    if (tid == 0) {
      const unsigned tag = base + static_cast<unsigned>(m);
#pragma unroll
      for (int c = 0; c < NV; ++c) {
        if (c > 0 && (!with_g || m - LAG + (c - 1) < 0)) continue;
        double t = sw[c * DW];
#pragma unroll
        for (int q = 1; q < DW; ++q) t += sw[c * DW + q];
        const unsigned long long bb = static_cast<unsigned long long>(__double_as_longlong(t));
        unsigned long long* sl = c == 0 ? aslots + static_cast<size_t>(m & 3) * 2 * kChainMaxWG + 2 * blockIdx.x
                                        : gslots + static_cast<size_t>(LAG - c) * 2 * kChainMaxWG + 2 * blockIdx.x;
        chain_store(sl, tag, static_cast<unsigned>(bb));
        chain_store(sl + 1, tag, static_cast<unsigned>(bb >> 32));
      }
    }
  };
  // y -= h q (MGS's update, contraction off)
  auto update = [&](double h, const double2 (&q)[PER]) {
#pragma unroll
    for (int k = 0; k < PER; ++k)
      if (data && p0 + k * DT < npair) {
        const double a0 = h * q[k].x, a1 = h * q[k].y;
        y[k].x = y[k].x - a0;
        y[k].y = y[k].y - a1;
      }
  };
  // partials of E_m with q_m in slot RD: a_m = q_m . y (y = w^{(max(0, m-LAG))} when called),
  // with G(m, l) for m == j (the slots of q_l: RD - LAG + d, ring order)
  auto dots = [&](auto RDC, int m) {
    constexpr int RD = decltype(RDC)::value;
    const bool with_g = m == j;
    double v[NV];
#pragma unroll
    for (int c = 0; c < NV; ++c) v[c] = 0.0;
#pragma unroll
    for (int k = 0; k < PER; ++k)
      if (data && p0 + k * DT < npair) {
        v[0] += S[RD][k].x * y[k].x;
        v[0] += S[RD][k].y * y[k].y;
        if (with_g) {
#pragma unroll
          for (int d = 0; d < LAG; ++d) {
            const int rl = (RD - LAG + d + 2 * NS) % NS;  // constant once unrolled
            v[1 + d] += S[RD][k].x * S[rl][k].x;
            v[1 + d] += S[RD][k].y * S[rl][k].y;
          }
        }
      }
    publish_m(v, with_g, m);
  };
  // one MGS step at ring position R = i % NS; false once the chain is finished (or failed)
  auto step = [&](auto RC, int i) -> bool {
    constexpr int R = decltype(RC)::value;
    constexpr int RM = (R + NS - 1) % NS;  // q_{i-1}, then q_{i+NS-1}
    if (i >= 1) {
      double hu = 0.0;
      if (!wait_h(i - 1, &hu)) return false;  // (i = 1: h_0 from E_0)
      update(hu, S[RM]);
    }
    if (i == j) {  // last: subtract h_j q_j, ||w||^2 through the gatherer, normalise
      if (FX) {  // x is complete (its last term, q_{px-1}, passed at step j - 1): stored now, its
                 // write drains during the two exchanges still ahead instead of after them
        vm_drain();  // x0's LDS DMA (issued after the ring's first loads) has landed
        const __amdgpu_buffer_rsrc_t xr = span_rsrc(xo);
#pragma unroll
        for (int k = 0; k < PER; ++k)
          if (data && p0 + k * DT < npair) {
            const double2 a = s_acc[k * DT + tid];
            const double2 b = s_x0[k * DT + tid];
            const double2 xv = make_double2(a.x + b.x, a.y + b.y);
            if (wt)
              buf_st2_wt(xr, static_cast<int>((p0 + k * DT) * 16), xv);
            else
              buf_st2(xr, static_cast<int>((p0 + k * DT) * 16), 0, xv);
          }
      }
      double hj = 0.0;
      if (!wait_h(j, &hj)) return false;  // (j = 0: h_0 from E_0)
      update(hj, S[R]);
      double v[NV];
#pragma unroll
      for (int c = 0; c < NV; ++c) v[c] = 0.0;
#pragma unroll
      for (int k = 0; k < PER; ++k)
        if (data && p0 + k * DT < npair) {
          v[0] += y[k].x * y[k].x;
          v[0] += y[k].y * y[k].y;
        }
      publish_m(v, false, j + 1);
      double nn = 0.0;
      if (!wait_h(j + 1, &nn)) return false;
      const double hh = sqrt(nn);
      double2* q2 = reinterpret_cast<double2*>(Q + static_cast<int64_t>(j + 1) * pitch);
      const __amdgpu_buffer_rsrc_t qr = span_rsrc(q2);
#pragma unroll
      for (int k = 0; k < PER; ++k)
        if (data && p0 + k * DT < npair) {
          const double2 qv = hh == 0.0 ? make_double2(0.0, 0.0) : make_double2(y[k].x / hh, y[k].y / hh);
          if (wt)
            buf_st2_wt(qr, static_cast<int>((p0 + k * DT) * 16), qv);
          else
            buf_st2(qr, static_cast<int>((p0 + k * DT) * 16), 0, qv);
        }
      if (tid == 0 && tr_row >= 0) CHAIN_TR(tr_row, 40);
      return false;
    }
    // q_{i+NS-1} into the slot q_{i-1} just left
    if (i + NS - 1 <= j) load(S[RM], Q + static_cast<int64_t>(i + NS - 1) * pitch, NT && i + NS - 1 >= tw);
    // E_{i+LAG} (at i = 0 also E_1 .. E_{LAG-1}: their dots against w^{(0)} as well)
    if (i == 0) {
      if (LAG >= 2 && 1 <= j) dots(std::integral_constant<int, (R + 1) % NS>{}, 1);
    }
    if (i + LAG <= j) dots(std::integral_constant<int, (R + LAG) % NS>{}, i + LAG);
    // x += yx_i q_i (K4's order; x0 is added after the last coefficient), after this step's
    // partials are published: its LDS read-modify-write overlaps the exchange instead of
    // delaying the dots (q_i stays in slot R until the next step's update)
    if (FX && i < px) {
      const double cf = yx.v[i];
#pragma unroll
      for (int k = 0; k < PER; ++k)
        if (data) {
          double2 a = s_acc[k * DT + tid];
          const double m0 = S[R][k].x * cf, m1 = S[R][k].y * cf;
          a.x = a.x + m0;
          a.y = a.y + m1;
          s_acc[k * DT + tid] = a;
        }
    }
    return true;
  };
  for (int i = 0;; i += NS) {
    if (!step(std::integral_constant<int, 0>{}, i)) break;
    if (!step(std::integral_constant<int, 1>{}, i + 1)) break;
    if (!step(std::integral_constant<int, 2>{}, i + 2)) break;
    if (!step(std::integral_constant<int, 3>{}, i + 3)) break;
    if constexpr (NS > 4) {
      if (!step(std::integral_constant<int, 4>{}, i + 4)) break;
    }
    if constexpr (NS > 5) {
      if (!step(std::integral_constant<int, 5>{}, i + 5)) break;
    }
  }
}

// The exchange of one chain step (K2p's protocol): the gathering workgroup's wave sweeps every
// data workgroup's {tag, half} granules, sums the partials in a fixed order and publishes h as two
// granules at hs; every other workgroup's wave polls those two.  Bounded spins (0.5 s).
__device__ __forceinline__ void chain_exchange(int lane, bool gatherer, int GD, unsigned tag,
                                               unsigned long long* slots, unsigned long long* hs, unsigned* err,
                                               double* s_h, int* s_fail) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  bool all_ok = false;
  double acc = 0.0;
  if (gatherer) {
    unsigned long long g[8];
    for (unsigned spins = 0;; ++spins) {
      bool ok = true;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int idx = lane + 64 * k;
        g[k] = idx < 2 * GD ? chain_load(slots + idx) : (static_cast<unsigned long long>(tag) << 32);
        ok &= static_cast<unsigned>(g[k] >> 32) == tag;
      }
      if (__all(ok)) {
        all_ok = true;
        break;
      }
      if ((spins & 63) == 63 && __builtin_amdgcn_s_memrealtime() - t0 > kChainWaitTicks) break;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {  // lane pairs (2m, 2m+1) of round k hold partial (64 k + 2 m) / 2
      const unsigned lo = static_cast<unsigned>(g[k]);
      const unsigned hi = static_cast<unsigned>(__shfl_xor(static_cast<int>(static_cast<unsigned>(g[k])), 1, 64));
      const double v = __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo));
      if ((lane & 1) == 0 && lane + 64 * k < 2 * GD) acc += v;
    }
    acc = wave_sum_dpp(acc);
    if (lane == 0) {
      const unsigned long long bits = static_cast<unsigned long long>(__double_as_longlong(acc));
      chain_store(hs, tag, static_cast<unsigned>(bits));
      chain_store(hs + 1, tag, static_cast<unsigned>(bits >> 32));
    }
  } else {
    unsigned long long g = 0;
    for (unsigned spins = 0;; ++spins) {
      g = lane < 2 ? chain_load(hs + lane) : (static_cast<unsigned long long>(tag) << 32);
      if (__all(static_cast<unsigned>(g >> 32) == tag)) {
        all_ok = true;
        break;
      }
      if ((spins & 63) == 63 && __builtin_amdgcn_s_memrealtime() - t0 > kChainWaitTicks) break;
    }
    const unsigned lo = static_cast<unsigned>(__shfl(static_cast<int>(static_cast<unsigned>(g)), 0, 64));
    const unsigned hi = static_cast<unsigned>(__shfl(static_cast<int>(static_cast<unsigned>(g)), 1, 64));
    acc = __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo));
  }
  if (lane == 0) {
    *s_h = acc;
    if (!all_ok) {
      *s_fail = 1;
      atomicOr(err, 1u);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// K2b: the persistent MGS chain for large N (K2p's limit < N <= 10.4 M; K2 launches beyond).
// Only w lives in registers (PER double2 per thread, 8 waves per workgroup, 255 data workgroups +
// the gathering one, one workgroup per CU).  Each step streams q_i (mostly still in the Infinity
// Cache from the previous step's dot) and q_{i+1} in chunks of 2 pairs, two chunks in flight:
// 16 N bytes per step instead of K2's 32 N (w is neither re-read nor written back) and no kernel
// boundary.  Wave 0 runs the exchange after the data phase (no loads in flight then).  Tags,
// exchange and arithmetic as K2p (contraction off; partials grouped per workgroup).
// ---------------------------------------------------------------------------------------------
constexpr int kBigThreads = 512;
template <int PER>
__global__ __launch_bounds__(kBigThreads, 1) void mgs_chain_big_kernel(
    int64_t n, const double* __restrict__ w, double* __restrict__ Q, int64_t pitch, int j,
    const double* __restrict__ part_in, int n_in, double* __restrict__ hcol, unsigned long long* gran,
    unsigned* epoch, unsigned* err, const double* __restrict__ xpart, int n_x, double* __restrict__ x_out,
    unsigned long long* __restrict__ flag, const unsigned long long* __restrict__ seq) {
#pragma clang fp contract(off)
  constexpr int NW = kBigThreads / 64;
  constexpr int CH = 2;  // pairs per streamed chunk
  constexpr int NC = PER / CH;
  static_assert(NC % 2 == 0, "chunks are consumed in pairs");
  __shared__ double s_wave[NW];
  __shared__ double s_h;
  __shared__ int s_fail;
  const int GD = static_cast<int>(gridDim.x) - 1;  // the last workgroup gathers
  const int tid = threadIdx.x;
  const bool data = static_cast<int>(blockIdx.x) != GD;
  const int64_t npair = n >> 1;
  const int64_t p0 = static_cast<int64_t>(blockIdx.x) * kBigThreads * PER + tid;
  const int voff = static_cast<int>(p0 * 16);      // this thread's first pair, bytes
  constexpr int kStep = kBigThreads * 16;           // bytes between a thread's consecutive pairs
  const int64_t vbytes = npair * 16;
  // pairs k < kv of this thread exist (every access is predicated on it)
  const int kv = (data && p0 < npair) ? static_cast<int>(min<int64_t>(PER, (npair - p0 + kBigThreads - 1) / kBigThreads)) : 0;
  double2 y[PER];
  {
    const __amdgpu_buffer_rsrc_t rw = vec_rsrc(w, vbytes);
#pragma unroll
    for (int k = 0; k < PER; ++k) y[k] = k < kv ? buf_ld2(rw, voff, k * kStep) : make_double2(0.0, 0.0);
  }
  const unsigned base = *epoch;
  const bool tail = (n & 1) && blockIdx.x == 0 && tid == 0;  // odd element: workgroup 0, lane 0
  double yt = tail ? w[n - 1] : 0.0;
  if (tid == 0) s_fail = 0;
  double h = chain_sum_partials(part_in, n_in, s_wave);
  if (blockIdx.x == 0 && tid == 0) pin_store(hcol, h);
  if (xpart != nullptr && blockIdx.x == 0) {  // piggybacked reduction (the previous update's residual)
    const double t = chain_sum_partials(xpart, n_x, s_wave);
    if (tid == 0) publish(x_out, t, flag, seq);
  }
  for (int i = 0; i <= j; ++i) {
    const bool last = i == j;
    double part = 0.0;
    if (data) {
      // q_i and q_{i+1} (none at the last step: a zero-length range reads zeros)
      const __amdgpu_buffer_rsrc_t ru = vec_rsrc(Q + static_cast<int64_t>(i) * pitch, vbytes);
      const __amdgpu_buffer_rsrc_t rd = vec_rsrc(Q + static_cast<int64_t>(i + 1) * pitch, vbytes);
      double2 ua[CH], da[CH], ub[CH], db[CH];
      auto fetch = [&](double2 (&uu)[CH], double2 (&dd)[CH], int c) {
#pragma unroll
        for (int q = 0; q < CH; ++q) {
          const bool ok = c * CH + q < kv;
          uu[q] = ok ? buf_ld2(ru, voff, (c * CH + q) * kStep) : make_double2(0.0, 0.0);
          dd[q] = (ok && !last) ? buf_ld2(rd, voff, (c * CH + q) * kStep) : make_double2(0.0, 0.0);
        }
      };
      auto consume = [&](const double2 (&uu)[CH], const double2 (&dd)[CH], int c) {
#pragma unroll
        for (int q = 0; q < CH; ++q) {
          const int k = c * CH + q;
          if (k < kv) {
            const double a0 = h * uu[q].x, a1 = h * uu[q].y;
            y[k].x = y[k].x - a0;
            y[k].y = y[k].y - a1;
            if (!last) {
              part += dd[q].x * y[k].x;
              part += dd[q].y * y[k].y;
            } else {
              part += y[k].x * y[k].x;
              part += y[k].y * y[k].y;
            }
          }
        }
      };
      fetch(ua, da, 0);
#pragma unroll
      for (int c = 0; c < NC; c += 2) {
        fetch(ub, db, c + 1);
        consume(ua, da, c);
        if (c + 2 < NC) fetch(ua, da, c + 2);
        consume(ub, db, c + 1);
      }
    }
    if (tail) {
      const double a = h * Q[static_cast<int64_t>(i) * pitch + n - 1];
      yt = yt - a;
      part += last ? yt * yt : Q[static_cast<int64_t>(i + 1) * pitch + n - 1] * yt;
    }
    {  // workgroup partial: DPP wave sums, fixed combine
      const double wv = wave_sum_dpp(part);
      if (data && (tid & 63) == 0) s_wave[tid >> 6] = wv;
    }
    __syncthreads();
    const unsigned tag = base + static_cast<unsigned>(i) + 1u;
    unsigned long long* slots = gran + static_cast<size_t>(i & 1) * 2 * kChainMaxWG;
    if (tid < 64) {
      if (tid == 0 && data) {
        double tot = s_wave[0];
#pragma unroll
        for (int ww = 1; ww < NW; ++ww) tot += s_wave[ww];
        const unsigned long long bits = static_cast<unsigned long long>(__double_as_longlong(tot));
        chain_store(slots + 2 * blockIdx.x, tag, static_cast<unsigned>(bits));
        chain_store(slots + 2 * blockIdx.x + 1, tag, static_cast<unsigned>(bits >> 32));
      }
      chain_exchange(tid, !data, GD, tag, slots, gran + 4 * kChainMaxWG + 2 * (i & 1), err, &s_h, &s_fail);
    }
    __syncthreads();
    const double hn = s_h;
    if (s_fail) break;  // uniform: a workgroup never arrived; the host reports it
    if (!last) {
      h = hn;
      if (blockIdx.x == 0 && tid == 0) pin_store(hcol + i + 1, hn);
    } else {  // K3: h_{j+1,j} = ||y||, q_{j+1} = y / h (zeros on breakdown)
      const double hh = sqrt(hn);
      if (blockIdx.x == 0 && tid == 0) pin_store(hcol + j + 1, hh);
      const __amdgpu_buffer_rsrc_t rq = vec_rsrc(Q + static_cast<int64_t>(j + 1) * pitch, vbytes);
#pragma unroll
      for (int k = 0; k < PER; ++k)
        if (k < kv)
          buf_st2(rq, voff, k * kStep, hh == 0.0 ? make_double2(0.0, 0.0) : make_double2(y[k].x / hh, y[k].y / hh));
      if (tail) Q[static_cast<int64_t>(j + 1) * pitch + n - 1] = hh == 0.0 ? 0.0 : yt / hh;
    }
  }
  if (blockIdx.x == 0 && tid == 0) *epoch = base + static_cast<unsigned>(j) + 2u;
}

static int g_chain_lag = kLagDepth;
void set_chain_lag(int lag) { g_chain_lag = lag == 1 ? 1 : 2; }

hipError_t launch_mgs_chain(int64_t n, const double* w, double* Q, int64_t pitch, int j, const double* part_in,
                            int n_in, double* hcol, unsigned long long* gran, unsigned* epoch, unsigned* err,
                            hipStream_t s, const LaunchEv* ev, const double* xpart, int n_x, double* x_out,
                            unsigned long long* flag, const unsigned long long* seq, bool aggregator, bool nt,
                            double* gsub, const double* yx_host, int px, const double* x0, double* xo, int tw) {
  const int64_t npair = n >> 1;
  if (!aligned16(w) || !aligned16(Q) || (pitch & 1)) return hipErrorInvalidValue;
  // K2q counts (n + 1) / 2 pairs (an odd n's last pair padded): its fallback test must too
  const int64_t npk = gsub != nullptr ? (n + 1) >> 1 : npair;
  if (aggregator && npk > (kChainMaxWG - 1) * int64_t(kBlock) * 8) {  // K2b (K2q falls back to it)
    if (px > 0) return hipErrorInvalidValue;  // the fused GEMV is K2q's only
    if (npair > kChainBigMaxPairs) return hipErrorInvalidValue;
    const int64_t wd = kChainMaxWG - 1;
    const int per = npair <= wd * kBigThreads * 8    ? 8
                    : npair <= wd * kBigThreads * 16 ? 16
                    : npair <= wd * kBigThreads * 24 ? 24
                    : npair <= wd * kBigThreads * 32 ? 32
                                                     : 40;
    const int64_t span = int64_t(kBigThreads) * per;
    const int GD = static_cast<int>((npair + span - 1) / span);
#define SPIS_BIG(PER_)                                                                                             \
  launch_k(mgs_chain_big_kernel<PER_>, dim3(GD + 1), dim3(kBigThreads), 0, s, ev, n, w, Q, pitch, j, part_in, n_in, \
           hcol, gran, epoch, err, xpart, n_x, x_out, flag, seq)
    switch (per) {
      case 8: SPIS_BIG(8); break;
      case 16: SPIS_BIG(16); break;
      case 24: SPIS_BIG(24); break;
      case 32: SPIS_BIG(32); break;
      default: SPIS_BIG(40); break;
    }
#undef SPIS_BIG
    return hipGetLastError();
  }
  if (npair > kChainMaxPairs) return hipErrorInvalidValue;
  if (gsub != nullptr) {  // K2q: always with the dedicated gatherer; 8 data waves (kLagDW)
    const int64_t wd = kChainMaxWG - 1;
    constexpr int DT = kLagDW * 64;
    const int64_t npr = (n + 1) >> 1;  // K2q pads an odd n's last pair with the zero padding
    if (pitch < 2 * npr) return hipErrorInvalidValue;
    const int per = npr <= wd * DT * 1 ? 1 : npr <= wd * DT * 2 ? 2 : 4;
    const int64_t span = int64_t(DT) * per;
    const int GD = static_cast<int>(std::max<int64_t>(1, (npr + span - 1) / span));
    if (GD > wd) return hipErrorInvalidValue;
    if (px < 0 || px > j || px > kYArg || (px > 0 && (!yx_host || !x0 || !xo || !aligned16(x0) || !aligned16(xo))))
      return hipErrorInvalidValue;
    YArg ya;
    for (int i = 0; i < px; ++i) ya.v[i] = yx_host[i];
#define SPIS_LAG(PER_, FX_, NT_, LAG_)                                                                          \
  launch_k(mgs_chain_lag_kernel<kLagDW, PER_, kLagNS, LAG_, FX_, NT_>, dim3(GD + 1), dim3(DT + 64), 0, s, ev, n, w, Q, \
           pitch, j, part_in, n_in, hcol, gran, epoch, err, xpart, n_x, x_out, flag, seq, gsub, ya, px, x0, xo, tw, \
           wt_mgs())
#define SPIS_LAG_PER(FX_, NT_, LAG_)          \
  switch (per) {                              \
    case 1: SPIS_LAG(1, FX_, NT_, LAG_); break; \
    case 2: SPIS_LAG(2, FX_, NT_, LAG_); break; \
    default: SPIS_LAG(4, FX_, NT_, LAG_); break; \
  }
#define SPIS_LAG_D(LAG_)                                     \
  if (px > 0 && nt) SPIS_LAG_PER(true, true, LAG_)           \
  else if (px > 0) SPIS_LAG_PER(true, false, LAG_)           \
  else if (nt) SPIS_LAG_PER(false, true, LAG_)               \
  else SPIS_LAG_PER(false, false, LAG_)
    if (g_chain_lag == 1) {
      SPIS_LAG_D(1)
    } else {
      SPIS_LAG_D(2)
    }
#undef SPIS_LAG_D
#undef SPIS_LAG_PER
#undef SPIS_LAG
    return hipGetLastError();
  }
  const int64_t wmax = kChainMaxWG - (aggregator ? 1 : 0);  // one workgroup per CU in all
  const int per = npair <= wmax * kBlock * 2 ? 2 : npair <= wmax * kBlock * 4 ? 4 : 8;
  const int64_t span = int64_t(kBlock) * per;
  const int GD = static_cast<int>(std::max<int64_t>(1, (npair + span - 1) / span));
  if (GD > wmax) return hipErrorInvalidValue;
  const int G = GD + (aggregator ? 1 : 0);
  const int agg_wg = aggregator ? GD : -1;
#define SPIS_CHAIN(PER_)                                                                                   \
  launch_k(mgs_chain_kernel<PER_>, dim3(G), dim3(kChainThreads), 0, s, ev, n, w, Q, pitch, j, part_in, n_in, hcol, \
           gran, epoch, err, xpart, n_x, x_out, flag, seq, agg_wg, nt)
  switch (per) {
    case 2: SPIS_CHAIN(2); break;
    case 4: SPIS_CHAIN(4); break;
    default: SPIS_CHAIN(8); break;
  }
#undef SPIS_CHAIN
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K3: h_{j+1,j} = ||y|| = sqrt(y.y) (numpy's norm), q_{j+1} = y / h (true division, :198).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void normalize_kernel(int64_t n, const double* __restrict__ y,
                                                           double* __restrict__ qn,
                                                           const double* __restrict__ part_in,
                                                           int n_in, double* __restrict__ h_out, int wt) {
  __shared__ double s_wave[4];
  const bool vec = ((reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(qn)) & 15) == 0;
  const int64_t npair = vec ? (n >> 1) : 0;
  const double2* y2 = reinterpret_cast<const double2*>(y);
  double2* q2 = reinterpret_cast<double2*>(qn);
  const int64_t round = static_cast<int64_t>(gridDim.x) * kBlock * kMgsPer;
  int64_t base = static_cast<int64_t>(blockIdx.x) * kBlock * kMgsPer + threadIdx.x;
  double2 yv[kMgsPer];
#pragma unroll
  for (int u = 0; u < kMgsPer; ++u)
    if (base + u * kBlock < npair) yv[u] = y2[base + u * kBlock];
  const double h = sqrt(sum_partials(part_in, n_in, s_wave));
  if (blockIdx.x == 0 && threadIdx.x == 0) pin_store(h_out, h);  // a host spinning on the slot sees it whole
  // breakdown (h == 0): cgmres/gmres stop (solvers.py:199-202); cgmres_p carries on with the
  // q[j+1] row it never wrote, i.e. zeros (solvers.py:172,376-377) — reproduce that here
  while (base - threadIdx.x < npair) {
#pragma unroll
    for (int u = 0; u < kMgsPer; ++u) {
      const int64_t p = base + u * kBlock;
      if (p < npair) {
        const double2 qv = h == 0.0 ? make_double2(0.0, 0.0) : make_double2(yv[u].x / h, yv[u].y / h);
        if (wt) {
          st_wt(qn + 2 * p, qv.x);
          st_wt(qn + 2 * p + 1, qv.y);
        } else {
          q2[p] = qv;
        }
      }
    }
    base += round;
#pragma unroll
    for (int u = 0; u < kMgsPer; ++u)
      if (base + u * kBlock < npair) yv[u] = y2[base + u * kBlock];
  }
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;  // scalar tail / unaligned
  for (int64_t e = 2 * npair + static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; e < n; e += stride)
    st_out(qn + e, h == 0.0 ? 0.0 : y[e] / h, wt);
}

hipError_t launch_normalize(int64_t n, const double* y, double* qnext, const double* part_in,
                            int n_in, double* h_out, hipStream_t s, int grid, const LaunchEv* ev) {
  launch_k(normalize_kernel, dim3(grid), dim3(kBlock), 0, s, ev, n, y, qnext, part_in, n_in, h_out, wt_k2w());
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K2c: CGS2 ("classical Gram-Schmidt, twice") — the opt-in low-synchronisation orthogonalisation
// (SURVEY §8e).  Per Arnoldi step with nv = j+1 <= kCgsMax basis vectors:
//   cgs_dot:       c1_i partials = q_i . w                 (one pass, all nv dots)
//   cgs_finalize:  c1 (device)
//   cgs_update<1>: w' = w - sum_i c1_i q_i ; c2_i partials = q_i . w'
//   cgs_finalize:  c2 (device); h_i = c1_i + c2_i -> host H column
//   cgs_update<0>: w'' = w' - sum_i c2_i q_i ; ||w''||^2 partials   -> normalize_kernel
// 3 reductions per step instead of MGS's j+2 (one all-reduce each on several GPUs); not MGS's
// arithmetic (the reference's, solvers.py:193-195), so it is never the default.
// ---------------------------------------------------------------------------------------------
// Basis vectors are split over the workgroup's 4 waves (vector i -> wave i % 4, 8 per wave), all
// 4 waves walk the same 256-element chunks (lane: 2 x double2, i.e. 2 KB contiguous per vector and
// chunk): 8 accumulators and 8 address streams per lane.  The scalar tail (odd n, unaligned
// chunks) is handled element-wise by wave 0's lanes in the last chunk.
constexpr int kCgsPerWave = kCgsMax / (kBlock / 64);
constexpr int kCgsChunk = 256;

__host__ __device__ __forceinline__ bool aligned16d(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

__global__ __launch_bounds__(kBlock) void cgs_dot_kernel(int64_t n, const double* __restrict__ w,
                                                         const double* __restrict__ Q, int64_t pitch, int nv,
                                                         double* __restrict__ part) {
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  double acc[kCgsPerWave];
#pragma unroll
  for (int m = 0; m < kCgsPerWave; ++m) acc[m] = 0.0;
  const double* Qw = Q + wid * pitch;
  const int64_t step = 4 * pitch;
  const bool vec = aligned16d(w) && aligned16d(Q) && (pitch % 2 == 0);
  const int64_t n_vec = vec ? (n / kCgsChunk) * kCgsChunk : 0;
  for (int64_t e0 = static_cast<int64_t>(blockIdx.x) * kCgsChunk; e0 < n_vec;
       e0 += static_cast<int64_t>(gridDim.x) * kCgsChunk) {
    const int64_t e = e0 + 2 * lane;  // elements e, e+1 and e+128, e+129
    const double2 wa = *reinterpret_cast<const double2*>(w + e);
    const double2 wb = *reinterpret_cast<const double2*>(w + e + 128);
#pragma unroll
    for (int m = 0; m < kCgsPerWave; ++m) {
      if (wid + 4 * m < nv) {
        const double* qv = Qw + m * step;
        const double2 qa = *reinterpret_cast<const double2*>(qv + e);
        const double2 qb = *reinterpret_cast<const double2*>(qv + e + 128);
        acc[m] += qa.x * wa.x;
        acc[m] += qa.y * wa.y;
        acc[m] += qb.x * wb.x;
        acc[m] += qb.y * wb.y;
      }
    }
  }
  for (int64_t e = n_vec + static_cast<int64_t>(blockIdx.x) * 64 + lane; e < n;
       e += static_cast<int64_t>(gridDim.x) * 64) {
    const double we = w[e];
#pragma unroll
    for (int m = 0; m < kCgsPerWave; ++m)
      if (wid + 4 * m < nv) acc[m] += Qw[m * step + e] * we;
  }
#pragma unroll
  for (int m = 0; m < kCgsPerWave; ++m) {
    const int i = wid + 4 * m;
    if (i < nv) {
      const double t = wave_sum(acc[m]);
      if (lane == 0) part[static_cast<int64_t>(i) * gridDim.x + blockIdx.x] = t;
    }
  }
}

// FX (several GPUs, L mode; DOT = 0): the same pass also forms U_{px-1}'s iterate
// x = Z[:, :px] y + x0 (Z = Q, px <= nv) from the basis values it already holds: each wave sums
// its vectors' y_l q_l (l = wid, wid + 4, ... with fma, in that order), the four wave sums combine
// through LDS in wave order, then + x0; rows [n, n_gx) (x's ghost rows, from the basis vectors'
// ghost entries) by the same arithmetic one row per thread, so a rank's ghost copy of x equals its
// owner's bitwise and x needs no halo exchange
// K2w's coefficients, formed by every update workgroup before its pass (COEF; the separate
// one-workgroup launch and its gap are gone): from the 2 nv - 1 reduced dots d, Gram row nv - 1
// (to G by workgroup 0: rows < nv - 1 were written by the earlier steps of this solve), then
// h_l = ((q_l . w - h_0 G(l, 0)) - h_1 G(l, 1)) - ... in l order -> s_c, and workgroup 0 writes the
// host H column.  The Gram triangle is staged in LDS (packed: row i at i (i - 1) / 2), and the
// forward substitution runs column by column on one wave: lane i holds t_i and, once h_l = t_l is
// broadcast, subtracts h_l G(i, l) — for every i the same subtractions in the same l order as the
// row-by-row recurrence, so every workgroup forms the same bits.  (Thread 0 running the recurrence
// with h[] in private memory took 17 us per step: the dynamically indexed array lived in scratch.)
struct CoefArg {
  const double* d;  // nullptr: coef holds the coefficients already
  double* G;        // kCgsMax x kCgsMax, row-major
  double* h_out;    // the host H column (nullable)
  // (nullable) a true residual's partials, reduced and published by workgroup 0 as finalize_kernel
  // does (the residual that rode the dots' all-reduce; one launch fewer per Arnoldi step)
  const double* rpart;
  int r_in;
  double* r_out;
  unsigned long long* flag;
  const unsigned long long* seq;
};
constexpr int kGramTri = kCgsMax * (kCgsMax - 1) / 2;

__device__ __forceinline__ void icwy_coefficients(const CoefArg ca, int nv, double* s_c, double* s_gt, double* s_d) {
#pragma clang fp contract(off)
  static_assert(kCgsMax <= 64, "one lane per coefficient");
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const bool writer = blockIdx.x == 0;
  if (ca.d != nullptr)  // (else the caller staged the dots in s_d: K2s)
    for (int i = threadIdx.x; i < 2 * nv - 1; i += kBlock) s_d[i] = ca.d[i];
  for (int i = 1 + wid; i < nv - 1; i += kBlock / 64)
    if (lane < i) s_gt[i * (i - 1) / 2 + lane] = ca.G[static_cast<int64_t>(i) * kCgsMax + lane];
  __syncthreads();
  const int nr = (nv - 1) * (nv - 2) / 2;  // the newest row, to LDS and (workgroup 0) to G
  for (int l = threadIdx.x; l < nv - 1; l += kBlock) {
    s_gt[nr + l] = s_d[nv + l];
    if (writer) ca.G[static_cast<int64_t>(nv - 1) * kCgsMax + l] = s_d[nv + l];
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int i = threadIdx.x;
    const double* gi = s_gt + (i > 0 ? i * (i - 1) / 2 : 0);
    double t = i < nv ? s_d[i] : 0.0;
    for (int l = 0; l + 1 < nv; ++l) {
      const double hl = __shfl(t, l, 64);  // h_l: t_l is final once columns 0 .. l-1 are applied
      if (i > l && i < nv) t -= hl * gi[l];
    }
    if (i < nv) {
      s_c[i] = t;
      if (writer && ca.h_out != nullptr) pin_store(ca.h_out + i, t);
    }
  }
  __syncthreads();
}

template <int DOT, bool NT = false, bool FX = false, bool COEF = false>
__global__ __launch_bounds__(kBlock) void cgs_update_kernel(int64_t n, double* __restrict__ w,
                                                            const double* __restrict__ Q, int64_t pitch, int nv,
                                                            const double* __restrict__ coef,
                                                            double* __restrict__ part, int px, YArg yx,
                                                            const double* __restrict__ x0, double* __restrict__ xo,
                                                            int64_t n_gx, CoefArg ca, int tw, int wt) {
  // contraction off: every product rounded, then added, in all three one-reduce kernels (K2w's
  // two passes and K2s), so their arithmetic is fixed by the source, not by the compiler's
  // choice of fused multiply-adds in each kernel
#pragma clang fp contract(off)
  __shared__ double s_c[kCgsMax];
  __shared__ double s_sum[4][4][64];  // [wave][element slot][lane]
  __shared__ double s_x[FX ? 4 : 1][4][64];
  __shared__ double s_wave[4];
  __shared__ double s_gt[COEF ? kGramTri : 1];
  __shared__ double s_d[COEF ? 2 * kCgsMax : 1];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (COEF) {
    icwy_coefficients(ca, nv, s_c, s_gt, s_d);
    if (ca.rpart != nullptr && blockIdx.x == 0) {
      const double t = sum_partials(ca.rpart, ca.r_in, s_wave);
      if (threadIdx.x == 0) publish(ca.r_out, t, ca.flag, ca.seq);
    }
  } else {
    if (threadIdx.x < nv) s_c[threadIdx.x] = coef[threadIdx.x];
    __syncthreads();
  }
  double acc[kCgsPerWave];
#pragma unroll
  for (int m = 0; m < kCgsPerWave; ++m) acc[m] = 0.0;
  const double* Qw = Q + wid * pitch;
  const int64_t step = 4 * pitch;
  const bool vec = aligned16d(w) && aligned16d(Q) && (pitch % 2 == 0) && (!FX || (aligned16d(x0) && aligned16d(xo)));
  const int64_t n_vec = vec ? (n / kCgsChunk) * kCgsChunk : 0;
  // w' = w - Q c: each wave sums its vectors' share (basis order within the wave), the 4 shares
  // combine in a fixed order through LDS (every wave gets the same w'); wave 0 stores it
  for (int64_t e0 = static_cast<int64_t>(blockIdx.x) * kCgsChunk; e0 < n_vec;
       e0 += static_cast<int64_t>(gridDim.x) * kCgsChunk) {
    const int64_t e = e0 + 2 * lane;
    double2 qa[kCgsPerWave], qb[kCgsPerWave];
    double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
    double g0 = 0.0, g1 = 0.0, g2 = 0.0, g3 = 0.0;
    // w (and, for the GEMV's wave, x0) issued with the basis loads: loaded after the barrier, they
    // were a full memory latency per chunk during which the workgroup's other waves sat at the
    // second barrier
    const double2 wa = *reinterpret_cast<const double2*>(w + e);
    const double2 wb = *reinterpret_cast<const double2*>(w + e + 128);
    double2 ba = make_double2(0.0, 0.0), bb = make_double2(0.0, 0.0);
    if (FX && wid == 1) {
      ba = *reinterpret_cast<const double2*>(x0 + e);
      bb = *reinterpret_cast<const double2*>(x0 + e + 128);
    }
#pragma unroll
    for (int m = 0; m < kCgsPerWave; ++m) {
      if (wid + 4 * m < nv) {
        const double* qv = Qw + m * step;
        qa[m] = ld_basis(reinterpret_cast<const double2*>(qv + e), NT && wid + 4 * m >= tw);
        qb[m] = ld_basis(reinterpret_cast<const double2*>(qv + e + 128), NT && wid + 4 * m >= tw);
        const double cm = s_c[wid + 4 * m];
        p0 += cm * qa[m].x;
        p1 += cm * qa[m].y;
        p2 += cm * qb[m].x;
        p3 += cm * qb[m].y;
        if (FX && wid + 4 * m < px) {
          const double ym = yx.v[wid + 4 * m];
          g0 = fma(ym, qa[m].x, g0);
          g1 = fma(ym, qa[m].y, g1);
          g2 = fma(ym, qb[m].x, g2);
          g3 = fma(ym, qb[m].y, g3);
        }
      } else {
        qa[m] = make_double2(0.0, 0.0);
        qb[m] = make_double2(0.0, 0.0);
      }
    }
    s_sum[wid][0][lane] = p0;
    s_sum[wid][1][lane] = p1;
    s_sum[wid][2][lane] = p2;
    s_sum[wid][3][lane] = p3;
    if (FX) {
      s_x[wid][0][lane] = g0;
      s_x[wid][1][lane] = g1;
      s_x[wid][2][lane] = g2;
      s_x[wid][3][lane] = g3;
    }
    __syncthreads();
    double t[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      t[k] = (((s_sum[0][k][lane] + s_sum[1][k][lane]) + s_sum[2][k][lane]) + s_sum[3][k][lane]);
    t[0] = wa.x - t[0];
    t[1] = wa.y - t[1];
    t[2] = wb.x - t[2];
    t[3] = wb.y - t[3];
    if (wid == 0) {  // (buffer stores from the chunk base: sc1 when wt, see st_wt)
      const __amdgpu_buffer_rsrc_t wr = span_rsrc(w + e0);
      if (wt) {
        buf_st2_wt(wr, 16 * lane, make_double2(t[0], t[1]));
        buf_st2_wt(wr, 16 * lane + 1024, make_double2(t[2], t[3]));
      } else {
        buf_st2(wr, 16 * lane, 0, make_double2(t[0], t[1]));
        buf_st2(wr, 16 * lane + 1024, 0, make_double2(t[2], t[3]));
      }
    }
    if (FX && wid == 1) {
      double xs[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        xs[k] = (((s_x[0][k][lane] + s_x[1][k][lane]) + s_x[2][k][lane]) + s_x[3][k][lane]);
      const __amdgpu_buffer_rsrc_t xr = span_rsrc(xo + e0);
      if (wt) {
        buf_st2_wt(xr, 16 * lane, make_double2(xs[0] + ba.x, xs[1] + ba.y));
        buf_st2_wt(xr, 16 * lane + 1024, make_double2(xs[2] + bb.x, xs[3] + bb.y));
      } else {
        buf_st2(xr, 16 * lane, 0, make_double2(xs[0] + ba.x, xs[1] + ba.y));
        buf_st2(xr, 16 * lane + 1024, 0, make_double2(xs[2] + bb.x, xs[3] + bb.y));
      }
    }
    if (DOT) {
#pragma unroll
      for (int m = 0; m < kCgsPerWave; ++m) {
        acc[m] += qa[m].x * t[0];
        acc[m] += qa[m].y * t[1];
        acc[m] += qb[m].x * t[2];
        acc[m] += qb[m].y * t[3];
      }
    } else if (wid == 0) {
      acc[0] += t[0] * t[0];
      acc[0] += t[1] * t[1];
      acc[0] += t[2] * t[2];
      acc[0] += t[3] * t[3];
    }
    __syncthreads();
  }
  // scalar tail (odd / unaligned n): the same 4-wave structure, one element per lane
  for (int64_t e0 = n_vec + static_cast<int64_t>(blockIdx.x) * 64; e0 < n; e0 += static_cast<int64_t>(gridDim.x) * 64) {
    const int64_t e = e0 + lane;
    const bool ok = e < n;
    double q[kCgsPerWave];
    double ps = 0.0, gs = 0.0;
#pragma unroll
    for (int m = 0; m < kCgsPerWave; ++m) {
      q[m] = (ok && wid + 4 * m < nv) ? Qw[m * step + e] : 0.0;
      if (wid + 4 * m < nv) ps += s_c[wid + 4 * m] * q[m];
      if (FX && wid + 4 * m < px) gs = fma(yx.v[wid + 4 * m], q[m], gs);
    }
    const double we = ok ? w[e] : 0.0;
    s_sum[wid][0][lane] = ps;
    if (FX) s_x[wid][0][lane] = gs;
    __syncthreads();
    const double t = we - (((s_sum[0][0][lane] + s_sum[1][0][lane]) + s_sum[2][0][lane]) + s_sum[3][0][lane]);
    if (wid == 0 && ok) st_out(w + e, t, wt);
    if (FX && wid == 1 && ok)
      st_out(xo + e, (((s_x[0][0][lane] + s_x[1][0][lane]) + s_x[2][0][lane]) + s_x[3][0][lane]) + x0[e], wt);
    if (DOT) {
#pragma unroll
      for (int m = 0; m < kCgsPerWave; ++m) acc[m] += q[m] * t;
    } else if (wid == 0) {
      acc[0] += t * t;
    }
    __syncthreads();
  }
  if (FX) {  // x's ghost rows: the four wave sums in wave order, each over its vectors in order
    for (int64_t e = n + static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; e < n_gx;
         e += static_cast<int64_t>(gridDim.x) * kBlock) {
      double sw[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        double g = 0.0;
        for (int l = v; l < px; l += 4) g = fma(yx.v[l], Q[static_cast<int64_t>(l) * pitch + e], g);
        sw[v] = g;
      }
      xo[e] = (((sw[0] + sw[1]) + sw[2]) + sw[3]) + x0[e];
    }
  }
  if (DOT) {
#pragma unroll
    for (int m = 0; m < kCgsPerWave; ++m) {
      const int i = wid + 4 * m;
      if (i < nv) {
        const double t = wave_sum(acc[m]);
        if (lane == 0) part[static_cast<int64_t>(i) * gridDim.x + blockIdx.x] = t;
      }
    }
  } else {
    const double tot = block_sum(acc[0], s_wave);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
  }
}

// ---------------------------------------------------------------------------------------------
// Multi-dot for the incremental constraint Gram (spis.cpp con_inc_enqueue): part[i * grid + blk]
// = the workgroup's partial of L.v[i] . u, i < nvec (<= kMdMax), where the last n2 vectors take u2
// instead of u (a constraint's v . z_a riding with its M z_a pass).  Vector i goes to wave i % 4
// (as cgs_dot): each wave reads u's (and u2's) chunk once for its vectors; 256-element chunks per
// workgroup iteration (16-B loads when every pointer is 16-B aligned), a scalar tail otherwise;
// the products are rounded, then added (contraction off); fixed-order wave sums.
// GX: the update GEMV of the step before rides along, xo = x0 + sum_{i < px} y_i L.v[i] (L.v[0 ..
// px-1] = z_0 .. z_{px-1}, read here anyway): each wave sums its vectors' terms in order, the
// four waves' sums are added in wave order through LDS, then x0 (numpy's Z @ y + x0 order).
// Bytes: (nvec + 4 (+ 4)) 8 N (+ 16 N with GX).
// ---------------------------------------------------------------------------------------------
template <bool GX>
__global__ __launch_bounds__(kBlock) void multidot_kernel(int64_t n, const double* __restrict__ u, VecList L,
                                                          int nvec, const double* __restrict__ u2, int n2, bool vec,
                                                          double* __restrict__ part, int px, YArg ya,
                                                          const double* __restrict__ x0, double* __restrict__ xo) {
#pragma clang fp contract(off)
  constexpr int kPerW = kMdMax / 4;
  __shared__ double s_g[GX ? 4 : 1][4][64];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int first2 = nvec - n2;  // vectors first2 .. nvec - 1 are dotted with u2
  double acc[kPerW];
#pragma unroll
  for (int m = 0; m < kPerW; ++m) acc[m] = 0.0;
  const int64_t n_vec = vec ? (n / kCgsChunk) * kCgsChunk : 0;
  for (int64_t e0 = static_cast<int64_t>(blockIdx.x) * kCgsChunk; e0 < n_vec;
       e0 += static_cast<int64_t>(gridDim.x) * kCgsChunk) {
    const int64_t e = e0 + 2 * lane;
    const double2 ua = *reinterpret_cast<const double2*>(u + e);
    const double2 ub = *reinterpret_cast<const double2*>(u + e + 128);
    double2 wa = make_double2(0.0, 0.0), wb = wa;
    if (n2 > 0) {
      wa = *reinterpret_cast<const double2*>(u2 + e);
      wb = *reinterpret_cast<const double2*>(u2 + e + 128);
    }
    double g0 = 0.0, g1 = 0.0, g2 = 0.0, g3 = 0.0;
#pragma unroll
    for (int m = 0; m < kPerW; ++m) {
      const int i = wid + 4 * m;
      if (i < nvec) {
        const double2 va = *reinterpret_cast<const double2*>(L.v[i] + e);
        const double2 vb = *reinterpret_cast<const double2*>(L.v[i] + e + 128);
        const double2 xa = i < first2 ? ua : wa, xb = i < first2 ? ub : wb;
        acc[m] += va.x * xa.x;
        acc[m] += va.y * xa.y;
        acc[m] += vb.x * xb.x;
        acc[m] += vb.y * xb.y;
        if (GX && i < px) {
          const double yi = ya.v[i];
          g0 += yi * va.x;
          g1 += yi * va.y;
          g2 += yi * vb.x;
          g3 += yi * vb.y;
        }
      }
    }
    if (GX) {
      s_g[wid][0][lane] = g0;
      s_g[wid][1][lane] = g1;
      s_g[wid][2][lane] = g2;
      s_g[wid][3][lane] = g3;
      __syncthreads();
      if (wid == 0) {
        double t[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) t[q] = ((s_g[0][q][lane] + s_g[1][q][lane]) + s_g[2][q][lane]) + s_g[3][q][lane];
        const double2 xa = *reinterpret_cast<const double2*>(x0 + e);
        const double2 xb = *reinterpret_cast<const double2*>(x0 + e + 128);
        *reinterpret_cast<double2*>(xo + e) = make_double2(t[0] + xa.x, t[1] + xa.y);
        *reinterpret_cast<double2*>(xo + e + 128) = make_double2(t[2] + xb.x, t[3] + xb.y);
      }
      __syncthreads();
    }
  }
  // the scalar tail: 64 elements per workgroup iteration, the trip count uniform over the
  // workgroup (GX's barriers), lanes past n idle
  for (int64_t eb = n_vec + static_cast<int64_t>(blockIdx.x) * 64; eb < n; eb += static_cast<int64_t>(gridDim.x) * 64) {
    const int64_t e = eb + lane;
    const bool in = e < n;
    const double ue = in ? u[e] : 0.0;
    const double we = in && n2 > 0 ? u2[e] : 0.0;
    double ge = 0.0;
#pragma unroll
    for (int m = 0; m < kPerW; ++m) {
      const int i = wid + 4 * m;
      if (i < nvec && in) {
        const double le = L.v[i][e];
        acc[m] += le * (i < first2 ? ue : we);
        if (GX && i < px) ge += ya.v[i] * le;
      }
    }
    if (GX) {
      s_g[wid][0][lane] = ge;
      __syncthreads();
      if (wid == 0 && in) xo[e] = ((s_g[0][0][lane] + s_g[1][0][lane]) + s_g[2][0][lane]) + s_g[3][0][lane] + x0[e];
      __syncthreads();
    }
  }
#pragma unroll
  for (int m = 0; m < kPerW; ++m) {
    const int i = wid + 4 * m;
    if (i < nvec) {
      const double t = wave_sum(acc[m]);
      if (lane == 0) part[static_cast<int64_t>(i) * gridDim.x + blockIdx.x] = t;
    }
  }
}

hipError_t launch_multidot(int64_t n, const double* u, const VecList& L, int nvec, double* part, int grid,
                           hipStream_t s, const double* u2, int n2, int px, const double* y, const double* x0,
                           double* xo) {
  if (nvec < 1 || nvec > kMdMax || grid < 1 || grid > kRedGrid || n2 < 0 || n2 > nvec || (n2 > 0 && u2 == nullptr) ||
      px < 0 || px > nvec - n2 || px > kYArg || (px > 0 && (y == nullptr || x0 == nullptr || xo == nullptr)))
    return hipErrorInvalidValue;
  bool vec = aligned16d(u) && (n2 == 0 || aligned16d(u2)) && (px == 0 || (aligned16d(x0) && aligned16d(xo)));
  for (int i = 0; i < nvec; ++i) vec = vec && aligned16d(L.v[i]);
  YArg ya;
  for (int i = 0; i < px; ++i) ya.v[i] = y[i];
  if (px > 0)
    hipLaunchKernelGGL(multidot_kernel<true>, dim3(grid), dim3(kBlock), 0, s, n, u, L, nvec, u2, n2, vec, part, px, ya,
                       x0, xo);
  else
    hipLaunchKernelGGL(multidot_kernel<false>, dim3(grid), dim3(kBlock), 0, s, n, u, L, nvec, u2, n2, vec, part, 0, ya,
                       x0, xo);
  return hipGetLastError();
}

// workgroup i reduces vector i's partials; add (nullable) + c -> h_out (host H column, nullable)
// zero_to > gridDim.x: workgroup 0 also zeroes c[gridDim.x, zero_to) (the slack a merged
// all-reduce carries beside the dots: summed every step, it must not grow)
// pin: c is host memory a host thread polls (system-scope stores, each value its own flag)
__global__ __launch_bounds__(kBlock) void cgs_finalize_kernel(const double* __restrict__ part, int n_in,
                                                              double* __restrict__ c, const double* __restrict__ add,
                                                              double* __restrict__ h_out, int zero_to, bool pin) {
  __shared__ double s_wave[4];
  const int i = blockIdx.x;
  const double t = sum_partials(part + static_cast<int64_t>(i) * n_in, n_in, s_wave);
  if (threadIdx.x == 0) {
    if (pin)
      pin_store(c + i, t);
    else
      c[i] = t;
    if (h_out != nullptr) h_out[i] = add[i] + t;
  }
  if (i == 0)
    for (int z = static_cast<int>(gridDim.x) + threadIdx.x; z < zero_to; z += kBlock) c[z] = 0.0;
}

hipError_t launch_cgs_dot(int64_t n, const double* w, const double* Q, int64_t pitch, int nv, double* part, int grid,
                          hipStream_t s, const LaunchEv* ev) {
  if (nv < 1 || nv > kCgsMax) return hipErrorInvalidValue;
  launch_k(cgs_dot_kernel, dim3(grid), dim3(kBlock), 0, s, ev, n, w, Q, pitch, nv, part);
  return hipGetLastError();
}

template <bool NT, bool FX, bool COEF>
static void launch_update0(int grid, hipStream_t s, int64_t n, double* w, const double* Q, int64_t pitch, int nv,
                           const double* coef, double* part, int px, const YArg& ya, const double* x0, double* xo,
                           int64_t n_gx, const CoefArg& ca, int tw) {
  hipLaunchKernelGGL((cgs_update_kernel<0, NT, FX, COEF>), dim3(grid), dim3(kBlock), 0, s, n, w, Q, pitch, nv, coef,
                     part, px, ya, x0, xo, n_gx, ca, tw, wt_k2w());
}

template <bool NT, bool FX>
static void launch_update0c(bool cf, int grid, hipStream_t s, int64_t n, double* w, const double* Q, int64_t pitch,
                            int nv, const double* coef, double* part, int px, const YArg& ya, const double* x0,
                            double* xo, int64_t n_gx, const CoefArg& ca, int tw) {
  if (cf)
    launch_update0<NT, FX, true>(grid, s, n, w, Q, pitch, nv, coef, part, px, ya, x0, xo, n_gx, ca, tw);
  else
    launch_update0<NT, FX, false>(grid, s, n, w, Q, pitch, nv, coef, part, px, ya, x0, xo, n_gx, ca, tw);
}

static hipError_t cgs_update_any(int64_t n, double* w, const double* Q, int64_t pitch, int nv, const double* coef,
                                 bool dot, double* part, int grid, hipStream_t s, bool nt, int px, const double* yx,
                                 const double* x0, double* xo, int64_t n_gx, const CoefArg& ca, int tw = 0) {
  if (nv < 1 || nv > kCgsMax) return hipErrorInvalidValue;
  YArg ya;
  const bool fx = px > 0;
  if (fx) {
    if (dot || px > nv || px > kYArg || yx == nullptr || x0 == nullptr || xo == nullptr || n_gx < n)
      return hipErrorInvalidValue;
    for (int i = 0; i < px; ++i) ya.v[i] = yx[i];
  }
  const bool cf = ca.d != nullptr;
  if (cf && (dot || ca.G == nullptr)) return hipErrorInvalidValue;
  if (dot)
    hipLaunchKernelGGL(cgs_update_kernel<1>, dim3(grid), dim3(kBlock), 0, s, n, w, Q, pitch, nv, coef, part, 0, ya,
                       x0, xo, n_gx, ca, 0, wt_k2w());
  else if (fx && nt)
    launch_update0c<true, true>(cf, grid, s, n, w, Q, pitch, nv, coef, part, px, ya, x0, xo, n_gx, ca, tw);
  else if (fx)
    launch_update0c<false, true>(cf, grid, s, n, w, Q, pitch, nv, coef, part, px, ya, x0, xo, n_gx, ca, tw);
  else if (nt)
    launch_update0c<true, false>(cf, grid, s, n, w, Q, pitch, nv, coef, part, 0, ya, x0, xo, n_gx, ca, tw);
  else
    launch_update0c<false, false>(cf, grid, s, n, w, Q, pitch, nv, coef, part, 0, ya, x0, xo, n_gx, ca, tw);
  return hipGetLastError();
}

hipError_t launch_cgs_update(int64_t n, double* w, const double* Q, int64_t pitch, int nv, const double* coef,
                             bool dot, double* part, int grid, hipStream_t s, bool nt, int px, const double* yx,
                             const double* x0, double* xo, int64_t n_gx) {
  return cgs_update_any(n, w, Q, pitch, nv, coef, dot, part, grid, s, nt, px, yx, x0, xo, n_gx,
                        CoefArg{nullptr, nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr});
}

hipError_t launch_icwy_update(int64_t n, double* w, const double* Q, int64_t pitch, int nv, const double* d,
                              double* G, double* h_out, double* part, int grid, hipStream_t s, bool nt, int px,
                              const double* yx, const double* x0, double* xo, int64_t n_gx, const double* rpart,
                              int r_in, double* r_out, unsigned long long* flag, const unsigned long long* seq,
                              int tw) {
  if (d == nullptr || (rpart != nullptr && (r_in < 1 || r_out == nullptr))) return hipErrorInvalidValue;
  return cgs_update_any(n, w, Q, pitch, nv, nullptr, false, part, grid, s, nt, px, yx, x0, xo, n_gx,
                        CoefArg{d, G, h_out, rpart, r_in, r_out, flag, seq}, tw);
}

hipError_t launch_cgs_finalize(const double* part, int n_in, int nv, double* c, const double* add, double* h_out,
                               hipStream_t s, int zero_to, bool pin) {
  hipLaunchKernelGGL(cgs_finalize_kernel, dim3(nv), dim3(kBlock), 0, s, part, n_in, c, add, h_out, zero_to, pin);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K2w: one-reduce MGS for several GPUs (MGS in its inverse-compact-WY form).  MGS's projections
// h_l = q_l . w^(l), w^(l+1) = w^(l) - h_l q_l are, by the distributive law K2q uses with a lag
// of 2, h_l = q_l . w - sum_{m<l} h_m G(l, m) with G(l, m) = q_l . q_m: one pass computes every
// q_l . w and the newest Gram row G(j, .) (q_j arrived with the previous step), ONE all-reduce
// carries them, one workgroup forms h in l order (the same correction order as K2q's gatherer),
// then cgs_update subtracts Q h with the ||w'||^2 partials (the second all-reduce) and K3
// normalises.  Two reductions per Arnoldi step instead of MGS's j + 2; exact arithmetic is MGS's.
// ---------------------------------------------------------------------------------------------
// The fold (FOLD, the default): the launch also reduces its own partials into d, so no finalize
// launch (4.9 us + its gap per Arnoldi step at C3) sits between the dots and the update.  Each
// workgroup publishes its partial of value i as two tagged 32-bit halves (chain_store: agent-scope
// relaxed stores, each slot its own flag, no fence, the K2q exchange's protocol); the LAST
// min(grid, 2 nv - 1) workgroups of the grid, dispatched after every producer, then each reduce
// value r, r + nred, ... in sum_partials' order (thread t: partials t, t + 256, ... then
// block_sum), so d is bitwise cgs_finalize's.  tag: a per-launch host counter (never 0), so the
// slots need no reset; a spin bounded by kChainWaitTicks sets *err instead of hanging.
// tw: basis vectors l < tw load with ordinary loads (they stay in the Infinity Cache, as K2q's).
template <bool NT, bool FOLD>
__global__ __launch_bounds__(kBlock) void icwy_dot_kernel(int64_t n, const double* __restrict__ w,
                                                          const double* __restrict__ Q, int64_t pitch, int nv,
                                                          double* __restrict__ part, int tw,
                                                          unsigned long long* __restrict__ slots, unsigned tag,
                                                          double* __restrict__ d, int zero_to, unsigned* err) {
  // contraction off: every product rounded, then added, in all three one-reduce kernels (K2w's
  // two passes and K2s), so their arithmetic is fixed by the source, not by the compiler's
  // choice of fused multiply-adds in each kernel
#pragma clang fp contract(off)
  // rows [0, nv): q_l . w ; rows [nv, 2 nv - 1): q_l . q_{nv-1}, l < nv - 1
  __shared__ double s_wave[4];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  double acc[kCgsPerWave], acg[kCgsPerWave];
#pragma unroll
  for (int m = 0; m < kCgsPerWave; ++m) acc[m] = acg[m] = 0.0;
  const double* Qw = Q + wid * pitch;
  const double* ql = Q + static_cast<int64_t>(nv - 1) * pitch;
  const int64_t step = 4 * pitch;
  const bool vec = aligned16d(w) && aligned16d(Q) && (pitch % 2 == 0);
  const int64_t n_vec = vec ? (n / kCgsChunk) * kCgsChunk : 0;
  for (int64_t e0 = static_cast<int64_t>(blockIdx.x) * kCgsChunk; e0 < n_vec;
       e0 += static_cast<int64_t>(gridDim.x) * kCgsChunk) {
    const int64_t e = e0 + 2 * lane;
    const double2 wa = *reinterpret_cast<const double2*>(w + e);
    const double2 wb = *reinterpret_cast<const double2*>(w + e + 128);
    const double2 la = *reinterpret_cast<const double2*>(ql + e);
    const double2 lb = *reinterpret_cast<const double2*>(ql + e + 128);
#pragma unroll
    for (int m = 0; m < kCgsPerWave; ++m) {
      const int i = wid + 4 * m;
      if (i < nv) {
        const double* qv = Qw + m * step;
        const double2 qa = ld_basis(reinterpret_cast<const double2*>(qv + e), NT && i >= tw);
        const double2 qb = ld_basis(reinterpret_cast<const double2*>(qv + e + 128), NT && i >= tw);
        acc[m] += qa.x * wa.x;
        acc[m] += qa.y * wa.y;
        acc[m] += qb.x * wb.x;
        acc[m] += qb.y * wb.y;
        if (i < nv - 1) {
          acg[m] += qa.x * la.x;
          acg[m] += qa.y * la.y;
          acg[m] += qb.x * lb.x;
          acg[m] += qb.y * lb.y;
        }
      }
    }
  }
  for (int64_t e = n_vec + static_cast<int64_t>(blockIdx.x) * 64 + lane; e < n;
       e += static_cast<int64_t>(gridDim.x) * 64) {
    const double we = w[e];
    const double le = ql[e];
#pragma unroll
    for (int m = 0; m < kCgsPerWave; ++m) {
      const int i = wid + 4 * m;
      if (i < nv) {
        const double q = Qw[m * step + e];
        acc[m] += q * we;
        if (i < nv - 1) acg[m] += q * le;
      }
    }
  }
  const int gc = static_cast<int>(gridDim.x);
  auto put = [&](int i, double t) {
    if (FOLD) {
      const unsigned long long u = static_cast<unsigned long long>(__double_as_longlong(t));
      unsigned long long* sl = slots + 2 * (static_cast<int64_t>(i) * gc + blockIdx.x);
      chain_store(sl, tag, static_cast<unsigned>(u));
      chain_store(sl + 1, tag, static_cast<unsigned>(u >> 32));
    } else {
      part[static_cast<int64_t>(i) * gc + blockIdx.x] = t;
    }
  };
#pragma unroll
  for (int m = 0; m < kCgsPerWave; ++m) {
    const int i = wid + 4 * m;
    if (i < nv) {
      const double t = wave_sum(acc[m]);
      if (lane == 0) put(i, t);
    }
    if (i < nv - 1) {
      const double t = wave_sum(acg[m]);
      if (lane == 0) put(nv + i, t);
    }
  }
  if (!FOLD) return;
  const int nval = 2 * nv - 1;
  const int nred = min(gc, nval);
  const int r = static_cast<int>(blockIdx.x) - (gc - nred);
  if (r < 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = r; i < nval; i += nred) {
    const unsigned long long* sl = slots + 2 * static_cast<int64_t>(i) * gc;
    constexpr int kPer = kRedGrid / kBlock;  // partials per thread (gc <= kRedGrid)
    unsigned long long g[2 * kPer];
    for (unsigned spins = 0;; ++spins) {
      bool ok = true;
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        const int b = threadIdx.x + k * kBlock;
        if (b < gc) {
          g[2 * k] = chain_load(sl + 2 * b);
          g[2 * k + 1] = chain_load(sl + 2 * b + 1);
          ok &= static_cast<unsigned>(g[2 * k] >> 32) == tag && static_cast<unsigned>(g[2 * k + 1] >> 32) == tag;
        }
      }
      if (__all(ok)) break;
      if ((spins & 63) == 63 && __builtin_amdgcn_s_memrealtime() - t0 > kChainWaitTicks) {
        if (lane == 0) atomicOr(err, 2u);
        break;
      }
    }
    double v = 0.0;
#pragma unroll
    for (int k = 0; k < kPer; ++k)
      if (threadIdx.x + k * kBlock < gc)
        v += __longlong_as_double(static_cast<long long>((g[2 * k + 1] << 32) | (g[2 * k] & 0xffffffffull)));
    const double tot = block_sum(v, s_wave);
    if (threadIdx.x == 0) d[i] = tot;
  }
  if (r == 0)
    for (int z = nval + static_cast<int>(threadIdx.x); z < zero_to; z += kBlock) d[z] = 0.0;
}

hipError_t launch_icwy_dot(int64_t n, const double* w, const double* Q, int64_t pitch, int nv, double* part, int grid,
                           hipStream_t s, const LaunchEv* ev, bool nt, int tw, unsigned long long* slots,
                           unsigned tag, double* d, int zero_to, unsigned* err) {
  if (nv < 1 || nv > kCgsMax || grid < 1 || grid > kRedGrid) return hipErrorInvalidValue;
  const bool fold = slots != nullptr;
  if (fold && (tag == 0 || d == nullptr || err == nullptr)) return hipErrorInvalidValue;
  if (fold && nt)
    launch_k(icwy_dot_kernel<true, true>, dim3(grid), dim3(kBlock), 0, s, ev, n, w, Q, pitch, nv, part, tw, slots,
             tag, d, zero_to, err);
  else if (fold)
    launch_k(icwy_dot_kernel<false, true>, dim3(grid), dim3(kBlock), 0, s, ev, n, w, Q, pitch, nv, part, tw, slots,
             tag, d, zero_to, err);
  else if (nt)
    launch_k(icwy_dot_kernel<true, false>, dim3(grid), dim3(kBlock), 0, s, ev, n, w, Q, pitch, nv, part, tw, slots,
             tag, d, zero_to, err);
  else
    launch_k(icwy_dot_kernel<false, false>, dim3(grid), dim3(kBlock), 0, s, ev, n, w, Q, pitch, nv, part, tw, slots,
             tag, d, zero_to, err);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K2s: K2w in ONE launch and ONE pass over the basis, for small N on one GPU.  Each workgroup owns
// one 256-element chunk (grid = ceil(n / 256), every workgroup resident at once: the host checks
// the occupancy), and its four waves keep their basis vectors' slices of it in registers from the
// dots to the update:
//   1. the dots of icwy_dot (q_l . w, q_l . q_{nv-1}) -> tagged partial slots (as the fold);
//   2. the last min(grid, 2 nv - 1) workgroups reduce them (sum_partials' order) and publish each
//      reduced dot as tagged halves; every workgroup polls the 2 nv - 1 of them;
//   3. icwy_coefficients (every workgroup the same bits; workgroup 0 writes G's row and H[:, j]);
//   4. cgs_update's arithmetic on the register slices: w' (stored), the fused GEMV, ||w'||^2
//      partial -> tagged slot;
//   5. the last workgroup reduces the norm partials and publishes ||w'||^2; every workgroup forms
//      q_{j+1} = w' / ||w'|| as normalize_kernel does (workgroup 0: H[j+1, j] to the host).
// For n a multiple of 256 (n <= 262,144) the two-pass launches group every partial and every sum
// the same way, and all three kernels compile with contraction off, so the solves are bitwise
// equal (tests/test_gpu_parity.py, n = 65,536 and 196,608; with contraction on, hipcc had fused
// different multiply-adds in the two forms and one ||w'|| at 196,608 came out one ulp apart);
// otherwise the last chunk's elements are grouped differently (the two-pass kernels take them in
// a scalar tail): roundoff.
// Spins are bounded (kChainWaitTicks) and set *err, as the chain's.
// slots: [P: 2 (2 kCgsMax - 1) kRedGrid][D: 2 (2 kCgsMax - 1)][N: 2 kRedGrid][H: 2] words.
// ---------------------------------------------------------------------------------------------
constexpr int64_t kOnePassP = 2 * (2 * kCgsMax - 1) * static_cast<int64_t>(kRedGrid);
constexpr int64_t kOnePassD = kOnePassP;
constexpr int64_t kOnePassN = kOnePassD + 2 * (2 * kCgsMax - 1);
constexpr int64_t kOnePassH = kOnePassN + 2 * kRedGrid;

__device__ __forceinline__ void tag_put(unsigned long long* sl, unsigned tag, double v) {
  const unsigned long long u = static_cast<unsigned long long>(__double_as_longlong(v));
  chain_store(sl, tag, static_cast<unsigned>(u));
  chain_store(sl + 1, tag, static_cast<unsigned>(u >> 32));
}
// one lane's tagged double: spins until both halves carry tag (false: timed out, *err set)
__device__ __forceinline__ bool tag_get(const unsigned long long* sl, unsigned tag, double* v,
                                        unsigned long long t0, unsigned* err) {
  for (unsigned spins = 0;; ++spins) {
    const unsigned long long lo = chain_load(sl), hi = chain_load(sl + 1);
    if (static_cast<unsigned>(lo >> 32) == tag && static_cast<unsigned>(hi >> 32) == tag) {
      *v = __longlong_as_double(static_cast<long long>((hi << 32) | (lo & 0xffffffffull)));
      return true;
    }
    if ((spins & 63) == 63 && __builtin_amdgcn_s_memrealtime() - t0 > kChainWaitTicks) {
      atomicOr(err, 2u);
      *v = 0.0;
      return false;
    }
  }
}
// the workgroup sums grid (<= kRedGrid) tagged partials (slot pairs at sl + 2 b) in sum_partials'
// order; each thread's slots are loaded together and re-polled until all carry tag
__device__ __forceinline__ double tag_sum(const unsigned long long* sl, int grid, unsigned tag, double* s_wave,
                                          unsigned long long t0, unsigned* err) {
  constexpr int kPer = kRedGrid / kBlock;
  unsigned long long g[2 * kPer];
  for (unsigned spins = 0;; ++spins) {
    bool ok = true;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int b = threadIdx.x + k * kBlock;
      if (b < grid) {
        g[2 * k] = chain_load(sl + 2 * b);
        g[2 * k + 1] = chain_load(sl + 2 * b + 1);
        ok &= static_cast<unsigned>(g[2 * k] >> 32) == tag && static_cast<unsigned>(g[2 * k + 1] >> 32) == tag;
      }
    }
    if (__all(ok)) break;
    if ((spins & 63) == 63 && __builtin_amdgcn_s_memrealtime() - t0 > kChainWaitTicks) {
      if ((threadIdx.x & 63) == 0) atomicOr(err, 2u);
      break;
    }
  }
  double v = 0.0;
#pragma unroll
  for (int k = 0; k < kPer; ++k)
    if (threadIdx.x + k * kBlock < grid)
      v += __longlong_as_double(static_cast<long long>((g[2 * k + 1] << 32) | (g[2 * k] & 0xffffffffull)));
  return block_sum(v, s_wave);
}

template <bool FX, bool TWO>
__global__ __launch_bounds__(kBlock, 4) void icwy_onepass_kernel(int64_t n, double* __restrict__ w,
                                                              const double* __restrict__ Q, double* __restrict__ qn,
                                                              int64_t pitch, int nv, unsigned long long* slots,
                                                              unsigned tag, unsigned* err, CoefArg ca, int px,
                                                              YArg yx, const double* __restrict__ x0,
                                                              double* __restrict__ xo, double* h_out) {
  // contraction off: every product rounded, then added, in all three one-reduce kernels (K2w's
  // two passes and K2s), so their arithmetic is fixed by the source, not by the compiler's
  // choice of fused multiply-adds in each kernel
#pragma clang fp contract(off)
  __shared__ double s_c[kCgsMax];
  __shared__ double s_sum[4][4][64];
  __shared__ double s_x[FX ? 4 : 1][4][64];
  __shared__ double s_wave[4];
  __shared__ double s_gt[kGramTri];
  __shared__ double s_d[2 * kCgsMax];
  __shared__ double s_h;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grid = static_cast<int>(gridDim.x);
  const int nval = 2 * nv - 1;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const int64_t e = static_cast<int64_t>(blockIdx.x) * kCgsChunk + 2 * lane;  // e, e+1, e+128, e+129
  // TWO: the workgroup also owns chunk blockIdx.x + grid (when it exists), streamed from memory in
  // both passes instead of held in registers (n up to twice the resident chunks)
  const int64_t e2 = (static_cast<int64_t>(blockIdx.x) + grid) * kCgsChunk + 2 * lane;
  const bool two = TWO && (static_cast<int64_t>(blockIdx.x) + grid) * kCgsChunk < n;
  auto ld2 = [&](const double* p, int64_t i) -> double2 {
    if (i + 1 < n) return *reinterpret_cast<const double2*>(p + i);
    return make_double2(i < n ? p[i] : 0.0, 0.0);
  };
  auto st2 = [&](double* p, int64_t i, double a, double b) {
    if (i + 1 < n)
      *reinterpret_cast<double2*>(p + i) = make_double2(a, b);
    else if (i < n)
      p[i] = a;
  };
  const double* Qw = Q + wid * pitch;
  const int64_t step = 4 * pitch;
  const double2 wa = ld2(w, e), wb = ld2(w, e + 128);
  double2 ba = make_double2(0.0, 0.0), bb = make_double2(0.0, 0.0);
  if (FX && wid == 1) {
    ba = ld2(x0, e);
    bb = ld2(x0, e + 128);
  }
  // 0. the previous update's true residual (its partials are complete: stream order), published
  // before anything else, so that the host, which enqueues the next dual SpMV once it has read it,
  // gets the whole launch to do so (published after the dots, it left a 3-10 us gap before that
  // SpMV at C2 and C4)
  if (ca.rpart != nullptr && blockIdx.x == 0) {
    const double t = sum_partials(ca.rpart, ca.r_in, s_wave);
    if (threadIdx.x == 0) publish(ca.r_out, t, ca.flag, ca.seq);
  }
  double2 qa[kCgsPerWave], qb[kCgsPerWave];
  {
    const double* ql = Q + static_cast<int64_t>(nv - 1) * pitch;
    const double2 la = ld2(ql, e), lb = ld2(ql, e + 128);
    double2 wa2 = make_double2(0.0, 0.0), wb2 = wa2, la2 = wa2, lb2 = wa2;
    if (two) {
      wa2 = ld2(w, e2);
      wb2 = ld2(w, e2 + 128);
      la2 = ld2(ql, e2);
      lb2 = ld2(ql, e2 + 128);
    }
    // 1. the dots, icwy_dot's arithmetic (TWO: the second chunk's products after the first's)
#pragma unroll
    for (int m = 0; m < kCgsPerWave; ++m) {
      const int i = wid + 4 * m;
      if (i < nv) {
        qa[m] = ld2(Qw + m * step, e);
        qb[m] = ld2(Qw + m * step, e + 128);
      } else {
        qa[m] = make_double2(0.0, 0.0);
        qb[m] = make_double2(0.0, 0.0);
      }
    }
#pragma unroll
    for (int m = 0; m < kCgsPerWave; ++m) {
      const int i = wid + 4 * m;
      if (i < nv) {
        double2 qa2 = make_double2(0.0, 0.0), qb2 = qa2;
        if (two) {
          qa2 = ld2(Qw + m * step, e2);
          qb2 = ld2(Qw + m * step, e2 + 128);
        }
        double acc = 0.0, acg = 0.0;
        acc += qa[m].x * wa.x;
        acc += qa[m].y * wa.y;
        acc += qb[m].x * wb.x;
        acc += qb[m].y * wb.y;
        if (two) {
          acc += qa2.x * wa2.x;
          acc += qa2.y * wa2.y;
          acc += qb2.x * wb2.x;
          acc += qb2.y * wb2.y;
        }
        acc = wave_sum(acc);
        if (lane == 0) tag_put(slots + 2 * (static_cast<int64_t>(i) * grid + blockIdx.x), tag, acc);
        if (i < nv - 1) {
          acg += qa[m].x * la.x;
          acg += qa[m].y * la.y;
          acg += qb[m].x * lb.x;
          acg += qb[m].y * lb.y;
          if (two) {
            acg += qa2.x * la2.x;
            acg += qa2.y * la2.y;
            acg += qb2.x * lb2.x;
            acg += qb2.y * lb2.y;
          }
          acg = wave_sum(acg);
          if (lane == 0) tag_put(slots + 2 * (static_cast<int64_t>(nv + i) * grid + blockIdx.x), tag, acg);
        }
      }
    }
  }
  // 2. the last workgroups reduce the dots and publish them; everyone polls
  const int nred = min(grid, nval);
  const int r = static_cast<int>(blockIdx.x) - (grid - nred);
  if (r >= 0)
    for (int i = r; i < nval; i += nred) {
      const double tot = tag_sum(slots + 2 * static_cast<int64_t>(i) * grid, grid, tag, s_wave, t0, err);
      if (threadIdx.x == 0) tag_put(slots + kOnePassD + 2 * i, tag, tot);
    }
  if (threadIdx.x < nval) tag_get(slots + kOnePassD + 2 * threadIdx.x, tag, &s_d[threadIdx.x], t0, err);
  __syncthreads();
  // 3. the coefficients (d already in s_d: ca.d == nullptr)
  icwy_coefficients(ca, nv, s_c, s_gt, s_d);
  // 4. cgs_update's arithmetic on one chunk's slices (the register ones, or TWO's second chunk
  // loaded again): w' = w - sum (stored), the fused GEMV, wave 0's ||w'||^2 terms into a0
  double a0 = 0.0;
  auto update = [&](int64_t ec, const double2 (&ua)[kCgsPerWave], const double2 (&ub)[kCgsPerWave], double2 va,
                    double2 vb, double2 xa, double2 xb, double (&t)[4]) __attribute__((always_inline)) {
    double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
    double g0 = 0.0, g1 = 0.0, g2 = 0.0, g3 = 0.0;
#pragma unroll
    for (int m = 0; m < kCgsPerWave; ++m) {
      if (wid + 4 * m < nv) {
        const double cm = s_c[wid + 4 * m];
        p0 += cm * ua[m].x;
        p1 += cm * ua[m].y;
        p2 += cm * ub[m].x;
        p3 += cm * ub[m].y;
        if (FX && wid + 4 * m < px) {
          const double ym = yx.v[wid + 4 * m];
          g0 = fma(ym, ua[m].x, g0);
          g1 = fma(ym, ua[m].y, g1);
          g2 = fma(ym, ub[m].x, g2);
          g3 = fma(ym, ub[m].y, g3);
        }
      }
    }
    s_sum[wid][0][lane] = p0;
    s_sum[wid][1][lane] = p1;
    s_sum[wid][2][lane] = p2;
    s_sum[wid][3][lane] = p3;
    if (FX) {
      s_x[wid][0][lane] = g0;
      s_x[wid][1][lane] = g1;
      s_x[wid][2][lane] = g2;
      s_x[wid][3][lane] = g3;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) t[k] = (((s_sum[0][k][lane] + s_sum[1][k][lane]) + s_sum[2][k][lane]) + s_sum[3][k][lane]);
    t[0] = va.x - t[0];
    t[1] = va.y - t[1];
    t[2] = vb.x - t[2];
    t[3] = vb.y - t[3];
    // the tail of a chunk past n holds zeros (ld2), so its t are 0 and add nothing below
    if (wid == 0) {
      st2(w, ec, t[0], t[1]);
      st2(w, ec + 128, t[2], t[3]);
    }
    if (FX && wid == 1) {
      double xs[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) xs[k] = (((s_x[0][k][lane] + s_x[1][k][lane]) + s_x[2][k][lane]) + s_x[3][k][lane]);
      st2(xo, ec, xs[0] + xa.x, xs[1] + xa.y);
      st2(xo, ec + 128, xs[2] + xb.x, xs[3] + xb.y);
    }
    if (wid == 0) {
      a0 += t[0] * t[0];
      a0 += t[1] * t[1];
      a0 += t[2] * t[2];
      a0 += t[3] * t[3];
    }
  };
  double t[4], t2[4] = {0.0, 0.0, 0.0, 0.0};
  update(e, qa, qb, wa, wb, ba, bb, t);
  if (two) {
    __syncthreads();  // s_sum / s_x read by every wave before they are written again
#pragma unroll
    for (int m = 0; m < kCgsPerWave; ++m) {
      if (wid + 4 * m < nv) {
        qa[m] = ld2(Qw + m * step, e2);
        qb[m] = ld2(Qw + m * step, e2 + 128);
      }
    }
    double2 xa2 = make_double2(0.0, 0.0), xb2 = xa2;
    if (FX && wid == 1) {
      xa2 = ld2(x0, e2);
      xb2 = ld2(x0, e2 + 128);
    }
    update(e2, qa, qb, ld2(w, e2), ld2(w, e2 + 128), xa2, xb2, t2);
  }
  const double part = block_sum(a0, s_wave);
  if (threadIdx.x == 0) tag_put(slots + kOnePassN + 2 * blockIdx.x, tag, part);
  // 5. ||w'||^2 by the last workgroup, then q_{j+1} = w' / ||w'|| everywhere
  if (static_cast<int>(blockIdx.x) == grid - 1) {
    const double hn = tag_sum(slots + kOnePassN, grid, tag, s_wave, t0, err);
    if (threadIdx.x == 0) tag_put(slots + kOnePassH, tag, hn);
  }
  if (threadIdx.x == 0) {
    double hn;
    tag_get(slots + kOnePassH, tag, &hn, t0, err);
    s_h = sqrt(hn);
  }
  __syncthreads();
  const double h = s_h;
  if (blockIdx.x == 0 && threadIdx.x == 0) pin_store(h_out, h);
  if (wid == 0) {
    st2(qn, e, h == 0.0 ? 0.0 : t[0] / h, h == 0.0 ? 0.0 : t[1] / h);
    st2(qn, e + 128, h == 0.0 ? 0.0 : t[2] / h, h == 0.0 ? 0.0 : t[3] / h);
    if (two) {
      st2(qn, e2, h == 0.0 ? 0.0 : t2[0] / h, h == 0.0 ? 0.0 : t2[1] / h);
      st2(qn, e2 + 128, h == 0.0 ? 0.0 : t2[2] / h, h == 0.0 ? 0.0 : t2[3] / h);
    }
  }
}

// resident workgroups of the K2s variant (TWO: the two-chunk one), 0 if the query fails
static int icwy_onepass_grid_cap(bool two) {
  static int cap[2] = {-1, -1};
  int& c = cap[two ? 1 : 0];
  if (c < 0) {
    int dev = 0, cus = 0, per = 0, per_fx = 0;
    hipError_t e0 = hipGetDevice(&dev);
    if (e0 == hipSuccess) e0 = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e0 == hipSuccess)
      e0 = two ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, icwy_onepass_kernel<false, true>, kBlock, 0)
               : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, icwy_onepass_kernel<false, false>, kBlock, 0);
    if (e0 == hipSuccess)
      e0 = two ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_fx, icwy_onepass_kernel<true, true>, kBlock, 0)
               : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_fx, icwy_onepass_kernel<true, false>, kBlock, 0);
    if (e0 != hipSuccess) return 0;
    // every workgroup must be resident at once.  A kernel running beside it on another stream (the
    // side-stream GEMV) only delays the last workgroups' placement: it waits on nothing in here
    c = std::min<int>(kRedGrid, cus * std::min(per, per_fx));
  }
  return c;
}

int icwy_onepass_max_grid() { return icwy_onepass_grid_cap(false); }

int64_t icwy_onepass_max_n() {
  return std::max<int64_t>(static_cast<int64_t>(kCgsChunk) * icwy_onepass_grid_cap(false),
                           2 * static_cast<int64_t>(kCgsChunk) * icwy_onepass_grid_cap(true));
}

hipError_t launch_icwy_onepass(int64_t n, double* w, const double* Q, int64_t pitch, int nv, double* G, double* h_col,
                               unsigned long long* slots, unsigned tag, unsigned* err, hipStream_t s,
                               const LaunchEv* ev, int px, const double* yx, const double* x0, double* xo,
                               const double* rpart, int r_in, double* r_out, unsigned long long* flag,
                               const unsigned long long* seq) {
  const int64_t chunks = (n + kCgsChunk - 1) / kCgsChunk;
  // one chunk per workgroup while they all fit, else two per workgroup, the second streamed.
  // Halving the grid beats filling it (C4, N = 300,006: 586 workgroups 28.0-28.4 us per launch vs
  // 1,024 with only 148 chunks streamed 30.9-31.8 us, K2q 30.4-31.0; gpurun_out/r05k2s2, r05k2s3):
  // the spin hand-offs' cost grows with the workgroups that publish and poll
  const bool two = chunks > icwy_onepass_grid_cap(false);
  const int64_t grid = two ? (chunks + 1) / 2 : chunks;
  if (nv < 1 || nv > kCgsMax || n < 1 || grid > icwy_onepass_grid_cap(two) || tag == 0 || slots == nullptr ||
      err == nullptr || G == nullptr || h_col == nullptr || !aligned16d(w) || !aligned16d(Q) || pitch % 2 != 0 ||
      (rpart != nullptr && (r_in < 1 || r_out == nullptr)))
    return hipErrorInvalidValue;
  YArg ya;
  if (px > 0) {
    if (px > nv || px > kYArg || yx == nullptr || x0 == nullptr || xo == nullptr || !aligned16d(x0) || !aligned16d(xo))
      return hipErrorInvalidValue;
    for (int i = 0; i < px; ++i) ya.v[i] = yx[i];
  }
  const CoefArg ca{nullptr, G, h_col, rpart, r_in, r_out, flag, seq};
  double* qn = const_cast<double*>(Q) + static_cast<int64_t>(nv) * pitch;
#define SPIS_K2S(F, T)                                                                                          \
  launch_k(icwy_onepass_kernel<F, T>, dim3(grid), dim3(kBlock), 0, s, ev, n, w, Q, qn, pitch, nv, slots, tag, \
           err, ca, px, ya, x0, xo, h_col + nv)
  if (px > 0) {
    if (two) SPIS_K2S(true, true);
    else SPIS_K2S(true, false);
  } else {
    if (two) SPIS_K2S(false, true);
    else SPIS_K2S(false, false);
  }
#undef SPIS_K2S
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K4: x = Z[:, :p] y + x0 (solvers.py:287).  For p <= kYArg the coefficients travel in the
// kernel-argument segment (scalar loads, no H2D copy in front of the launch); otherwise they
// are copied to LDS from a device buffer.  Each lane streams one (VEC: two) element(s) of every
// basis vector; sum in basis order, then + x0 (numpy's ``Z @ yk + x0`` adds x0 afterwards).
// ---------------------------------------------------------------------------------------------
template <bool VEC, bool ARG, bool NT = false>
__global__ __launch_bounds__(kBlock) void gemv_kernel(int64_t n, int p,
                                                      const double* __restrict__ Z, int64_t pitch,
                                                      YArg yarg, const double* __restrict__ ycoef,
                                                      const double* __restrict__ x0,
                                                      double* __restrict__ x, int wt) {
#pragma clang fp contract(off)
  __shared__ double s_y[ARG ? 1 : kMaxK];
  if (!ARG) {
    for (int i = threadIdx.x; i < p; i += kBlock) s_y[i] = ycoef[i];
    __syncthreads();
  }
  const double* yc = ARG ? yarg.v : s_y;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  const int64_t tid = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (VEC) {
    const int64_t npair = n >> 1;
    for (int64_t q = tid; q < npair; q += stride) {
      double a0 = 0.0, a1 = 0.0;
      for (int i = 0; i < p; ++i) {
        const double2 z = ld_basis(reinterpret_cast<const double2*>(Z + i * pitch) + q, NT);
        const double c = yc[i];
        a0 += z.x * c;
        a1 += z.y * c;
      }
      const double2 b = reinterpret_cast<const double2*>(x0)[q];
      if (wt) {
        st_wt(x + 2 * q, a0 + b.x);
        st_wt(x + 2 * q + 1, a1 + b.y);
      } else {
        reinterpret_cast<double2*>(x)[q] = make_double2(a0 + b.x, a1 + b.y);
      }
    }
    if ((n & 1) && tid == 0) {
      const int64_t e = n - 1;
      double a = 0.0;
      for (int i = 0; i < p; ++i) a += Z[i * pitch + e] * yc[i];
      st_out(x + e, a + x0[e], wt);
    }
  } else {
    for (int64_t e = tid; e < n; e += stride) {
      double a = 0.0;
      for (int i = 0; i < p; ++i) a += Z[i * pitch + e] * yc[i];
      st_out(x + e, a + x0[e], wt);
    }
  }
}

hipError_t launch_gemv(int64_t n, int p, const double* Z, int64_t pitch, const double* y_host_or_dev,
                       bool y_on_host, const double* x0, double* x, hipStream_t s, const LaunchEv* ev, bool nt) {
  if (p > kMaxK || p < 1) return hipErrorInvalidValue;
  const bool vec = aligned16(Z) && (pitch % 2 == 0) && aligned16(x0) && aligned16(x);
  int64_t g = (n / (vec ? 2 : 1) + kBlock - 1) / kBlock;
  if (g > 4 * kRedGrid) g = 4 * kRedGrid;
  if (g < 1) g = 1;
  YArg ya;
  const bool arg = y_on_host && p <= kYArg;
  if (y_on_host && !arg) return hipErrorInvalidValue;  // caller stages larger y in HBM
  if (arg)
    for (int i = 0; i < p; ++i) ya.v[i] = y_host_or_dev[i];
  const double* yd = arg ? nullptr : y_host_or_dev;
  if (vec && arg && nt)
    launch_k(gemv_kernel<true, true, true>, dim3(g), dim3(kBlock), 0, s, ev, n, p, Z, pitch, ya, yd, x0, x, wt_other());
  else if (vec && arg)
    launch_k(gemv_kernel<true, true>, dim3(g), dim3(kBlock), 0, s, ev, n, p, Z, pitch, ya, yd, x0, x, wt_other());
  else if (vec)
    launch_k(gemv_kernel<true, false>, dim3(g), dim3(kBlock), 0, s, ev, n, p, Z, pitch, ya, yd, x0, x, wt_other());
  else if (arg)
    launch_k(gemv_kernel<false, true>, dim3(g), dim3(kBlock), 0, s, ev, n, p, Z, pitch, ya, yd, x0, x, wt_other());
  else
    launch_k(gemv_kernel<false, false>, dim3(g), dim3(kBlock), 0, s, ev, n, p, Z, pitch, ya, yd, x0, x, wt_other());
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K5: multi-vector SpMV W[:, c] = M Z[:, c], c < nvec (constraint operators, solvers.py:33):
// one launch for all basis vectors; the row block's values and columns are staged in LDS once
// and reused for every vector.  Same product/sum order as K1 (bit-identical to SciPy per
// column).  Long rows: workgroup reduction per vector.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void spmm_rowblock_kernel(
    const int32_t* __restrict__ rp, const int32_t* __restrict__ ci, const double* __restrict__ va,
    const int32_t* __restrict__ blk_row, int n_blk, const double* __restrict__ X, int64_t ldx,
    int nvec, double* __restrict__ Y, int64_t ldy) {
  __shared__ double s_val[kNnzCap];
  __shared__ int32_t s_col[kNnzCap];
  __shared__ double s_prod[kNnzCap];
  __shared__ double s_wave[4];
  for (int blk = blockIdx.x; blk < n_blk; blk += gridDim.x) {
    const int r0 = blk_row[blk];
    const int r1 = blk_row[blk + 1];
    const int nz0 = rp[r0];
    const int nnz = rp[r1] - nz0;
    if (nnz > kNnzCap) {
      for (int c = 0; c < nvec; ++c) {
        const double* xc = X + c * ldx;
        double acc = 0.0;
        for (int i = nz0 + threadIdx.x; i < nz0 + nnz; i += kBlock) acc += va[i] * xc[ci[i]];
        const double sum = block_sum(acc, s_wave);
        if (threadIdx.x == 0) Y[c * ldy + r0] = sum;
      }
      continue;
    }
    for (int i = threadIdx.x; i < nnz; i += kBlock) {
      s_val[i] = va[nz0 + i];
      s_col[i] = ci[nz0 + i];
    }
    __syncthreads();
    const int r = r0 + threadIdx.x;
    const int s0 = r < r1 ? rp[r] - nz0 : 0;
    const int e0 = r < r1 ? rp[r + 1] - nz0 : 0;
    for (int c = 0; c < nvec; ++c) {
      const double* xc = X + c * ldx;
#pragma unroll 4
      for (int i = threadIdx.x; i < nnz; i += kBlock) s_prod[i] = s_val[i] * xc[s_col[i]];
      __syncthreads();
      if (r < r1) {
        double sum = 0.0;
        for (int t = s0; t < e0; ++t) sum += s_prod[t];
        Y[c * ldy + r] = sum;
      }
      __syncthreads();
    }
  }
}

hipError_t launch_spmm(const CsrView& A, const double* X, int64_t ldx, int nvec, double* Y,
                       int64_t ldy, hipStream_t s) {
  if (nvec <= 0) return hipSuccess;
  int g = A.n_blk < kSpmvGrid ? A.n_blk : kSpmvGrid;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(spmm_rowblock_kernel, dim3(g), dim3(kBlock), 0, s, A.indptr, A.indices, A.vals,
                     A.blk_row, A.n_blk, X, ldx, nvec, Y, ldy);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// BLAS-1 helpers: partial dot, finalize, axpy, copy, gather (halo pack)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void dot_kernel(int64_t n, const double* __restrict__ x,
                                                     const double* __restrict__ y,
                                                     double* __restrict__ part_out) {
  __shared__ double s_wave[4];
  double part = 0.0;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; e < n; e += stride)
    part += x[e] * y[e];
  const double tot = block_sum(part, s_wave);
  if (threadIdx.x == 0) part_out[blockIdx.x] = tot;
}

hipError_t launch_dot(int64_t n, const double* x, const double* y, double* part_out, int grid,
                      hipStream_t s) {
  hipLaunchKernelGGL(dot_kernel, dim3(grid), dim3(kBlock), 0, s, n, x, y, part_out);
  return hipGetLastError();
}

__global__ __launch_bounds__(kBlock) void finalize_kernel(const double* __restrict__ part, int n_in,
                                                          double* __restrict__ out, int op,
                                                          unsigned long long* __restrict__ flag,
                                                          const unsigned long long* __restrict__ seq) {
  __shared__ double s_wave[4];
  const double t = sum_partials(part, n_in, s_wave);
  if (threadIdx.x == 0) publish(out, op == 1 ? sqrt(t) : t, flag, seq);
}

// two reductions in one launch (the paired residuals): workgroup i reduces part_i into out_i
__global__ __launch_bounds__(kBlock) void finalize2_kernel(const double* __restrict__ part1,
                                                           const double* __restrict__ part2, int n_in,
                                                           double* __restrict__ out1, double* __restrict__ out2,
                                                           unsigned long long* __restrict__ flag) {
  __shared__ double s_wave[4];
  const double t = sum_partials(blockIdx.x == 0 ? part1 : part2, n_in, s_wave);
  if (threadIdx.x == 0) publish(blockIdx.x == 0 ? out1 : out2, t, flag, nullptr);
}

hipError_t launch_finalize2(const double* part1, const double* part2, int n_in, double* out1, double* out2,
                            hipStream_t s, unsigned long long* flag) {
  hipLaunchKernelGGL(finalize2_kernel, dim3(2), dim3(kBlock), 0, s, part1, part2, n_in, out1, out2, flag);
  return hipGetLastError();
}

hipError_t launch_finalize(const double* part, int n_in, double* out, int op, hipStream_t s, const LaunchEv* ev,
                           unsigned long long* flag, const unsigned long long* seq) {
  launch_k(finalize_kernel, dim3(1), dim3(kBlock), 0, s, ev, part, n_in, out, op, flag, seq);
  return hipGetLastError();
}

__global__ __launch_bounds__(kBlock) void axpy_kernel(int64_t n, double h,
                                                      const double* __restrict__ x,
                                                      double* __restrict__ y) {
#pragma clang fp contract(off)
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; e < n; e += stride) {
    const double a = h * x[e];
    y[e] = y[e] - a;
  }
}

hipError_t launch_axpy(int64_t n, double h, const double* x, double* y, hipStream_t s) {
  int64_t g = (n + kBlock - 1) / kBlock;
  if (g > 4 * kRedGrid) g = 4 * kRedGrid;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(axpy_kernel, dim3(g), dim3(kBlock), 0, s, n, h, x, y);
  return hipGetLastError();
}

__global__ __launch_bounds__(kBlock) void copy_kernel(int64_t n, const double* __restrict__ x,
                                                      double* __restrict__ y) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; e < n; e += stride)
    y[e] = x[e];
}

hipError_t launch_copy(int64_t n, const double* x, double* y, hipStream_t s) {
  int64_t g = (n + kBlock - 1) / kBlock;
  if (g > 4 * kRedGrid) g = 4 * kRedGrid;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(copy_kernel, dim3(g), dim3(kBlock), 0, s, n, x, y);
  return hipGetLastError();
}

// y = x, and *flag = gen if any x[e] != 0 (a plain store from every lane that sees one: they all
// write the same value).  The solver's x0 copy: with flag != gen afterwards x0 is all zeros and the
// r0 SpMV skips the matrix (spmv_pipe_kernel MODE 3, zf)
__global__ __launch_bounds__(kBlock) void copy_flag_kernel(int64_t n, const double* __restrict__ x,
                                                           double* __restrict__ y, unsigned* flag, unsigned gen,
                                                           int wt) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  bool nz = false;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; e < n; e += stride) {
    const double v = x[e];
    st_out(y + e, v, wt);
    nz = nz || v != 0.0;
  }
  if (nz) *flag = gen;
}

hipError_t launch_copy_flag(int64_t n, const double* x, double* y, unsigned* flag, unsigned gen, hipStream_t s) {
  int64_t g = (n + kBlock - 1) / kBlock;
  if (g > 4 * kRedGrid) g = 4 * kRedGrid;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(copy_flag_kernel, dim3(g), dim3(kBlock), 0, s, n, x, y, flag, gen, wt_other());
  return hipGetLastError();
}

// cache eviction for cold-cache measurements (spis_spmv_bench): a streaming read of a buffer
// larger than the 256 MB Infinity Cache, summed into one sink word so it is not dead code
__global__ __launch_bounds__(kBlock) void stream_read_kernel(int64_t n2, const double2* __restrict__ x,
                                                             double* __restrict__ sink) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  double acc = 0.0;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; e < n2; e += stride) {
    const double2 v = x[e];
    acc += v.x + v.y;
  }
  if (acc == 1.2345678e300) sink[0] = acc;  // never true for the zero-filled buffer
}

hipError_t launch_stream_read(int64_t n, const double* x, double* sink, hipStream_t s) {
  hipLaunchKernelGGL(stream_read_kernel, dim3(4096), dim3(kBlock), 0, s, n >> 1, reinterpret_cast<const double2*>(x),
                     sink);
  return hipGetLastError();
}

__global__ __launch_bounds__(kBlock) void gather_kernel(int64_t m, const int32_t* __restrict__ idx,
                                                        const double* __restrict__ x,
                                                        double* __restrict__ send) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; e < m; e += stride)
    send[e] = x[idx[e]];
}

// rows idx[i] of a row-major (., cols) array -> row i of send (the Ut halo of a constraint
// reduction on several GPUs): one thread per double
__global__ __launch_bounds__(kBlock) void gather_rows_kernel(int64_t m, int cols, const int32_t* __restrict__ idx,
                                                             const double* __restrict__ src,
                                                             double* __restrict__ send) {
  const int64_t total = m * cols;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; e < total; e += stride) {
    const int64_t r = e / cols;
    const int c = static_cast<int>(e - r * cols);
    send[e] = src[static_cast<int64_t>(idx[r]) * cols + c];
  }
}

hipError_t launch_gather_rows(int64_t m, int cols, const int32_t* idx, const double* src, double* send,
                              hipStream_t s) {
  if (m <= 0) return hipSuccess;
  int64_t g = (m * cols + kBlock - 1) / kBlock;
  if (g > 4 * kRedGrid) g = 4 * kRedGrid;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(g), dim3(kBlock), 0, s, m, cols, idx, src, send);
  return hipGetLastError();
}

hipError_t launch_gather(int64_t m, const int32_t* idx, const double* x, double* send,
                         hipStream_t s) {
  if (m <= 0) return hipSuccess;
  int64_t g = (m + kBlock - 1) / kBlock;
  if (g > 4 * kRedGrid) g = 4 * kRedGrid;
  hipLaunchKernelGGL(gather_kernel, dim3(g), dim3(kBlock), 0, s, m, idx, x, send);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K6: tall-skinny Gram G = U^T V (constraint terms, solvers.py:33-36; K = N is huge, nu, nv <=
// kGramMaxVec).  Each workgroup stages kGramChunk elements of the nu + nv vectors in LDS (rows
// padded to a multiple of 4 with zeros, leading dim kGramChunk + 1).  Thread t owns a 4 x 4
// register tile of G (tile = t % ntiles) and the elements e = t / ntiles (mod ksplit) of every
// chunk, so each 8 LDS reads feed 16 FMAs.  At the end the ksplit partial tiles are summed in
// a fixed order through LDS and the workgroup's partial G is written; gram_reduce_kernel sums
// the workgroup partials in workgroup order (4 waves x strided subsets, fixed combine):
// deterministic, independent of placement.
// ---------------------------------------------------------------------------------------------
constexpr int kGramLd = kGramChunk + 1;
constexpr int kTile = 4;

__global__ __launch_bounds__(kBlock) void gram_partial_kernel(int64_t n, int nu,
                                                              const double* const* __restrict__ U,
                                                              int nv,
                                                              const double* const* __restrict__ V,
                                                              double* __restrict__ partials) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int nup = (nu + kTile - 1) / kTile * kTile;
  const int nvp = (nv + kTile - 1) / kTile * kTile;
  double* sU = smem;
  double* sV = smem + nup * kGramLd;
  const int ta = nup / kTile, tb = nvp / kTile, ntiles = ta * tb;
  const int ksplit = kBlock / ntiles;  // >= 1 since ntiles <= 256
  const int t = threadIdx.x;
  const int tile = t % ntiles;
  const int ks = t / ntiles;
  const bool active = ks < ksplit;
  const int a0 = (tile / tb) * kTile, b0 = (tile % tb) * kTile;
  double acc[kTile][kTile];
#pragma unroll
  for (int i = 0; i < kTile; ++i)
#pragma unroll
    for (int j = 0; j < kTile; ++j) acc[i][j] = 0.0;
  const int nload = (nup + nvp) * kGramChunk;
  for (int64_t c0 = static_cast<int64_t>(blockIdx.x) * kGramChunk; c0 < n;
       c0 += static_cast<int64_t>(gridDim.x) * kGramChunk) {
    for (int idx = t; idx < nload; idx += kBlock) {
      const int vec = idx / kGramChunk;
      const int e = idx - vec * kGramChunk;
      const int64_t g = c0 + e;
      if (vec < nup)
        sU[vec * kGramLd + e] = (vec < nu && g < n) ? U[vec][g] : 0.0;
      else
        sV[(vec - nup) * kGramLd + e] = (vec - nup < nv && g < n) ? V[vec - nup][g] : 0.0;
    }
    __syncthreads();
    if (active) {
      for (int e = ks; e < kGramChunk; e += ksplit) {
        double u[kTile], v[kTile];
#pragma unroll
        for (int i = 0; i < kTile; ++i) u[i] = sU[(a0 + i) * kGramLd + e];
#pragma unroll
        for (int j = 0; j < kTile; ++j) v[j] = sV[(b0 + j) * kGramLd + e];
#pragma unroll
        for (int i = 0; i < kTile; ++i)
#pragma unroll
          for (int j = 0; j < kTile; ++j) acc[i][j] += u[i] * v[j];
      }
    }
    __syncthreads();
  }
  // fixed-order reduction of the ksplit partial tiles: slot [ks][tile][16]
  double* red = smem;
  if (active)
#pragma unroll
    for (int i = 0; i < kTile; ++i)
#pragma unroll
      for (int j = 0; j < kTile; ++j) red[(ks * ntiles + tile) * 16 + i * kTile + j] = acc[i][j];
  __syncthreads();
  const int npairs = nu * nv;
  for (int pr = t; pr < npairs; pr += kBlock) {
    const int a = pr / nv, b = pr - (pr / nv) * nv;
    const int tl = (a / kTile) * tb + (b / kTile);
    const int slot = (a % kTile) * kTile + (b % kTile);
    double sum = 0.0;
    for (int k = 0; k < ksplit; ++k) sum += red[(k * ntiles + tl) * 16 + slot];
    partials[static_cast<int64_t>(blockIdx.x) * npairs + pr] = sum;
  }
}

// out[j] = sum over rows of part[row][j] (row-major rows x npairs), one workgroup per output:
// strided per-thread sums then block_sum's fixed tree (deterministic); optional symmetrize:
// out[a np1 + b] += (the same sum of part[.][b np1 + a]) for the np1 x np1 prefix (K7t's H + H^T)
// (pin: out is host memory a host thread polls, system-scope stores, each value its own flag)
__global__ __launch_bounds__(kBlock) void reduce_cols_kernel(int npairs, int rows, const double* __restrict__ part,
                                                             double* __restrict__ out, int sym_np1, bool pin) {
  __shared__ double s_wave[4];
  const int j = blockIdx.x;
  double s = 0.0;
  for (int r = threadIdx.x; r < rows; r += kBlock) s += part[static_cast<int64_t>(r) * npairs + j];
  double tot = block_sum(s, s_wave);
  if (sym_np1 > 0 && j < sym_np1 * sym_np1) {
    const int a = j / sym_np1, b = j - (j / sym_np1) * sym_np1;
    const int jt = b * sym_np1 + a;
    double st = 0.0;
    for (int r = threadIdx.x; r < rows; r += kBlock) st += part[static_cast<int64_t>(r) * npairs + jt];
    tot = tot + block_sum(st, s_wave);
  }
  if (threadIdx.x == 0) {
    if (pin)
      pin_store(out + j, tot);
    else
      out[j] = tot;
  }
}

// K7t's H + H^T for the np1 x np1 block: one workgroup per pair a <= b (np1 (np1 + 1) / 2 of them,
// about half of reduce_cols_kernel's np1^2).  Both sums are reduce_cols_kernel's (same strided
// per-thread sums, same block_sum tree), and out[a][b] = s_ab + s_ba, out[b][a] = s_ba + s_ab are
// the same double (addition commutes), so every value is bitwise reduce_cols_kernel's.
// Blocks past the pairs (lin.npairs of them) reduce lin's columns as reduce_cols_kernel does (the
// transpose's linear terms: one launch fewer on the constrained step).
__global__ __launch_bounds__(kBlock) void reduce_sym_kernel(int np1, int rows, const double* __restrict__ part,
                                                            double* __restrict__ out, bool pin, ColReduce lin) {
  __shared__ double s_wave[4];
  const int np2 = np1 * np1;
  const int nsym = np1 * (np1 + 1) / 2;
  if (static_cast<int>(blockIdx.x) >= nsym) {
    const int j = static_cast<int>(blockIdx.x) - nsym;
    double s = 0.0;
    for (int r = threadIdx.x; r < lin.rows; r += kBlock) s += lin.part[static_cast<int64_t>(r) * lin.npairs + j];
    const double tot = block_sum(s, s_wave);
    if (threadIdx.x == 0) {
      if (pin)
        pin_store(lin.out + j, tot);
      else
        lin.out[j] = tot;
    }
    return;
  }
  int a = 0, t = static_cast<int>(blockIdx.x);
  while (t >= np1 - a) {  // row a of the upper triangle holds np1 - a pairs
    t -= np1 - a;
    ++a;
  }
  const int b = a + t;
  const int j = a * np1 + b, jt = b * np1 + a;
  double s = 0.0, st = 0.0;
  for (int r = threadIdx.x; r < rows; r += kBlock) s += part[static_cast<int64_t>(r) * np2 + j];
  const double s_ab = block_sum(s, s_wave);
  for (int r = threadIdx.x; r < rows; r += kBlock) st += part[static_cast<int64_t>(r) * np2 + jt];
  const double s_ba = block_sum(st, s_wave);
  if (threadIdx.x == 0) {
    const double tot = s_ab + s_ba;
    if (pin) {
      pin_store(out + j, tot);
      if (jt != j) pin_store(out + jt, tot);
    } else {
      out[j] = tot;
      out[jt] = tot;
    }
  }
}

__global__ __launch_bounds__(kBlock) void gram_reduce_kernel(int npairs, int grid,
                                                             const double* __restrict__ partials,
                                                             double* __restrict__ G) {
  __shared__ double s_acc[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int pr = blockIdx.x * 64 + lane;
  double s = 0.0;
  if (pr < npairs) {
#pragma unroll 8
    for (int b = w; b < grid; b += 4) s += partials[static_cast<int64_t>(b) * npairs + pr];
  }
  s_acc[w][lane] = s;
  __syncthreads();
  if (w == 0 && pr < npairs) G[pr] = ((s_acc[0][lane] + s_acc[1][lane]) + s_acc[2][lane]) + s_acc[3][lane];
}

size_t gram_lds_bytes(int nu, int nv) {
  const int nup = (nu + kTile - 1) / kTile * kTile;
  const int nvp = (nv + kTile - 1) / kTile * kTile;
  const size_t tiles = static_cast<size_t>(nup + nvp) * kGramLd * sizeof(double);
  const size_t red = static_cast<size_t>(kBlock) * 16 * sizeof(double);
  return tiles > red ? tiles : red;
}

hipError_t launch_gram(int64_t n, int nu, const double* const* U, int nv, const double* const* V,
                       double* partials, int grid, double* G, hipStream_t s) {
  if (nu > kGramMaxVec || nv > kGramMaxVec || nu < 1 || nv < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gram_partial_kernel, dim3(grid), dim3(kBlock), gram_lds_bytes(nu, nv), s, n, nu, U,
                     nv, V, partials);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int npairs = nu * nv;
  hipLaunchKernelGGL(gram_reduce_kernel, dim3((npairs + 63) / 64), dim3(kBlock), 0, s, npairs, grid,
                     partials, G);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K7: fused constraint reduction (solvers.py:33-36 for all constraints of a step at once).
//   U = [z_0 .. z_{p-1}, x0]           (np1 = p + 1 columns)
//   transpose_basis_kernel:  Ut (N x np1, row-major) = U^T, via LDS tiles of 64 rows
//   constraint_gram_kernel:  16-row chunks; XCD group g = blockIdx % 8 owns a contiguous eighth
//     of the rows and deals its chunks round-robin to its waves (compact L2 window).  Per chunk
//     the wave streams the contiguous nonzeros with 16 independent 8*np1-byte Ut-row gathers in
//     flight (lane a < np1 forms w_a = (M U)_{r,a}), stores each row's w to an LDS tile, then
//       G[a][b] += sum_i Ut[r0+i][a] * W[i][b]     (W rows read by LDS broadcast)
//       Gv[c][a] += Ut[r][a] * v_c[r]             (up to 4 linear terms v_c)
//     and each block writes one partial (its 4 waves combined in wave order); gram_reduce_kernel
//     sums the block partials in block order (deterministic).  G = U^T M U gives term2 = G[:p,:p]/2, x0'MZ = G[p,:p],
//     x0'Mx0 = G[p,p]; Gv gives v'Z and v.x0.
// ---------------------------------------------------------------------------------------------
// Ut row stride: 32 doubles (256 B, 16-B aligned rows) for np1 <= 32, else 64; zero padded
__host__ __device__ __forceinline__ int ut_ld(int np1) { return np1 <= 32 ? 32 : 64; }

// perm (ld 32 only, K7m / K7t): row position 2i holds column i and position 2i + 1 column
// i + 16, so that one 16-B load of lane i gives the two MFMA tiles' column i.
// nvv > 0 (K7t): the linear terms Gv[c][a] = sum_r U[r][a] v_c[r] ride along (the tile is in
// LDS anyway): thread c * np1 + a sums its tiles' rows in order, one partial per block in
// vpart[block][c * np1 + a] (grid-stride over the 64-row tiles, so a fixed grid).
__global__ __launch_bounds__(kBlock) void transpose_basis_kernel(int64_t n, int p,
                                                                 const double* __restrict__ Z,
                                                                 int64_t pitch,
                                                                 const double* __restrict__ x0,
                                                                 double* __restrict__ Ut, bool perm, int nvv,
                                                                 const double* __restrict__ v0,
                                                                 const double* __restrict__ v1,
                                                                 const double* __restrict__ v2,
                                                                 const double* __restrict__ v3,
                                                                 double* __restrict__ vpart) {
  extern __shared__ __attribute__((aligned(16))) double tile[];  // np1 x 65, then 4 x 64 (v)
  const int np1 = p + 1;
  double* s_v = tile + np1 * 65;
  const double* vv[4] = {v0, v1, v2, v3};
  const int ld = ut_ld(np1);
  const int nl = nvv * np1;
  const int tc = threadIdx.x / np1, ta = threadIdx.x - tc * np1;  // this thread's linear term
  double lin = 0.0;
  const int64_t ntiles = (n + 63) / 64;
  for (int64_t tb = blockIdx.x; tb < ntiles; tb += gridDim.x) {
    const int64_t r0 = tb * 64;
    const int rows = static_cast<int>(n - r0 < 64 ? n - r0 : 64);
    for (int idx = threadIdx.x; idx < np1 * 64; idx += kBlock) {
      const int a = idx >> 6, r = idx & 63;
      if (r < rows) tile[a * 65 + r] = a < p ? Z[a * pitch + r0 + r] : x0[r0 + r];
    }
    if (nvv > 0) {
      const int c = threadIdx.x >> 6, r = threadIdx.x & 63;
      if (c < nvv) s_v[c * 64 + r] = r < rows ? vv[c][r0 + r] : 0.0;
    }
    __syncthreads();
    double* out = Ut + r0 * ld;
    for (int idx = threadIdx.x; idx < rows * ld; idx += kBlock) {
      const int r = idx / ld, pos = idx - (idx / ld) * ld;
      const int a = perm ? (pos >> 1) + ((pos & 1) << 4) : pos;
      out[idx] = a < np1 ? tile[a * 65 + r] : 0.0;
    }
    if (threadIdx.x < nl)
      for (int r = 0; r < rows; ++r) lin += tile[ta * 65 + r] * s_v[tc * 64 + r];
    __syncthreads();
  }
  if (vpart != nullptr && threadIdx.x < nl) vpart[static_cast<int64_t>(blockIdx.x) * nl + threadIdx.x] = lin;
}

// K7t's transpose (perm order, np1 <= 32, Ut rows of 32 doubles): the same tiles, rows and linear
// terms as transpose_basis_kernel (bitwise: Ut is a copy, every linear partial sums its tiles' rows
// in the same order), software-pipelined: the next tile's 16-B loads are issued before this tile's
// rows are stored (16-B stores), so each block keeps one tile in flight while it writes the previous
// one (the one-tile-at-a-time form ran 94 us at C3, 504 MB).
__global__ __launch_bounds__(kBlock) void transpose_basis_pipe_kernel(int64_t n, int p, const double* __restrict__ Z,
                                                                      int64_t pitch, const double* __restrict__ x0,
                                                                      double* __restrict__ Ut, int nvv,
                                                                      const double* __restrict__ v0,
                                                                      const double* __restrict__ v1,
                                                                      const double* __restrict__ v2,
                                                                      const double* __restrict__ v3,
                                                                      double* __restrict__ vpart, int wt) {
  __shared__ double tile[32 * 65];
  __shared__ double s_v[4 * 64];
  const int np1 = p + 1;
  const double* vc = (threadIdx.x >> 6) == 0 ? v0 : (threadIdx.x >> 6) == 1 ? v1 : (threadIdx.x >> 6) == 2 ? v2 : v3;  // this wave's v (nvv > 0)
  const int nl = nvv * np1;
  const int tc = threadIdx.x / np1, ta = threadIdx.x - tc * np1;
  double lin = 0.0;
  const int64_t ntiles = (n + 63) / 64;
  // loader slot q of this thread: vector a = wave + 4 q (wave-uniform), row = lane
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  double nx[8];
  double nvx = 0.0;
  auto load = [&](int64_t tb) {
    const int64_t g = tb * 64 + ln;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int a = wv + 4 * q;
      const double* src = a < p ? Z + a * pitch : x0;
      nx[q] = (a < np1 && g < n) ? src[g] : 0.0;
    }
    if (nvv > 0) {
      const int c = threadIdx.x >> 6, r = threadIdx.x & 63;
      nvx = (c < nvv && tb * 64 + r < n) ? vc[tb * 64 + r] : 0.0;
    }
  };
  int64_t tb = blockIdx.x;
  if (tb < ntiles) load(tb);
  for (; tb < ntiles; tb += gridDim.x) {
    const int64_t r0 = tb * 64;
    const int rows = static_cast<int>(n - r0 < 64 ? n - r0 : 64);
#pragma unroll
    for (int q = 0; q < 8; ++q) tile[(wv + 4 * q) * 65 + ln] = nx[q];
    if (nvv > 0) s_v[threadIdx.x] = nvx;  // (c < 4: all 256 slots; unused ones never read)
    __syncthreads();
    if (tb + gridDim.x < ntiles) load(tb + gridDim.x);
    double* out = Ut + r0 * 32;
    const __amdgpu_buffer_rsrc_t orr = span_rsrc(out);  // (the tile base: wave-uniform)
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // row r, positions (2 m, 2 m + 1) = columns (m, m + 16)
      const int idx = threadIdx.x + kBlock * q;
      const int r = idx >> 4, m = idx & 15;
      if (r < rows) {
        const double lo = m < np1 ? tile[m * 65 + r] : 0.0;
        const double hi = m + 16 < np1 ? tile[(m + 16) * 65 + r] : 0.0;
        if (wt)
          buf_st2_wt(orr, (r * 32 + 2 * m) * 8, make_double2(lo, hi));
        else
          buf_st2(orr, (r * 32 + 2 * m) * 8, 0, make_double2(lo, hi));
      }
    }
    if (threadIdx.x < nl)
      for (int r = 0; r < rows; ++r) lin += tile[ta * 65 + r] * s_v[tc * 64 + r];
    __syncthreads();
  }
  if (vpart != nullptr && threadIdx.x < nl) vpart[static_cast<int64_t>(blockIdx.x) * nl + threadIdx.x] = lin;
}

__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const unsigned long long bits = __double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readlane(static_cast<unsigned>(bits), lane);
  const unsigned hi = __builtin_amdgcn_readlane(static_cast<unsigned>(bits >> 32), lane);
  return __longlong_as_double((static_cast<unsigned long long>(hi) << 32) | lo);
}

constexpr int kConRows = 16;   // rows per chunk of the fused constraint Gram
constexpr int kConBatch = 16;  // gather instructions in flight per wave (x P nonzeros each)
constexpr int kConWin = 256;   // nonzeros staged in LDS per window

// NP = column slots (32 or 64); P = 64 / NP nonzeros gathered per wave instruction (lane half h
// takes nonzero t = P*q + h of a batch); each lane keeps SEG = NP / P entries of its G row.
template <int NP>
__global__ __launch_bounds__(kBlock, NP <= 32 ? 3 : 2) void constraint_gram_kernel(
    int64_t n, int np1, const int32_t* __restrict__ rp, const int32_t* __restrict__ ci,
    const double* __restrict__ va, const double* __restrict__ Ut, int nvv,
    const double* __restrict__ v0, const double* __restrict__ v1, const double* __restrict__ v2,
    const double* __restrict__ v3, double* __restrict__ partials) {
  constexpr int P = 64 / NP;
  constexpr int SEG = NP / P;
  constexpr int NW = kBlock / 64;
  __shared__ __attribute__((aligned(16))) double s_w[NW][kConRows][NP];  // per-wave W tile
  __shared__ double s_val[NW][kConWin];
  __shared__ int s_col[NW][kConWin];
  __shared__ double s_acc[64 * (SEG + 4)];  // fixed-order wave combine: [lane][SEG G | 4 Gv]
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int la = lane % NP;  // column a of U this lane gathers / owns
  const int h = lane / NP;   // nonzero slot within a gather instruction
  const bool on = la < np1;
  const int lac = on ? la : 0;
  // XCD group = blockIdx % 8 (dispatch order; speed only, never correctness): each group owns a
  // contiguous eighth of the rows, its waves take 16-row chunks round-robin, so the group's
  // active window of Ut rows (and their banded column neighbourhood) stays in its own L2
  const int ngrp = (gridDim.x & 7) == 0 ? 8 : 1;
  const int grp = blockIdx.x % ngrp;
  const int64_t wpg = static_cast<int64_t>(gridDim.x / ngrp) * NW;  // waves per group
  const int64_t gw = static_cast<int64_t>(blockIdx.x / ngrp) * NW + wid;
  const int64_t rpg = ((n + ngrp - 1) / ngrp + kConRows - 1) / kConRows * kConRows;  // whole slices
  const int64_t g0 = grp * rpg;
  const int64_t g1 = g0 + rpg < n ? g0 + rpg : n;
  const int64_t nch = g1 > g0 ? (g1 - g0 + kConRows - 1) / kConRows : 0;
  const bool has_m = rp != nullptr;
  double acc[SEG];
#pragma unroll
  for (int j = 0; j < SEG; ++j) acc[j] = 0.0;
  double gv[4] = {0.0, 0.0, 0.0, 0.0};
  double (*W)[NP] = s_w[wid];
  double* sv = s_val[wid];
  int* sc = s_col[wid];
  auto chunk_rows = [&](int64_t ch) { return static_cast<int>(g1 - (g0 + ch * kConRows) < kConRows ? g1 - (g0 + ch * kConRows) : kConRows); };
  // row pointers of the wave's first chunk; later chunks' are prefetched one chunk ahead
  int rpl_next = 0;
  if (has_m && gw < nch) {
    const int nr = chunk_rows(gw);
    rpl_next = rp[g0 + gw * kConRows + (lane <= nr ? lane : nr)];
  }
  for (int64_t ch = gw; ch < nch; ch += wpg) {
    const int64_t r0 = g0 + ch * kConRows;
    const int nr = chunk_rows(ch);
    const int rpl = rpl_next;
    if (has_m && ch + wpg < nch) {  // next chunk's row pointers (issued before anything else)
      const int nr2 = chunk_rows(ch + wpg);
      rpl_next = rp[r0 + wpg * kConRows + (lane <= nr2 ? lane : nr2)];
    }
    const int nz0 = has_m ? __builtin_amdgcn_readlane(rpl, 0) : 0;
    const int nz1 = has_m ? __builtin_amdgcn_readlane(rpl, nr) : 0;
    // the first window's (col, val) loads go out first (vmcnt retires in order), clamped and
    // unconditional so the compiler keeps them in flight together
    constexpr int kStage = kConWin / 64;
    int cst[kStage];
    double vst[kStage];
    auto stage = [&](int wb, int wl) {
#pragma unroll
      for (int q = 0; q < kStage; ++q) {
        const int e = q * 64 + lane;
        const int idx = wb + (e < wl ? e : 0);
        cst[q] = ci[idx];
        vst[q] = va[idx];
      }
    };
    auto commit = [&]() {
#pragma unroll
      for (int q = 0; q < kStage; ++q) {
        sc[q * 64 + lane] = cst[q];
        sv[q * 64 + lane] = vst[q];
      }
      __builtin_amdgcn_wave_barrier();
    };
    if (nz1 > nz0) stage(nz0, nz1 - nz0 < kConWin ? nz1 - nz0 : kConWin);
    // rows of U for the update (unconditional, clamped: in flight during the gathers)
    double u[kConRows];
#pragma unroll
    for (int i = 0; i < kConRows; ++i) u[i] = Ut[(r0 + (i < nr ? i : 0)) * ut_ld(np1) + lac];
    double vc[4] = {0.0, 0.0, 0.0, 0.0};
    if (lane < nr) {
      if (nvv > 0) vc[0] = v0[r0 + lane];
      if (nvv > 1) vc[1] = v1[r0 + lane];
      if (nvv > 2) vc[2] = v2[r0 + lane];
      if (nvv > 3) vc[3] = v3[r0 + lane];
    }
    if (has_m) {
      // phase 1: w_a = sum_c M_rc Ut[c][a] per row over the chunk's contiguous nonzeros;
      // each row's w goes to the wave's LDS tile at the row end (empty rows store 0)
      int row = 0;
      int row_end = __builtin_amdgcn_readlane(rpl, 1);
      double w = 0.0;
      auto flush = [&]() {
        double wt = w;
        if (P == 2) wt += __shfl_xor(w, 32);
        if (h == 0) W[row][la] = wt;
        w = 0.0;
        ++row;
        row_end = __builtin_amdgcn_readlane(rpl, row + 1 <= kConRows ? row + 1 : kConRows);
      };
      if (nz1 > nz0) commit();  // first window: straight-line, waits for its own loads only
      for (int wb = nz0; wb < nz1; wb += kConWin) {
        const int wl = nz1 - wb < kConWin ? nz1 - wb : kConWin;
        if (wb != nz0) {  // chunks longer than one window (rare)
          stage(wb, wl);
          commit();
        }
        for (int tb = 0; tb < wl; tb += kConBatch * P) {
          double g[kConBatch];
#pragma unroll
          for (int q = 0; q < kConBatch; ++q) {
            const int t = tb + P * q + h;
            const int col = sc[t < wl ? t : 0];
            g[q] = Ut[static_cast<int64_t>(col) * ut_ld(np1) + lac];  // valid address for every lane
          }
#pragma unroll
          for (int q = 0; q < kConBatch; ++q) {
            const int tA = tb + P * q;  // wave-uniform position of slot 0
            if (tA >= wl) break;
            while (wb + tA >= row_end) flush();
            const double gq = on ? g[q] : 0.0;
            if (h == 0) w += sv[tA] * gq;
            if (P == 2 && tA + 1 < wl) {
              while (wb + tA + 1 >= row_end) flush();
              if (h == 1) w += sv[tA + 1] * gq;
            }
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
      while (row < kConRows) flush();  // last row with nonzeros, then empty / absent rows
      __builtin_amdgcn_wave_barrier();
      // phase 2: rank-16 update G[a][b] += sum_i Ut[r0+i][a] * W[i][b], b in this lane's
      // segment [SEG*h, SEG*h + SEG) (LDS broadcast reads)
#pragma unroll
      for (int i = 0; i < kConRows; ++i) {
        const double ui = (on && i < nr) ? u[i] : 0.0;
        const double2* wr = reinterpret_cast<const double2*>(&W[i][SEG * h]);
#pragma unroll
        for (int j = 0; j < SEG; j += 2) {
          const double2 x2 = wr[j >> 1];
          acc[j] += ui * x2.x;
          acc[j + 1] += ui * x2.y;
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
    if (h == 0) {
#pragma unroll
      for (int i = 0; i < kConRows; ++i) {  // Gv[c][a] += Ut[r][a] * v_c[r]
        const double ui = (on && i < nr) ? u[i] : 0.0;
        if (nvv > 0) gv[0] += ui * readlane_f64(vc[0], i);
        if (nvv > 1) gv[1] += ui * readlane_f64(vc[1], i);
        if (nvv > 2) gv[2] += ui * readlane_f64(vc[2], i);
        if (nvv > 3) gv[3] += ui * readlane_f64(vc[3], i);
      }
    }
  }
  // combine the block's waves in wave order through LDS (deterministic), one partial per block
  for (int w = 0; w < NW; ++w) {
    if (wid == w) {
#pragma unroll
      for (int j = 0; j < SEG; ++j) s_acc[lane * (SEG + 4) + j] = (w == 0 ? 0.0 : s_acc[lane * (SEG + 4) + j]) + acc[j];
#pragma unroll
      for (int c = 0; c < 4; ++c)
        s_acc[lane * (SEG + 4) + SEG + c] = (w == 0 ? 0.0 : s_acc[lane * (SEG + 4) + SEG + c]) + gv[c];
    }
    __syncthreads();
  }
  // partial layout per block: [np1 x np1 G | nvv x np1 Gv]; G[a][b] lives in lane a + NP*(b/SEG)
  const int64_t stride = static_cast<int64_t>(np1) * np1 + static_cast<int64_t>(nvv) * np1;
  double* out = partials + static_cast<int64_t>(blockIdx.x) * stride;
  for (int idx = threadIdx.x; idx < stride; idx += kBlock) {
    if (idx < np1 * np1) {
      const int a = idx / np1, b = idx - (idx / np1) * np1;
      out[idx] = has_m ? s_acc[(a + NP * (b / SEG)) * (SEG + 4) + (b % SEG)] : 0.0;
    } else {
      const int k2 = idx - np1 * np1;
      const int c = k2 / np1, a = k2 - (k2 / np1) * np1;
      out[idx] = s_acc[a * (SEG + 4) + SEG + c];
    }
  }
}

hipError_t launch_transpose_basis(int64_t n, int p, const double* Z, int64_t pitch, const double* x0,
                                  double* Ut, hipStream_t s, bool perm) {
  const int np1 = p + 1;
  if (np1 > 64 || (perm && np1 > 32)) return hipErrorInvalidValue;
  const int64_t g = (n + 63) / 64;
  hipLaunchKernelGGL(transpose_basis_kernel, dim3(static_cast<unsigned>(g)), dim3(kBlock),
                     static_cast<size_t>(np1) * 65 * sizeof(double) + 4 * 64 * sizeof(double), s, n, p, Z, pitch,
                     x0, Ut, perm, 0, nullptr, nullptr, nullptr, nullptr, nullptr);
  return hipGetLastError();
}

hipError_t launch_transpose_basis_lin(int64_t n, int p, const double* Z, int64_t pitch, const double* x0,
                                      double* Ut, int nvv, const double* const* v, double* vpart, double* Gv,
                                      hipStream_t s, bool pin, bool pipe, ColReduce* defer) {
  const int np1 = p + 1;
  if (np1 > 32 || nvv < 0 || nvv > 4 || nvv * np1 > kBlock) return hipErrorInvalidValue;
  if (defer != nullptr) *defer = ColReduce{0, 0, nullptr, nullptr};
  const double* vv[4] = {nullptr, nullptr, nullptr, nullptr};
  for (int c = 0; c < nvv; ++c) vv[c] = v[c];
  const int64_t ntiles = (n + 63) / 64;
  const int g = static_cast<int>(ntiles < kTransposeGrid ? (ntiles < 1 ? 1 : ntiles) : kTransposeGrid);
  if (pipe && aligned16d(Ut))
    hipLaunchKernelGGL(transpose_basis_pipe_kernel, dim3(static_cast<unsigned>(g)), dim3(kBlock), 0, s, n, p, Z, pitch,
                       x0, Ut, nvv, vv[0], vv[1], vv[2], vv[3], nvv > 0 ? vpart : nullptr, wt_other());
  else
    hipLaunchKernelGGL(transpose_basis_kernel, dim3(static_cast<unsigned>(g)), dim3(kBlock),
                       static_cast<size_t>(np1) * 65 * sizeof(double) + 4 * 64 * sizeof(double), s, n, p, Z, pitch,
                       x0, Ut, true, nvv, vv[0], vv[1], vv[2], vv[3], nvv > 0 ? vpart : nullptr);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || nvv == 0) return e;
  const int npairs = nvv * np1;
  if (defer != nullptr) {
    *defer = ColReduce{npairs, g, vpart, Gv};
    return hipSuccess;
  }
  hipLaunchKernelGGL(reduce_cols_kernel, dim3(npairs), dim3(kBlock), 0, s, npairs, g, vpart, Gv, 0, pin);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K7m: constraint Gram on the f64 matrix cores (p + 1 <= 32; Ut in the transpose's perm order).
//   G = U^T (M U) = sum over 4-row groups of U[rows]^T W[rows],  W = M U,
// one v_mfma_f64_16x16x4_f64 per (16-column tile of U) x (16-column tile of W) and group: the K
// index of the MFMA is the row within the group.  Lane (g, i) = (lane >> 4, lane & 15) owns row g
// of the group and columns i, i + 16: exactly the MFMA's A / B operand lanes (A[i][k = g], B[k =
// g][i]), so neither U nor W ever moves between lanes.
//   W[r] = sum_t M[r, c_t] U[c_t] (t ascending, the row's CSR order): the 16 lanes of row g each
// gather their 16 B of the 256-B Ut row of c_t (one wave instruction = 4 nonzeros' whole rows,
// twice the bytes per instruction of K7's 8-B gathers), up to 16 nonzeros of a row in flight; the
// (col, val) entries come in with one coalesced load per group and are broadcast by bpermute.
// Pipeline per wave: group q+2's row bounds and group q+1's entries, own U row and linear-term
// values are loaded while group q gathers.  Rows longer than 16 take further passes (direct
// loads).  Schedule: XCD group (blockIdx % 8) owns an eighth of the rows, its waves take the
// 4-row groups round-robin (compact L2 window); speed only, never correctness.  Fixed-order wave
// combine and block partials as in K7 (gram_reduce_kernel sums them in block order).
// Linear terms Gv[c][a] = sum_r U[r][a] v_c[r] from the same pass (VALU).
// ---------------------------------------------------------------------------------------------
typedef double v4d_t __attribute__((ext_vector_type(4)));

// host: 8 row ranges of weight(row) = nnz + kGramRowW each.  A wave pays about one memory
// round trip per 4-row group whatever its rows' lengths (the group's gathers are all in flight
// at once), so rows, not nonzeros, set the time: measured at C3 (swe energy matrix, rows of 14,
// 8 and 1 entries) 237 us with equal rows per XCD group vs 329 us with equal nonzeros + 2 rows
constexpr double kGramRowW = 1e9;
void gram_split(int64_t n, const int32_t* indptr, GramSplit* out) {
  const double total = static_cast<double>(indptr[n]) + kGramRowW * static_cast<double>(n);
  int64_t r = 0;
  out->row[0] = 0;
  for (int x = 1; x < 8; ++x) {
    const double want = total * x / 8.0;
    while (r < n && static_cast<double>(indptr[r]) + kGramRowW * static_cast<double>(r) < want) ++r;
    out->row[x] = static_cast<int32_t>(r);
  }
  out->row[8] = static_cast<int32_t>(n);
}

__global__ __launch_bounds__(kBlock, 2) void constraint_gram_mfma_kernel(
    int64_t n, int np1, GramSplit split, const int32_t* __restrict__ rp,
    const int32_t* __restrict__ ci, const double* __restrict__ va, const double* __restrict__ Ut, int nvv,
    const double* __restrict__ v0,
    const double* __restrict__ v1, const double* __restrict__ v2, const double* __restrict__ v3,
    double* __restrict__ partials) {
  constexpr int NW = kBlock / 64;
  constexpr int NA = 24;  // combine slots per lane: 16 G (4 tiles x 4 regs) + 2 x 4 Gv
  __shared__ double s_acc[64 * NA];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4;
  const int li = lane & 15;
  const double2* __restrict__ U2 = reinterpret_cast<const double2*>(Ut);  // 16 double2 per row
  const int ngrp = (gridDim.x & 7) == 0 ? 8 : 1;
  const int grp = blockIdx.x % ngrp;
  const int64_t wpg = static_cast<int64_t>(gridDim.x / ngrp) * NW;
  const int64_t gw = static_cast<int64_t>(blockIdx.x / ngrp) * NW + wid;
  // XCD group grp's rows: the split balances nonzeros + rows (swe: edge rows 14 entries, rho 1)
  const int64_t rb = ngrp == 8 ? split.row[grp] : 0;
  const int64_t re_ = ngrp == 8 ? split.row[grp + 1] : n;
  const int64_t ngroups = re_ > rb ? (re_ - rb + 3) / 4 : 0;
  const bool has_m = rp != nullptr;
  v4d_t acc00 = {0.0, 0.0, 0.0, 0.0}, acc01 = acc00, acc10 = acc00, acc11 = acc00;
  double gv0[4] = {0.0, 0.0, 0.0, 0.0}, gv1[4] = {0.0, 0.0, 0.0, 0.0};
  const double* vv[4] = {v0, v1, v2, v3};

  // stage A (group q + 2): this lane's row bounds
  auto load_a = [&](int64_t q, int& s, int& e, int& ro) {
    const int64_t r = rb + 4 * q + g;
    s = e = 0;
    ro = static_cast<int>(r);
    if (has_m && q < ngroups && r < re_) {
      s = rp[r];
      e = rp[r + 1];
    }
  };
  // stage B (group q + 1): the row's first 16 entries, its own U row and its v_c values
  struct StB {
    int s, e, col;
    double val;
    double2 u;
    double vc[4];
  };
  auto load_b = [&](int64_t q, int s, int e, int ro, StB& B) {
    const int64_t r = ro;
    const bool ok = q < ngroups && rb + 4 * q + g < re_;
    B.s = s;
    B.e = e;
    B.col = 0;
    B.val = 0.0;
    if (li < e - s) {
      B.col = ci[s + li];
      B.val = va[s + li];
    }
    B.u = ok ? U2[r * 16 + li] : make_double2(0.0, 0.0);
#pragma unroll
    for (int c = 0; c < 4; ++c) B.vc[c] = (ok && c < nvv) ? vv[c][r] : 0.0;
  };

  int64_t q = gw;
  int sa = 0, ea = 0, oa = 0, sa2 = 0, ea2 = 0, oa2 = 0;
  StB cur;
  load_a(q, sa, ea, oa);
  load_a(q + wpg, sa2, ea2, oa2);
  if (q < ngroups) load_b(q, sa, ea, oa, cur);
  for (; q < ngroups; q += wpg) {
    StB nxt;
    nxt.s = nxt.e = 0;
    int sa3 = 0, ea3 = 0, oa3 = 0;
    double w0 = 0.0, w1 = 0.0;
    const int len = cur.e - cur.s;
    const int l0 = __builtin_amdgcn_readlane(len, 0), l1 = __builtin_amdgcn_readlane(len, 16);
    const int l2 = __builtin_amdgcn_readlane(len, 32), l3 = __builtin_amdgcn_readlane(len, 48);
    const int maxlen = max(max(l0, l1), max(l2, l3));
    int mcol = cur.col;
    double mval = cur.val;
    // pass b0 over entries [b0, b0 + 16) of each row; the first pass's gathers go out before the
    // next groups' loads, so waiting for them never waits for those (vmcnt retires in order)
    for (int b0 = 0; b0 == 0 || b0 < maxlen; b0 += 16) {
      if (b0 > 0) {  // rows longer than 16 entries: the next 16, loaded directly
        mcol = 0;
        mval = 0.0;
        if (b0 + li < len) {
          mcol = ci[cur.s + b0 + li];
          mval = va[cur.s + b0 + li];
        }
      }
      double2 gt[16];
      const int nt = maxlen - b0;  // wave-uniform: gathers past every row's end are not issued
      if (has_m && maxlen > 0) {
#pragma unroll
        for (int t = 0; t < 16; ++t) {  // col 0 (a valid row) past a row's end
          const int c = __shfl(mcol, (g << 4) + t, 64);
          gt[t] = t < nt ? U2[static_cast<int64_t>(c) * 16 + li] : make_double2(0.0, 0.0);
        }
      }
      if (b0 == 0) {  // the next groups' loads: in flight through this group's gathers and MFMAs
        if (q + wpg < ngroups) load_b(q + wpg, sa2, ea2, oa2, nxt);
        load_a(q + 2 * wpg, sa3, ea3, oa3);
      }
      if (has_m && maxlen > 0) {
#pragma unroll
        for (int t = 0; t < 16; ++t) {
          if (t < nt) {
            const double v = __shfl(mval, (g << 4) + t, 64);
            if (b0 + t < len) {
              w0 += v * gt[t].x;
              w1 += v * gt[t].y;
            }
          }
        }
      }
    }
    if (has_m) {
      acc00 = __builtin_amdgcn_mfma_f64_16x16x4f64(cur.u.x, w0, acc00, 0, 0, 0);
      acc01 = __builtin_amdgcn_mfma_f64_16x16x4f64(cur.u.x, w1, acc01, 0, 0, 0);
      acc10 = __builtin_amdgcn_mfma_f64_16x16x4f64(cur.u.y, w0, acc10, 0, 0, 0);
      acc11 = __builtin_amdgcn_mfma_f64_16x16x4f64(cur.u.y, w1, acc11, 0, 0, 0);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (c < nvv) {
        gv0[c] += cur.u.x * cur.vc[c];
        gv1[c] += cur.u.y * cur.vc[c];
      }
    cur = nxt;
    sa2 = sa3;
    ea2 = ea3;
    oa2 = oa3;
  }
  // combine the block's waves in wave order (deterministic), one partial per block
  for (int w = 0; w < NW; ++w) {
    if (wid == w) {
      double v[NA];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = acc00[i];
        v[4 + i] = acc01[i];
        v[8 + i] = acc10[i];
        v[12 + i] = acc11[i];
        v[16 + i] = gv0[i];
        v[20 + i] = gv1[i];
      }
#pragma unroll
      for (int j = 0; j < NA; ++j) s_acc[lane * NA + j] = (w == 0 ? 0.0 : s_acc[lane * NA + j]) + v[j];
    }
    __syncthreads();
  }
  // G[16 ta + i][16 tb + j] = tile (ta, tb) register i >> 2 of lane ((i & 3) << 4) | j
  const int64_t stride = static_cast<int64_t>(np1) * np1 + static_cast<int64_t>(nvv) * np1;
  double* out = partials + static_cast<int64_t>(blockIdx.x) * stride;
  for (int idx = threadIdx.x; idx < stride; idx += kBlock) {
    if (idx < np1 * np1) {
      const int a = idx / np1, b = idx - (idx / np1) * np1;
      const int ta = a >> 4, ia = a & 15, tb = b >> 4, ib = b & 15;
      const int ln = ((ia & 3) << 4) | ib;
      out[idx] = has_m ? s_acc[ln * NA + (2 * ta + tb) * 4 + (ia >> 2)] : 0.0;
    } else {
      const int k2 = idx - np1 * np1;
      const int c = k2 / np1, a = k2 - (k2 / np1) * np1;
      const int slot = (a < 16 ? 16 : 20) + c;
      const int ln = a & 15;
      // the four row groups' sums in group order
      out[idx] = ((s_acc[ln * NA + slot] + s_acc[(16 + ln) * NA + slot]) + s_acc[(32 + ln) * NA + slot]) +
                 s_acc[(48 + ln) * NA + slot];
    }
  }
}

hipError_t launch_constraint_gram_mfma(int64_t n, int np1, const CsrView* M, const GramSplit* split,
                                       const double* Ut, int nvv, const double* const* v, double* partials,
                                       double* G, hipStream_t s) {
  if (np1 > 32 || nvv > 4 || (M == nullptr && nvv == 0)) return hipErrorInvalidValue;
  const double* vv[4] = {nullptr, nullptr, nullptr, nullptr};
  for (int c = 0; c < nvv; ++c) vv[c] = v[c];
  static const int grid = [] {  // resident workgroups, a multiple of 8, <= the partial slots
    int dev = 0, cus = 256, per = 1;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, constraint_gram_mfma_kernel, kBlock, 0) != hipSuccess ||
        per < 1)
      per = 1;
    int t = (cus * per) & ~7;
    return t < 8 ? 8 : (t > kConGramGrid ? kConGramGrid : t);
  }();
  GramSplit sp;
  if (M != nullptr && split != nullptr) {
    sp = *split;
  } else {  // rows only (no matrix): equal row ranges
    for (int x = 0; x <= 8; ++x) sp.row[x] = static_cast<int32_t>(n * x / 8);
  }
  hipLaunchKernelGGL(constraint_gram_mfma_kernel, dim3(grid), dim3(kBlock), 0, s, n, np1, sp,
                     M ? M->indptr : nullptr, M ? M->indices : nullptr, M ? M->vals : nullptr, Ut, nvv, vv[0],
                     vv[1], vv[2], vv[3], partials);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int npairs = np1 * np1 + nvv * np1;
  hipLaunchKernelGGL(reduce_cols_kernel, dim3(npairs), dim3(kBlock), 0, s, npairs, grid, partials, G, 0, false);
  return hipGetLastError();
}

int constraint_gram_partials() { return kConGramGrid; }

hipError_t launch_constraint_gram(int64_t n, int np1, const CsrView* M, const double* Ut, int nvv,
                                  const double* const* v, double* partials, double* G, hipStream_t s) {
  if (np1 > 64 || nvv > 4 || (M == nullptr && nvv == 0)) return hipErrorInvalidValue;
  const int32_t* rp = M ? M->indptr : nullptr;
  const int32_t* ci = M ? M->indices : nullptr;
  const double* va = M ? M->vals : nullptr;
  const double* vv[4] = {nullptr, nullptr, nullptr, nullptr};
  for (int c = 0; c < nvv; ++c) vv[c] = v[c];
  // one resident wave-set (256 CUs x blocks per CU at the kernel's occupancy): every group's
  // waves sweep their row range together; a multiple of 8 and <= constraint_gram_partials()
  const int grid = np1 <= 32 ? 256 * 3 : 256 * 2;
  if (np1 <= 32)
    hipLaunchKernelGGL(constraint_gram_kernel<32>, dim3(grid), dim3(kBlock), 0, s, n, np1, rp, ci, va, Ut,
                       nvv, vv[0], vv[1], vv[2], vv[3], partials);
  else
    hipLaunchKernelGGL(constraint_gram_kernel<64>, dim3(grid), dim3(kBlock), 0, s, n, np1, rp, ci, va, Ut,
                       nvv, vv[0], vv[1], vv[2], vv[3], partials);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int npairs = np1 * np1 + nvv * np1;
  hipLaunchKernelGGL(gram_reduce_kernel, dim3((npairs + 63) / 64), dim3(kBlock), 0, s, npairs, grid,
                     partials, G);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K7t: constraint Gram of a SYMMETRIC constraint matrix on the f64 matrix cores, from a slot
// table (p + 1 <= 32; Ut in the perm order; linear terms come from the transpose).
//   G = H + H^T,   H = sum_r U_r What_r^T,   What_r = (1/2) M_rr U_r + sum_{c > r} M_rc U_c
// (M = M^T: each off-diagonal pair is gathered once, the diagonal is the row's own U row), so a
// row gathers about half of its nonzeros.  Rows go in 4-row groups (the MFMA's K = 4, lane
// layout as K7m); a group's slots are its rows' own U rows (slot 0, value M_rr / 2) then their
// upper entries, padded to the longest row; groups longer than NS slots are cut into segments,
// each with its own own-row slot (H is linear in What).  Consecutive segments are packed into
// blocks of <= NS slots (a host-built table: per block NS x 4 (col, val) entries and a mask of
// segment starts), so short rows (swe: interior dofs ~2 slots, rho 1) share one round trip.
// Per block: one coalesced table load (prefetched a block ahead), <= NS 16-B gathers in flight
// per lane, then per segment What accumulated in slot order and 4 MFMAs.  Blocks: XCD group
// (blockIdx % 8) owns a contiguous eighth, its waves take them round-robin.
// ---------------------------------------------------------------------------------------------
template <int NS>
__global__ __launch_bounds__(kBlock, 2) void constraint_gram_sym_kernel(SymTabView T,
                                                                        const double* __restrict__ Ut,
                                                                        double* __restrict__ partials, int np1) {
  constexpr int NW = kBlock / 64;
  constexpr int NJ = NS / 16;  // table entries per lane and block
  constexpr int NA = 16;
  __shared__ double s_acc[64 * NA];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4;
  const int li = lane & 15;
  const double2* __restrict__ U2 = reinterpret_cast<const double2*>(Ut);
  // waves take the blocks round-robin over the whole table: blocks differ widely in cost (an
  // edge-row block of swe holds one segment, a rho-row block sixteen, with 4 MFMAs each), and
  // giving each XCD a contiguous eighth (K7m's schedule) measured 251 vs 141 us at C3; an
  // XCD-local schedule of table chunks measured 131-222 vs 122 us (profiles/r02e_k7t_chunk_sweep.txt)
  const int64_t wpg = static_cast<int64_t>(gridDim.x) * NW;
  const int64_t gw = static_cast<int64_t>(blockIdx.x) * NW + wid;
  const int64_t kb1 = T.nblk;
  v4d_t acc00 = {0.0, 0.0, 0.0, 0.0}, acc01 = acc00, acc10 = acc00, acc11 = acc00;
  struct Ent {  // zero-initialised: a block past the range is never loaded, never undefined
    unsigned long long mask = 0;
    int col[NJ] = {};
    double val[NJ] = {};
  };
  auto load = [&](int64_t kb, Ent& E) {
    E.mask = T.mask[kb];
    const int64_t base = kb * (4 * NS) + g * NS + li;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      E.col[j] = T.col[base + 16 * j];
      E.val[j] = T.val[base + 16 * j];
    }
  };
  auto flush = [&](const double2& a, double w0, double w1) {
    acc00 = __builtin_amdgcn_mfma_f64_16x16x4f64(a.x, w0, acc00, 0, 0, 0);
    acc01 = __builtin_amdgcn_mfma_f64_16x16x4f64(a.x, w1, acc01, 0, 0, 0);
    acc10 = __builtin_amdgcn_mfma_f64_16x16x4f64(a.y, w0, acc10, 0, 0, 0);
    acc11 = __builtin_amdgcn_mfma_f64_16x16x4f64(a.y, w1, acc11, 0, 0, 0);
  };
  int64_t L = gw;
  Ent cur, nxt;  // the table two blocks ahead is in flight: its wait never stalls a block
  if (L < kb1) load(L, cur);
  if (L + wpg < kb1) load(L + wpg, nxt);
  for (; L < kb1; L += wpg) {
    // readfirstlane returns int: widen through unsigned, or a start bit at slot 31 (32-slot
    // blocks) sign-extends into the slot count (ns = -1: the whole block skipped; the round-2
    // 32-slot failure, tools/k7t_probe.py)
    const unsigned long long mk =
        static_cast<unsigned long long>(static_cast<unsigned>(__builtin_amdgcn_readfirstlane(
            static_cast<unsigned>(cur.mask)))) |
        (static_cast<unsigned long long>(static_cast<unsigned>(__builtin_amdgcn_readfirstlane(
             static_cast<unsigned>(cur.mask >> 32))))
         << 32);
    const int ns = static_cast<int>(mk >> 32);
    const unsigned starts = static_cast<unsigned>(mk);
    // gathers in straight-line quads (a wave-uniform test per 4 slots): the bpermutes of a quad
    // go out together, then its loads; slots past ns hold (row 0, value 0) in the table
    double2 gt[NS];
    // the block's column indices in groups of GB bpermutes (one LDS wait per group), then the
    // gathers of the group's quads that hold slots.  32 slots: groups of 8 (166 -> 143 us at C3);
    // 16 slots: quads (groups of 8 measured 127 vs 124 us)
    constexpr int GB = NS >= 32 ? 8 : 4;
#pragma unroll
    for (int tg = 0; tg < NS; tg += GB) {
      if (tg < ns) {
        int c[GB];
#pragma unroll
        for (int u = 0; u < GB; ++u)
          c[u] = __shfl(cur.col[(tg + u) >> 4], (g << 4) + ((tg + u) & 15), 64);
#pragma unroll
        for (int q = 0; q < GB; q += 4) {
          if (q == 0 || tg + q < ns) {
#pragma unroll
            for (int u = q; u < q + 4; ++u) gt[tg + u] = U2[static_cast<int64_t>(c[u]) * 16 + li];
          }
        }
      }
    }
    Ent nx2;
    if (L + 2 * wpg < kb1) load(L + 2 * wpg, nx2);  // in flight through this block and the next
    double2 a = make_double2(0.0, 0.0);
    double w0 = 0.0, w1 = 0.0;
#pragma unroll
    for (int t4 = 0; t4 < NS; t4 += 4) {
      if (t4 < ns) {
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = __shfl(cur.val[(t4 + u) >> 4], (g << 4) + ((t4 + u) & 15), 64);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int t = t4 + u;
          if ((starts >> t) & 1u) {
            if (t > 0) flush(a, w0, w1);
            a = gt[t];
            w0 = 0.0;
            w1 = 0.0;
          }
          w0 += v[u] * gt[t].x;
          w1 += v[u] * gt[t].y;
        }
      }
    }
    if (ns > 0) flush(a, w0, w1);
    cur = nxt;
    nxt = nx2;
  }
  for (int w = 0; w < NW; ++w) {
    if (wid == w) {
      double v[NA];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = acc00[i];
        v[4 + i] = acc01[i];
        v[8 + i] = acc10[i];
        v[12 + i] = acc11[i];
      }
#pragma unroll
      for (int j = 0; j < NA; ++j) s_acc[lane * NA + j] = (w == 0 ? 0.0 : s_acc[lane * NA + j]) + v[j];
    }
    __syncthreads();
  }
  const int np2 = np1 * np1;
  double* out = partials + static_cast<int64_t>(blockIdx.x) * np2;
  for (int idx = threadIdx.x; idx < np2; idx += kBlock) {
    const int a = idx / np1, b = idx - (idx / np1) * np1;
    const int ta = a >> 4, ia = a & 15, tb = b >> 4, ib = b & 15;
    const int ln = ((ia & 3) << 4) | ib;
    out[idx] = s_acc[ln * NA + (2 * ta + tb) * 4 + (ia >> 2)];
  }
}

static int sym_grid() {
  static const int grid = [] {
    int dev = 0, cus = 256, per = 1;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, constraint_gram_sym_kernel<kSymSlots>, kBlock, 0) !=
            hipSuccess ||
        per < 1)
      per = 1;
    int t = (cus * per) & ~7;
    return t < 8 ? 8 : (t > kConGramGrid ? kConGramGrid : t);
  }();
  return grid;
}

hipError_t launch_constraint_gram_sym(int np1, const SymTabView& T, const double* Ut, double* partials, double* G,
                                      hipStream_t s, bool pin, const ColReduce* lin) {
  if (np1 > 32) return hipErrorInvalidValue;
  if (T.ns != kSymSlots) return hipErrorInvalidValue;
  const int grid = sym_grid();
  hipLaunchKernelGGL(constraint_gram_sym_kernel<kSymSlots>, dim3(grid), dim3(kBlock), 0, s, T, Ut, partials, np1);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const ColReduce lr = lin != nullptr ? *lin : ColReduce{0, 0, nullptr, nullptr};
  hipLaunchKernelGGL(reduce_sym_kernel, dim3(np1 * (np1 + 1) / 2 + lr.npairs), dim3(kBlock), 0, s, np1, grid, partials,
                     G, pin, lr);
  return hipGetLastError();
}

}  // namespace spis
