// kernels.hip — gfx950 (MI355X, CDNA4) kernels of the CGMRES/FGMRES inner loop.
//
// Everything here is HBM-bandwidth bound fp64 work (SpMV ~0.17 flop/B, BLAS-1
// <= 0.125 flop/B), so no MFMA: the design levers are coalesced 8/16-B-per-lane
// streams, LDS staging of the irregular SpMV products, enough waves in flight
// (256-thread workgroups, grid-stride), and deterministic reductions whose
// partials never leave the device.
//
// Reference call sites (solvers.py): SpMV :191 / :167 / :290, MGS :193-195,
// norm + normalise :196-198, GEMV :287, constraint Gram :33-36.
#include <hip/hip_runtime.h>

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

// every workgroup reduces the same partial array in the same order -> the same scalar
__device__ __forceinline__ double sum_partials(const double* __restrict__ part, int n, double* s_wave) {
  double v = 0.0;
  for (int i = threadIdx.x; i < n; i += kBlock) v += part[i];
  return block_sum(v, s_wave);
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
template <int EPI>
__global__ __launch_bounds__(kBlock) void spmv_rowblock_kernel(
    const int32_t* __restrict__ rp, const int32_t* __restrict__ ci, const double* __restrict__ va,
    const int32_t* __restrict__ blk_row, int n_blk, const double* __restrict__ x,
    double* __restrict__ y, const double* __restrict__ aux, double* __restrict__ partials) {
  __shared__ double s_prod[kNnzCap];
  __shared__ double s_wave[4];
  double part = 0.0;
  for (int blk = blockIdx.x; blk < n_blk; blk += gridDim.x) {
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
    const double* __restrict__ vb = va + nz0;
    const int32_t* __restrict__ cb = ci + nz0;
#pragma unroll 4
    for (int i = threadIdx.x; i < nnz; i += kBlock) s_prod[i] = vb[i] * x[cb[i]];
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

int spmv_grid(const CsrView& A, bool fixed) {
  if (fixed) return kSpmvGrid;
  int g = A.n_blk < kSpmvGrid ? A.n_blk : kSpmvGrid;
  return g < 1 ? 1 : g;
}

int blas_grid(int64_t n, bool fixed) {
  if (fixed) return kRedGrid;
  int64_t g = (n + 2 * kBlock * 2 - 1) / (2 * kBlock * 2);  // >= 2 pairs per thread
  if (g > kRedGrid) g = kRedGrid;
  return g < 1 ? 1 : static_cast<int>(g);
}

hipError_t launch_spmv(const CsrView& A, int epi, const double* x, double* y, const double* aux,
                       double* partials, int grid, hipStream_t s) {
  dim3 g(grid), b(kBlock);
  switch (epi) {
    case kEpiPlain:
      hipLaunchKernelGGL(spmv_rowblock_kernel<kEpiPlain>, g, b, 0, s, A.indptr, A.indices, A.vals,
                         A.blk_row, A.n_blk, x, y, aux, partials);
      break;
    case kEpiDot:
      hipLaunchKernelGGL(spmv_rowblock_kernel<kEpiDot>, g, b, 0, s, A.indptr, A.indices, A.vals,
                         A.blk_row, A.n_blk, x, y, aux, partials);
      break;
    case kEpiResNorm:
      hipLaunchKernelGGL(spmv_rowblock_kernel<kEpiResNorm>, g, b, 0, s, A.indptr, A.indices,
                         A.vals, A.blk_row, A.n_blk, x, y, aux, partials);
      break;
    default:
      hipLaunchKernelGGL(spmv_rowblock_kernel<kEpiR0>, g, b, 0, s, A.indptr, A.indices, A.vals,
                         A.blk_row, A.n_blk, x, y, aux, partials);
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
                                                          double* __restrict__ h_out) {
#pragma clang fp contract(off)
  __shared__ double s_wave[4];
  const double h = sum_partials(part_in, n_in, s_wave);
  if (blockIdx.x == 0 && threadIdx.x == 0) *h_out = h;
  double part = 0.0;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  const int64_t tid = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (VEC) {
    const int64_t npair = n >> 1;
    double2* y2 = reinterpret_cast<double2*>(y);
    const double2* q2 = reinterpret_cast<const double2*>(qi);
    const double2* n2 = reinterpret_cast<const double2*>(qn);
    for (int64_t p = tid; p < npair; p += stride) {
      const double2 qv = q2[p];
      double2 yv = y2[p];
      const double a0 = h * qv.x, a1 = h * qv.y;
      yv.x = yv.x - a0;
      yv.y = yv.y - a1;
      y2[p] = yv;
      if (qn) {
        const double2 nv = n2[p];
        part += nv.x * yv.x;
        part += nv.y * yv.y;
      } else {
        part += yv.x * yv.x;
        part += yv.y * yv.y;
      }
    }
    if ((n & 1) && tid == 0) {
      const int64_t e = n - 1;
      const double a = h * qi[e];
      const double yv = y[e] - a;
      y[e] = yv;
      part += qn ? qn[e] * yv : yv * yv;
    }
  } else {
    for (int64_t e = tid; e < n; e += stride) {
      const double a = h * qi[e];
      const double yv = y[e] - a;
      y[e] = yv;
      part += qn ? qn[e] * yv : yv * yv;
    }
  }
  const double tot = block_sum(part, s_wave);
  if (threadIdx.x == 0) part_out[blockIdx.x] = tot;
}

static inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

hipError_t launch_mgs_step(int64_t n, double* y, const double* qi, const double* qnext,
                           const double* part_in, int n_in, double* part_out, double* h_out,
                           int grid, hipStream_t s) {
  const bool vec = aligned16(y) && aligned16(qi) && (qnext == nullptr || aligned16(qnext));
  if (vec)
    hipLaunchKernelGGL(mgs_step_kernel<true>, dim3(grid), dim3(kBlock), 0, s, n, y, qi, qnext,
                       part_in, n_in, part_out, h_out);
  else
    hipLaunchKernelGGL(mgs_step_kernel<false>, dim3(grid), dim3(kBlock), 0, s, n, y, qi, qnext,
                       part_in, n_in, part_out, h_out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K3: h_{j+1,j} = ||y|| = sqrt(y.y) (numpy's norm), q_{j+1} = y / h (true division, :198).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void normalize_kernel(int64_t n, const double* __restrict__ y,
                                                           double* __restrict__ qn,
                                                           const double* __restrict__ part_in,
                                                           int n_in, double* __restrict__ h_out) {
  __shared__ double s_wave[4];
  const double h = sqrt(sum_partials(part_in, n_in, s_wave));
  if (blockIdx.x == 0 && threadIdx.x == 0) *h_out = h;
  // breakdown (h == 0): cgmres/gmres stop (solvers.py:199-202); cgmres_p carries on with the
  // q[j+1] row it never wrote, i.e. zeros (solvers.py:172,376-377) — reproduce that here
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; e < n; e += stride)
    qn[e] = h == 0.0 ? 0.0 : y[e] / h;
}

hipError_t launch_normalize(int64_t n, const double* y, double* qnext, const double* part_in,
                            int n_in, double* h_out, hipStream_t s, int grid) {
  hipLaunchKernelGGL(normalize_kernel, dim3(grid), dim3(kBlock), 0, s, n, y, qnext, part_in, n_in,
                     h_out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K4: x = Z[:, :p] y + x0 (solvers.py:287).  y is copied to LDS once per workgroup; each lane
// streams one (VEC: two) element(s) of every basis vector.  Sum in basis order, then + x0.
// ---------------------------------------------------------------------------------------------
template <bool VEC>
__global__ __launch_bounds__(kBlock) void gemv_kernel(int64_t n, int p,
                                                      const double* __restrict__ Z, int64_t pitch,
                                                      const double* __restrict__ ycoef,
                                                      const double* __restrict__ x0,
                                                      double* __restrict__ x) {
#pragma clang fp contract(off)
  __shared__ double s_y[kMaxK];
  for (int i = threadIdx.x; i < p; i += kBlock) s_y[i] = ycoef[i];
  __syncthreads();
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  const int64_t tid = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (VEC) {
    const int64_t npair = n >> 1;
    for (int64_t q = tid; q < npair; q += stride) {
      double a0 = 0.0, a1 = 0.0;
      for (int i = 0; i < p; ++i) {
        const double2 z = reinterpret_cast<const double2*>(Z + i * pitch)[q];
        a0 += z.x * s_y[i];
        a1 += z.y * s_y[i];
      }
      const double2 b = reinterpret_cast<const double2*>(x0)[q];
      reinterpret_cast<double2*>(x)[q] = make_double2(a0 + b.x, a1 + b.y);
    }
    if ((n & 1) && tid == 0) {
      const int64_t e = n - 1;
      double a = 0.0;
      for (int i = 0; i < p; ++i) a += Z[i * pitch + e] * s_y[i];
      x[e] = a + x0[e];
    }
  } else {
    for (int64_t e = tid; e < n; e += stride) {
      double a = 0.0;
      for (int i = 0; i < p; ++i) a += Z[i * pitch + e] * s_y[i];
      x[e] = a + x0[e];
    }
  }
}

hipError_t launch_gemv(int64_t n, int p, const double* Z, int64_t pitch, const double* y,
                       const double* x0, double* x, hipStream_t s) {
  if (p > kMaxK) return hipErrorInvalidValue;
  const bool vec = aligned16(Z) && (pitch % 2 == 0) && aligned16(x0) && aligned16(x);
  int64_t g = (n / (vec ? 2 : 1) + kBlock - 1) / kBlock;
  if (g > 4 * kRedGrid) g = 4 * kRedGrid;
  if (g < 1) g = 1;
  if (vec)
    hipLaunchKernelGGL(gemv_kernel<true>, dim3(g), dim3(kBlock), 0, s, n, p, Z, pitch, y, x0, x);
  else
    hipLaunchKernelGGL(gemv_kernel<false>, dim3(g), dim3(kBlock), 0, s, n, p, Z, pitch, y, x0, x);
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
                                                          double* __restrict__ out, int op) {
  __shared__ double s_wave[4];
  const double t = sum_partials(part, n_in, s_wave);
  if (threadIdx.x == 0) out[0] = op == 1 ? sqrt(t) : t;
}

hipError_t launch_finalize(const double* part, int n_in, double* out, int op, hipStream_t s) {
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(kBlock), 0, s, part, n_in, out, op);
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

__global__ __launch_bounds__(kBlock) void gather_kernel(int64_t m, const int32_t* __restrict__ idx,
                                                        const double* __restrict__ x,
                                                        double* __restrict__ send) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; e < m; e += stride)
    send[e] = x[idx[e]];
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
// K6: tall-skinny Gram G = U^T V (constraint terms, solvers.py:33-36).  Each workgroup stages
// kGramChunk elements of all nu + nv vectors in LDS (rows padded by one to spread banks), every
// thread owns up to kPairsPerThread (a, b) pairs in registers across its chunks; per-workgroup
// partials are then summed in workgroup order by gram_reduce_kernel (deterministic).
// ---------------------------------------------------------------------------------------------
constexpr int kPairsPerThread = (kGramMaxVec * kGramMaxVec + kBlock - 1) / kBlock;
constexpr int kGramLd = kGramChunk + 1;

__global__ __launch_bounds__(kBlock) void gram_partial_kernel(int64_t n, int nu,
                                                              const double* const* __restrict__ U,
                                                              int nv,
                                                              const double* const* __restrict__ V,
                                                              double* __restrict__ partials) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* sU = smem;
  double* sV = smem + nu * kGramLd;
  const int npairs = nu * nv;
  double acc[kPairsPerThread];
#pragma unroll
  for (int t = 0; t < kPairsPerThread; ++t) acc[t] = 0.0;
  const int nload = (nu + nv) * kGramChunk;
  for (int64_t c0 = static_cast<int64_t>(blockIdx.x) * kGramChunk; c0 < n;
       c0 += static_cast<int64_t>(gridDim.x) * kGramChunk) {
    for (int idx = threadIdx.x; idx < nload; idx += kBlock) {
      const int vec = idx / kGramChunk;
      const int e = idx - vec * kGramChunk;
      const int64_t g = c0 + e;
      if (vec < nu)
        sU[vec * kGramLd + e] = g < n ? U[vec][g] : 0.0;
      else
        sV[(vec - nu) * kGramLd + e] = g < n ? V[vec - nu][g] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < kPairsPerThread; ++t) {
      const int pr = threadIdx.x + t * kBlock;
      if (pr < npairs) {
        const int a = pr / nv;
        const int b = pr - a * nv;
        const double* ua = sU + a * kGramLd;
        const double* vb = sV + b * kGramLd;
        double s = 0.0;
        for (int e = 0; e < kGramChunk; ++e) s += ua[e] * vb[e];
        acc[t] += s;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int t = 0; t < kPairsPerThread; ++t) {
    const int pr = threadIdx.x + t * kBlock;
    if (pr < npairs) partials[static_cast<int64_t>(blockIdx.x) * npairs + pr] = acc[t];
  }
}

__global__ __launch_bounds__(kBlock) void gram_reduce_kernel(int npairs, int grid,
                                                             const double* __restrict__ partials,
                                                             double* __restrict__ G) {
  const int pr = blockIdx.x * kBlock + threadIdx.x;
  if (pr >= npairs) return;
  double s = 0.0;
  for (int b = 0; b < grid; ++b) s += partials[static_cast<int64_t>(b) * npairs + pr];
  G[pr] = s;
}

hipError_t launch_gram(int64_t n, int nu, const double* const* U, int nv, const double* const* V,
                       double* partials, int grid, double* G, hipStream_t s) {
  if (nu > kGramMaxVec || nv > kGramMaxVec || nu < 1 || nv < 1) return hipErrorInvalidValue;
  const size_t lds = static_cast<size_t>(nu + nv) * kGramLd * sizeof(double);
  hipLaunchKernelGGL(gram_partial_kernel, dim3(grid), dim3(kBlock), lds, s, n, nu, U, nv, V,
                     partials);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int npairs = nu * nv;
  hipLaunchKernelGGL(gram_reduce_kernel, dim3((npairs + kBlock - 1) / kBlock), dim3(kBlock), 0, s,
                     npairs, grid, partials, G);
  return hipGetLastError();
}

}  // namespace spis
