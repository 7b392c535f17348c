// spmv_variants.hip — SpMV kernel variants measured and not adopted (tuning tool only; included
// by tools/kbench.hip after csrc/kernels.hip, never part of libspis).  Moved out of the library in
// round 4.  Each was bit-identical to SciPy row by row and slower than the shipping
// K1p / K1dp (csrc/kernels.hip spmv_pipe_kernel); measurements (profiles/):
//   NT (nontemporal matrix stream): C5 cold Arnoldi SpMV 404 -> 397 us, dual 497 -> 627 us
//     (profiles/r03_c5_spmv_traffic_nt1.json);
//   WPE = 4 + BUF (4 waves per SIMD, buffer-descriptor stream and gathers, late values, partial
//     sums in LDS): C5 Arnoldi 367 -> 356 us, dual 449 -> 453 us, C3 dual 36.7 -> 37.3 us
//     (profiles/r03_spmv_sweep_w4.txt);
//   BUF at 3 waves per SIMD: C5 dual 452 -> 451 us, C3 dual 35.8 -> 37.3 us
//     (profiles/r03_spmv_sweep_buf3.txt);
//   TM (thread-major 16-bit columns, one 16-B column load per thread and block): C5 dual
//     454 -> 562 us, C3 dual 35.9 -> 48.8 us (profiles/r03_spmv_sweep_c16tm.txt);
//   spmv_pipe2_kernel (two-deep: the next block's gathers in flight too): slab order 49 vs 37.7 us
//     at C3, C5 553 vs 476 us cold;
//   spmv_sell_kernel (SELL-64 copy, lane = row, no LDS): C3 dual 43.2 vs 41.3 us, C5 530 vs 496 us
//     cold (profiles/r03_c5_spmv_sweep_sell.txt).
// Template parameters of spmv_pipe_var_kernel: <CAP, MODE, NT, WPE, C16, BUF, TM>, with the
// library kernel's arithmetic; <CAP, MODE, false, 1, C16> is the library kernel itself.
#pragma once

#include "win_table.h"

namespace spis {

constexpr int kSellW = 64;       // rows per SELL slice (a wave, lane = row)

typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
// one fp64 through a buffer descriptor at a 32-bit byte offset (K1s gathers: no 64-bit address
// registers per entry)
__device__ __forceinline__ double buf_ld1(__amdgpu_buffer_rsrc_t r, int voff) {
  const u32x2_t v = __builtin_amdgcn_raw_buffer_load_b64(r, voff, 0, 0);
  return __hiloint2double(static_cast<int>(v.y), static_cast<int>(v.x));
}

// the same with the element's distance in the scalar offset (K1p's matrix stream: one lane offset
// for all of a block's loads, the block's start in the descriptor's base)
__device__ __forceinline__ double buf_ld1s(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  const u32x2_t v = __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0);
  return __hiloint2double(static_cast<int>(v.y), static_cast<int>(v.x));
}

// block lb of the table (entries lb * ms, lb * ms + 1: ms = 1 consecutive starts, 2 (start, end)
// pairs); C16: the columns from the 16-bit copy and the block's bases base[lb]
// BUF stage: the values only (LATEV: issued once the current block's products are in LDS, so the
// next block's values are not live in registers across the current block's gathers)
template <int CAP>
__device__ __forceinline__ void pipe_load_vals_v(PipeStage<CAP>& st, const double* __restrict__ va) {
  if (st.nnz > CAP) return;
  const __amdgpu_buffer_rsrc_t rv = span_rsrc(va + st.nz0);
#pragma unroll
  for (int u = 0; u < PipeStage<CAP>::kPer; ++u)
    st.vals[u] = threadIdx.x + u * kBlock < st.nnz ? buf_ld1s(rv, threadIdx.x * 8, u * kBlock * 8) : 0.0;
}

template <int CAP, int MODE, bool NT = false, bool C16 = false, bool BUF = false, bool VALS = true, bool TM = false>
__device__ __forceinline__ void pipe_load_v(PipeStage<CAP>& st, const int2* __restrict__ meta, int lb, int ms,
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
  if constexpr (TM && C16 && !NT && !BUF) {
    // thread-major copy: this thread's kPer 16-bit columns in one 16-B load (no long rows here:
    // the host builds the copy only for matrices without them)
    static_assert(PipeStage<CAP>::kPer == 8, "one 16-B load = 8 columns");
    const uint4 v = *reinterpret_cast<const uint4*>(c16 + static_cast<int64_t>(lb) * CAP + threadIdx.x * 8);
    st.cols[0] = static_cast<int>(v.x & 0xffffu);
    st.cols[1] = static_cast<int>(v.x >> 16);
    st.cols[2] = static_cast<int>(v.y & 0xffffu);
    st.cols[3] = static_cast<int>(v.y >> 16);
    st.cols[4] = static_cast<int>(v.z & 0xffffu);
    st.cols[5] = static_cast<int>(v.z >> 16);
    st.cols[6] = static_cast<int>(v.w & 0xffffu);
    st.cols[7] = static_cast<int>(v.w >> 16);
#pragma unroll
    for (int u = 0; u < PipeStage<CAP>::kPer; ++u) {
      const int i = threadIdx.x + u * kBlock;
      st.vals[u] = i < st.nnz ? va[st.nz0 + i] : 0.0;
    }
  } else if constexpr (BUF && !NT) {
    // buffer descriptors based at the block's first nonzero: every load of the block shares the
    // lane offset, its distance u * kBlock elements rides in the scalar offset (no 64-bit address
    // registers per element, which is what kept the stage at 3 waves per SIMD)
    if constexpr (C16) {
      const __amdgpu_buffer_rsrc_t rc = span_rsrc(c16 + st.nz0);
#pragma unroll
      for (int u = 0; u < PipeStage<CAP>::kPer; ++u)
        st.cols[u] = threadIdx.x + u * kBlock < st.nnz
                         ? static_cast<int>(__builtin_amdgcn_raw_buffer_load_b16(rc, threadIdx.x * 2, u * kBlock * 2, 0))
                         : 0;
    } else {
      const __amdgpu_buffer_rsrc_t rc = span_rsrc(ci + st.nz0);
#pragma unroll
      for (int u = 0; u < PipeStage<CAP>::kPer; ++u)
        st.cols[u] = threadIdx.x + u * kBlock < st.nnz
                         ? static_cast<int>(__builtin_amdgcn_raw_buffer_load_b32(rc, threadIdx.x * 4, u * kBlock * 4, 0))
                         : 0;
    }
    if constexpr (VALS) pipe_load_vals_v<CAP>(st, va);
  } else {
#pragma unroll
  for (int u = 0; u < PipeStage<CAP>::kPer; ++u) {
    const int i = threadIdx.x + u * kBlock;
    if (C16 && NT) {  // streamed once (beyond the Infinity Cache): keep it for the gathered vectors
      st.cols[u] = i < st.nnz ? __builtin_nontemporal_load(c16 + st.nz0 + i) : 0;
      st.vals[u] = i < st.nnz ? __builtin_nontemporal_load(va + st.nz0 + i) : 0.0;
    } else if (C16) {
      st.cols[u] = i < st.nnz ? c16[st.nz0 + i] : 0;  // raw: decoded at the gathers, so the prefetch
                                                      // stays in flight (0 decodes to a column of the block)
      st.vals[u] = i < st.nnz ? va[st.nz0 + i] : 0.0;
    } else if (NT) {  // streamed once: keep L2 for the gathered vectors
      st.cols[u] = i < st.nnz ? __builtin_nontemporal_load(ci + st.nz0 + i) : 0;
      st.vals[u] = i < st.nnz ? __builtin_nontemporal_load(va + st.nz0 + i) : 0.0;
    } else {
      st.cols[u] = i < st.nnz ? ci[st.nz0 + i] : 0;
      st.vals[u] = i < st.nnz ? va[st.nz0 + i] : 0.0;
    }
  }
  }
  const int r = st.r0 + threadIdx.x;
  if (r < st.r1) {
    st.rs = rp[r] - st.nz0;
    st.re = rp[r + 1] - st.nz0;
    if (MODE != kEpiPlain) st.a1 = aux1[r];
    if (MODE == 4) st.a2 = aux2[r];
  } else {
    st.rs = st.re = 0;
  }
}

// x1/aux1/y1/part1: the single SpMV (MODE 0-3) or the residual half of the dual (aux1 = b);
// x2/aux2 (= q0)/y2 (= w)/part2: the dual's Arnoldi half
// C16: columns from the 16-bit copy (c16, per-block bases; col16.h)
// BUF: the matrix stream and the gathers through buffer descriptors (32-bit lane offsets), which
// frees the registers for WPE = 4 waves per SIMD (4 workgroups per CU instead of 3)
// FAKEG (timing probe only, wrong results): 1 = the x gathers replaced by coalesced loads of the
// block's own row range, 2 = by one broadcast address: what the kernel costs without gather latency;
// 3 (correct, DUAL only): x1 holds interleaved (x1, x2) pairs, one 16-B gather per nonzero
template <int CAP, int MODE, bool NT = false, int WPE = 1, bool C16 = false, bool BUF = false, bool TM = false,
          int FAKEG = 0>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WPE, WPE > 3 ? WPE : (C16 ? 3 : 8)))) void spmv_pipe_var_kernel(
    const int32_t* __restrict__ rp, const int32_t* __restrict__ ci, const double* __restrict__ va,
    const int2* __restrict__ meta, int n_blk, int walk, const double* __restrict__ x1,
    const double* __restrict__ aux1, double* __restrict__ y1, double* __restrict__ part1,
    const double* __restrict__ x2, const double* __restrict__ aux2, double* __restrict__ y2,
    double* __restrict__ part2, const uint16_t* __restrict__ c16, const int4* __restrict__ base) {
  constexpr bool DUAL = MODE == 4;
  constexpr int kPer = PipeStage<CAP>::kPer;
  constexpr bool LATEV = BUF && !NT && WPE > 3;  // 4 waves per SIMD: the next values loaded late
  // products at padded index i + i/16: one thread per row reads its row left to right, and rows
  // of 16 entries (swe's edge rows) would otherwise put a wave's lanes 256 B apart, all in one
  // LDS bank group; the pad staggers them
  __shared__ typename std::conditional<DUAL, double2, double>::type s_p[CAP + CAP / 16];
  __shared__ double s_wave[4];
  // LATEV: each thread's partial sums live in its own LDS slot between blocks (in registers they
  // were spilled, and a scratch reload waits for every load issued before it: the prefetch)
  __shared__ double2 s_pt[LATEV ? kBlock : 1];
  double pt1 = 0.0, pt2 = 0.0;
  if (LATEV) s_pt[threadIdx.x] = make_double2(0.0, 0.0);
  int b0, b1, bs;
  block_walk(n_blk, walk, b0, b1, bs);
  const int ms = walk == 2 ? 2 : 1;  // walk 2: (start, end) pair per block (an ordered table)
  const __amdgpu_buffer_rsrc_t rx1 = span_rsrc(x1);
  const __amdgpu_buffer_rsrc_t rx2 = span_rsrc(DUAL ? x2 : x1);
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
          if constexpr (FAKEG == 3) {
            acc1 += va[i] * x1[2 * c];
            acc2 += va[i] * x1[2 * c + 1];
          } else {
            acc1 += va[i] * x1[c];
            if (DUAL) acc2 += va[i] * x2[c];
          }
        }
        s1 = block_sum(acc1, s_wave);
        if (DUAL) s2 = block_sum(acc2, s_wave);
      }
      if (threadIdx.x == 0) {
        const int r0 = cur.r0;
        if (LATEV) {
          pt1 = s_pt[0].x;
          pt2 = s_pt[0].y;
        }
        if (DUAL) {
          const double t = s1 - aux1[r0];
          pt1 += t * t;
          y2[r0] = s2;
          pt2 += aux2[r0] * s2;
        }
        if (MODE == kEpiPlain) y1[r0] = s1;
        if (MODE == kEpiDot) { y1[r0] = s1; pt1 += aux1[r0] * s1; }
        if (MODE == kEpiResNorm) { const double t = s1 - aux1[r0]; pt1 += t * t; }
        if (MODE == kEpiR0) { const double t = aux1[r0] - s1; y1[r0] = t; pt1 += t * t; }
        if (LATEV) s_pt[0] = make_double2(pt1, pt2);
      }
      nxt.nnz = 0;
      if (nb < b1) pipe_load_v<CAP, MODE, NT, C16, BUF, true, TM>(nxt, meta, nb, ms, rp, ci, c16, base, va, aux1, aux2);
      return;
    }
    // this block's gathers first, then the next block's loads: the gathers' vmcnt wait does not
    // include the prefetch, and the prefetch is in flight through the LDS phase below
    double g1[kPer], g2[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      int c = C16 ? col16_decode(cur.cols[u], cur.bs0, cur.bs1, cur.bs2, cur.bs3) : cur.cols[u];
      if constexpr (FAKEG == 1) c = min(cur.r0 + ((threadIdx.x + u * kBlock) & 255), cur.r1 - 1);
      if constexpr (FAKEG == 2) c = cur.r0;
      if constexpr (FAKEG == 3) {
        const double2 pr = reinterpret_cast<const double2*>(x1)[c];
        g1[u] = pr.x;
        g2[u] = pr.y;
      } else if constexpr (BUF) {
        g1[u] = buf_ld1(rx1, c * 8);
        if (DUAL) g2[u] = buf_ld1(rx2, c * 8);
      } else {
        g1[u] = x1[c];
        if (DUAL) g2[u] = x2[c];
      }
    }
    nxt.nnz = 0;
    if (nb < b1) pipe_load_v<CAP, MODE, NT, C16, BUF, !LATEV, TM>(nxt, meta, nb, ms, rp, ci, c16, base, va, aux1, aux2);
    // entry i = tid + u kBlock sits at i + i/16 = (tid + tid/16) + u (kBlock + kBlock/16): one base
    // register and an immediate offset per u (the compiler's own form of i + i/16 kept 8 addresses
    // live, which spilled at 4 waves per SIMD)
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
    if (LATEV && nb < b1) pipe_load_vals_v<CAP>(nxt, va);
    const int r = cur.r0 + threadIdx.x;
    if (r < cur.r1) {
      double s1 = 0.0, s2 = 0.0;
      // LDS reads in flight in groups, then the adds in row order (the sum is still left to right)
      int t = cur.rs;
      for (; WPE < 4 && t + 8 <= cur.re; t += 8) {  // (at 4 waves per SIMD the group of 8 spills)
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
      if (LATEV) {
        pt1 = s_pt[threadIdx.x].x;
        pt2 = s_pt[threadIdx.x].y;
      }
      if (DUAL) {
        const double t = s1 - cur.a1;
        pt1 += t * t;
        y2[r] = s2;
        pt2 += cur.a2 * s2;
      }
      if (MODE == kEpiPlain) y1[r] = s1;
      if (MODE == kEpiDot) { y1[r] = s1; pt1 += cur.a1 * s1; }
      if (MODE == kEpiResNorm) { const double t = s1 - cur.a1; pt1 += t * t; }
      if (MODE == kEpiR0) { const double t = cur.a1 - s1; y1[r] = t; pt1 += t * t; }
      if (LATEV) s_pt[threadIdx.x] = make_double2(pt1, pt2);
    }
    __syncthreads();
  };
  PipeStage<CAP> sa, sb;
  if (b0 < b1) pipe_load_v<CAP, MODE, NT, C16, BUF, true, TM>(sa, meta, b0, ms, rp, ci, c16, base, va, aux1, aux2);
  for (int blk = b0; blk < b1; blk += 2 * bs) {
    step(sa, sb, blk);
    if (blk + bs >= b1) break;
    step(sb, sa, blk + bs);
  }
  if (LATEV) {
    pt1 = s_pt[threadIdx.x].x;
    pt2 = s_pt[threadIdx.x].y;
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

// Two-deep variant: block i+1's gathers and block i+2's val/col loads are in flight while block
// i's products go through LDS, so a workgroup's wait per block is max(memory latency, LDS phase)
// rather than their sum (~110 VGPRs: 4 workgroups per CU).  Same arithmetic as above.
template <int CAP, int MODE>
struct PipeGath {
  double g1[CAP / kBlock], g2[CAP / kBlock];
};

template <int CAP, int MODE>
__device__ __forceinline__ void pipe_gather(PipeGath<CAP, MODE>& G, const PipeStage<CAP>& st,
                                            const double* __restrict__ x1, const double* __restrict__ x2) {
  if (st.nnz > CAP) return;
#pragma unroll
  for (int u = 0; u < PipeStage<CAP>::kPer; ++u) {
    G.g1[u] = x1[st.cols[u]];
    if (MODE == 4) G.g2[u] = x2[st.cols[u]];
  }
}

template <int CAP, int MODE>
__global__ __launch_bounds__(kBlock) void spmv_pipe2_kernel(
    const int32_t* __restrict__ rp, const int32_t* __restrict__ ci, const double* __restrict__ va,
    const int2* __restrict__ meta, int n_blk, int walk, const double* __restrict__ x1,
    const double* __restrict__ aux1, double* __restrict__ y1, double* __restrict__ part1,
    const double* __restrict__ x2, const double* __restrict__ aux2, double* __restrict__ y2,
    double* __restrict__ part2) {
  constexpr bool DUAL = MODE == 4;
  constexpr int kPer = PipeStage<CAP>::kPer;
  __shared__ typename std::conditional<DUAL, double2, double>::type s_p[CAP + CAP / 16];
  __shared__ double s_wave[4];
  double pt1 = 0.0, pt2 = 0.0;
  int b0, b1, bs;
  block_walk(n_blk, walk, b0, b1, bs);
  const int ms = walk == 2 ? 2 : 1;  // walk 2: (start, end) pair per block (an ordered table)
  PipeStage<CAP> s0, s1;
  PipeGath<CAP, MODE> g0, g1n;
  s0.nnz = 0;
  s1.nnz = 0;
  if (b0 < b1) pipe_load_v<CAP, MODE>(s0, meta, b0, ms, rp, ci, nullptr, nullptr, va, aux1, aux2);
  if (b0 < b1) pipe_gather<CAP, MODE>(g0, s0, x1, x2);
  if (b0 + bs < b1) pipe_load_v<CAP, MODE>(s1, meta, b0 + bs, ms, rp, ci, nullptr, nullptr, va, aux1, aux2);
  for (int blk = b0; blk < b1; blk += bs) {
    // in flight from the previous round: g0 (block blk) and s1 (block blk + bs)
    if (blk + bs < b1) pipe_gather<CAP, MODE>(g1n, s1, x1, x2);
    PipeStage<CAP> s2;
    s2.nnz = 0;
    if (blk + 2 * bs < b1) pipe_load_v<CAP, MODE>(s2, meta, blk + 2 * bs, ms, rp, ci, nullptr, nullptr, va, aux1, aux2);
    if (s0.nnz > CAP) {  // one long row (r1 == r0 + 1): K1's workgroup reduction
      double acc1 = 0.0, acc2 = 0.0;
      for (int i = s0.nz0 + threadIdx.x; i < s0.nz0 + s0.nnz; i += kBlock) {
        acc1 += va[i] * x1[ci[i]];
        if (DUAL) acc2 += va[i] * x2[ci[i]];
      }
      const double s1v = block_sum(acc1, s_wave);
      const double s2v = DUAL ? block_sum(acc2, s_wave) : 0.0;
      if (threadIdx.x == 0) {
        const int r0 = s0.r0;
        if (DUAL) {
          const double t = s1v - aux1[r0];
          pt1 += t * t;
          y2[r0] = s2v;
          pt2 += aux2[r0] * s2v;
        }
        if (MODE == kEpiPlain) y1[r0] = s1v;
        if (MODE == kEpiDot) { y1[r0] = s1v; pt1 += aux1[r0] * s1v; }
        if (MODE == kEpiResNorm) { const double t = s1v - aux1[r0]; pt1 += t * t; }
        if (MODE == kEpiR0) { const double t = aux1[r0] - s1v; y1[r0] = t; pt1 += t * t; }
      }
    } else {
#pragma unroll
      for (int u = 0; u < kPer; ++u) {
        const int i = threadIdx.x + u * kBlock;
        if (i < s0.nnz) {
          if constexpr (DUAL)
            s_p[i + (i >> 4)] = make_double2(s0.vals[u] * g0.g1[u], s0.vals[u] * g0.g2[u]);
          else
            s_p[i + (i >> 4)] = s0.vals[u] * g0.g1[u];
        }
      }
      __syncthreads();
      const int r = s0.r0 + threadIdx.x;
      if (r < s0.r1) {
        double sa = 0.0, sb = 0.0;
        for (int t = s0.rs; t < s0.re; ++t) {
          if constexpr (DUAL) {
            const double2 pp = s_p[t + (t >> 4)];
            sa += pp.x;
            sb += pp.y;
          } else {
            sa += s_p[t + (t >> 4)];
          }
        }
        if (DUAL) {
          const double t = sa - s0.a1;
          pt1 += t * t;
          y2[r] = sb;
          pt2 += s0.a2 * sb;
        }
        if (MODE == kEpiPlain) y1[r] = sa;
        if (MODE == kEpiDot) { y1[r] = sa; pt1 += s0.a1 * sa; }
        if (MODE == kEpiResNorm) { const double t = sa - s0.a1; pt1 += t * t; }
        if (MODE == kEpiR0) { const double t = s0.a1 - sa; y1[r] = t; pt1 += t * t; }
      }
      __syncthreads();
    }
    s0 = s1;
    g0 = g1n;
    s1 = s2;
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

// ---------------------------------------------------------------------------------------------
// K1s: SpMV on a SELL-64 copy (sliced ELL, 64-row slices, entries t-major within a slice): one
// wave per slice, lane = row.  Entry t of all 64 rows is one coalesced 256-B col / 512-B val
// load, so a wave has its whole slice's (col, val) and gathers in flight with no LDS staging, no
// barrier and no row-sum phase (K1p: two barriers and an LDS pass per 2048-nnz block).  Each
// lane sums its row's rounded products left to right (contraction off): SciPy's csr_matvec
// order, so rows are bit-identical to K1 / K1p and to A @ x.  Padding (t >= the row's length)
// is loaded (col = the row itself) but never added.  MODE as K1p (0-3 = K1's epilogues on x1,
// 4 = the dual: residual of x1, Arnoldi of x2).  Walk: XCD-local eighths (walk 1) or
// grid-stride; partials per workgroup in wave order (deterministic).
// Measured at C3 (opt-in, SPIS_OPT_SPMV_PIPE = 6): dual 43.2 vs 41.3 us for K1dp (130 VGPRs, 3
// waves per SIMD, each slice two dependent round trips: col, then the gathers); forced to 4
// waves per SIMD 46.3 us (spills); with the next slice's (col, val) prefetched (207 VGPRs, 2
// waves per SIMD) 51.7 us.  The LDS-staged K1dp keeps more bytes in flight per VGPR.
// ---------------------------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(kBlock) void spmv_sell_kernel(
    int64_t n, int n_sl, int walk, const int64_t* __restrict__ off, const int32_t* __restrict__ scol,
    const double* __restrict__ sval, const uint16_t* __restrict__ slen, const double* __restrict__ x1,
    const double* __restrict__ aux1, double* __restrict__ y1, double* __restrict__ part1,
    const double* __restrict__ x2, const double* __restrict__ aux2, double* __restrict__ y2,
    double* __restrict__ part2) {
#pragma clang fp contract(off)
  constexpr bool DUAL = MODE == 4;
  constexpr int TW = 16;  // entries per lane in flight per chunk
  constexpr int NW = kBlock / 64;
  __shared__ double s_wave[4];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int64_t s0, s1e, ss;
  if (walk == 1 && (gridDim.x & 7) == 0) {  // XCD x = blockIdx % 8 walks the x-th eighth of the slices
    const int x = blockIdx.x & 7;
    s0 = (static_cast<int64_t>(n_sl) * x >> 3) + static_cast<int64_t>(blockIdx.x >> 3) * NW + wid;
    s1e = static_cast<int64_t>(n_sl) * (x + 1) >> 3;
    ss = static_cast<int64_t>(gridDim.x >> 3) * NW;
  } else {
    s0 = static_cast<int64_t>(blockIdx.x) * NW + wid;
    s1e = n_sl;
    ss = static_cast<int64_t>(gridDim.x) * NW;
  }
  // gathers through buffer descriptors (32-bit offsets; the host checks 8 n < 2^31)
  const __amdgpu_buffer_rsrc_t rx1 = vec_rsrc(x1, 8 * n);
  const __amdgpu_buffer_rsrc_t rx2 = vec_rsrc(DUAL ? x2 : x1, 8 * n);
  double pt1 = 0.0, pt2 = 0.0;
  for (int64_t sl = s0; sl < s1e; sl += ss) {
    const int64_t r = sl * kSellW + lane;
    const bool valid = r < n;
    const int len = valid ? static_cast<int>(slen[r]) : 0;
    const int64_t o = off[sl];
    const int w = static_cast<int>((off[sl + 1] - o) / kSellW);
    double a1 = 0.0, a2 = 0.0;
    for (int t0 = 0; t0 < w; t0 += TW) {
      int c[TW];
      double v[TW];
#pragma unroll
      for (int u = 0; u < TW; ++u)
        if (t0 + u < w) {  // wave-uniform
          c[u] = scol[o + static_cast<int64_t>(t0 + u) * kSellW + lane];
          v[u] = sval[o + static_cast<int64_t>(t0 + u) * kSellW + lane];
        }
      double g1[TW], g2[TW];
#pragma unroll
      for (int u = 0; u < TW; ++u)
        if (t0 + u < w) {
          g1[u] = buf_ld1(rx1, c[u] * 8);
          if (DUAL) g2[u] = buf_ld1(rx2, c[u] * 8);
        }
#pragma unroll
      for (int u = 0; u < TW; ++u)
        if (t0 + u < len) {
          a1 += v[u] * g1[u];
          if (DUAL) a2 += v[u] * g2[u];
        }
    }
    if (valid) {
      if (DUAL) {
        const double t = a1 - aux1[r];
        pt1 += t * t;
        y2[r] = a2;
        pt2 += aux2[r] * a2;
      }
      if (MODE == kEpiPlain) y1[r] = a1;
      if (MODE == kEpiDot) { y1[r] = a1; pt1 += aux1[r] * a1; }
      if (MODE == kEpiResNorm) { const double t = a1 - aux1[r]; pt1 += t * t; }
      if (MODE == kEpiR0) { const double t = aux1[r] - a1; y1[r] = t; pt1 += t * t; }
    }
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

// host side of TM (was col16.h)
// The same 16-bit columns thread-major per block, for the pipelined SpMV: table block k (nonzeros
// [e0, e1), in the table's order) occupies cap entries at k * cap, and thread t's per = cap / threads
// entries (its nonzeros e0 + t + u * threads, u < per) are contiguous, so a thread loads its
// columns with one 16-B load instead of per 2-B loads.  Padding entries are 0 (they decode to the
// block's first base column, as the kernels' predicated loads do).
inline void build_col16_tm(const std::vector<uint16_t>& col16, const std::vector<int32_t>& nz_ranges, int cap,
                           int threads, std::vector<uint16_t>& out) {
  const int64_t nb = static_cast<int64_t>(nz_ranges.size()) / 2;
  const int per = cap / threads;
  out.assign(static_cast<size_t>(std::max<int64_t>(nb, 1) * cap), 0);
  for (int64_t k = 0; k < nb; ++k) {
    const int64_t e0 = nz_ranges[2 * k], len = nz_ranges[2 * k + 1] - nz_ranges[2 * k];
    uint16_t* o = out.data() + k * cap;
    for (int t = 0; t < threads; ++t)
      for (int u = 0; u < per; ++u) {
        const int64_t i = t + static_cast<int64_t>(u) * threads;
        if (i < len) o[t * per + u] = col16[e0 + i];
      }
  }
}

// ---------------------------------------------------------------------------------------------
// K1w: the pipelined dual SpMV with windowed gathers (win_table.h).  K1dp gathers x1[c], x2[c]
// from global memory after the block's columns arrive: a dependent round trip per block that a
// probe measured at a third of the kernel (C3 dual 36.2 -> 24.6 us warm, C5 474 -> 300 us, with
// the gathers replaced by coalesced loads; profiles/r05_spmv_gather_probe.txt).  Here each block's
// x values arrive as whole 64-column chunks (its window, <= kWinChunks chunks, chunk ids from a
// table), loaded one block ahead with the block's values and 16-bit window positions: nothing in
// the prefetch depends on another load except the chunk ids, which are themselves loaded one
// block earlier still.  The window goes to LDS as (x1, x2) pairs, the products gather from it,
// and the row sums are K1's (left to right): rows bit-identical to SciPy.
// LDS: window 32 KB + products 34 KB: two workgroups per CU.
// ---------------------------------------------------------------------------------------------
#ifndef SPIS_WIN_WPE
#define SPIS_WIN_WPE 2  // waves per SIMD the kernel is compiled for (LDS allows 2 at 32 chunks)
#endif
constexpr int kWinPer = kWinChunks * 64 / kBlock;  // window pairs per thread
template <int CAP>
struct WinStage {
  static constexpr int kPer = CAP / kBlock;
  int r0, r1, nz0, nnz;
  int lid[kPer];
  double vals[kPer];
  int rs, re;
  double a1, a2;
  double2 win[kWinPer];
};

template <int CAP, int MODE>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(SPIS_WIN_WPE, SPIS_WIN_WPE))) void spmv_win_kernel(
    const int32_t* __restrict__ rp, const int32_t* __restrict__ ci, const double* __restrict__ va,
    const uint16_t* __restrict__ lidx, const int32_t* __restrict__ chunks, const int2* __restrict__ meta, int n_blk,
    int walk, const double* __restrict__ x1, const double* __restrict__ aux1, double* __restrict__ part1,
    const double* __restrict__ x2, const double* __restrict__ aux2, double* __restrict__ y2,
    double* __restrict__ part2) {
  static_assert(MODE == 4, "the dual (residual of x1 against aux1 = b, Arnoldi w = A x2, q0 . w)");
  constexpr int kPer = WinStage<CAP>::kPer;
  __shared__ double2 s_p[CAP + CAP / 16];
  __shared__ double2 s_w[kWinChunks * 64];
  __shared__ double s_wave[4];
  double pt1 = 0.0, pt2 = 0.0;
  int b0, b1, bs;
  block_walk(n_blk, walk, b0, b1, bs);
  const int ms = walk == 2 ? 2 : 1;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // chunk ids of this thread's window pairs (slot wave + 4 u) for a block
  auto load_ids = [&](int lb, int (&ids)[kWinPer]) {
#pragma unroll
    for (int u = 0; u < kWinPer; ++u) ids[u] = lb < b1 ? chunks[static_cast<int64_t>(lb) * kWinChunks + wave + 4 * u] : -1;
  };
  auto load = [&](WinStage<CAP>& st, int lb, const int (&ids)[kWinPer]) {
    const int2 m0 = meta[lb * ms];
    const int2 m1 = meta[lb * ms + 1];
    st.r0 = m0.x;
    st.r1 = m1.x;
    st.nz0 = m0.y;
    st.nnz = m1.y - m0.y;
#pragma unroll
    for (int u = 0; u < kWinPer; ++u) {
      const int c = ids[u] * 64 + lane;
      st.win[u] = ids[u] >= 0 ? make_double2(x1[c], x2[c]) : make_double2(0.0, 0.0);
    }
    if (st.nnz > CAP) return;  // a long row: read directly by the workgroup-wide path
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int i = threadIdx.x + u * kBlock;
      st.lid[u] = i < st.nnz ? lidx[st.nz0 + i] : 0;
      st.vals[u] = i < st.nnz ? va[st.nz0 + i] : 0.0;
    }
    const int r = st.r0 + threadIdx.x;
    if (r < st.r1) {
      st.rs = rp[r] - st.nz0;
      st.re = rp[r + 1] - st.nz0;
      st.a1 = aux1[r];
      st.a2 = aux2[r];
    } else {
      st.rs = st.re = 0;
    }
  };
  int ids[kWinPer];  // the chunk ids of the block after the next one
  auto step = [&](WinStage<CAP>& cur, WinStage<CAP>& nxt, int blk) __attribute__((always_inline)) {
    const int nb = blk + bs;
    if (cur.nnz > CAP) {  // one long row (r1 == r0 + 1): K1's workgroup reduction on the columns
      double acc1 = 0.0, acc2 = 0.0;
      for (int i = cur.nz0 + threadIdx.x; i < cur.nz0 + cur.nnz; i += kBlock) {
        const int c = ci[i];
        acc1 += va[i] * x1[c];
        acc2 += va[i] * x2[c];
      }
      const double s1 = block_sum(acc1, s_wave), s2 = block_sum(acc2, s_wave);
      if (threadIdx.x == 0) {
        const int r0 = cur.r0;
        const double t = s1 - aux1[r0];
        pt1 += t * t;
        y2[r0] = s2;
        pt2 += aux2[r0] * s2;
      }
      if (nb < b1) load(nxt, nb, ids);
      load_ids(nb + bs, ids);
      return;
    }
    // the next block's window, values and positions first: in flight through this block's LDS phases
    if (nb < b1) load(nxt, nb, ids);
    load_ids(nb + bs, ids);
#pragma unroll
    for (int u = 0; u < kWinPer; ++u) s_w[threadIdx.x + u * kBlock] = cur.win[u];
    __syncthreads();
    const int pbase = threadIdx.x + (threadIdx.x >> 4);
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int i = threadIdx.x + u * kBlock;
      if (i < cur.nnz) {
        const double2 g = s_w[cur.lid[u]];
        s_p[pbase + u * (kBlock + kBlock / 16)] = make_double2(cur.vals[u] * g.x, cur.vals[u] * g.y);
      }
    }
    __syncthreads();
    const int r = cur.r0 + threadIdx.x;
    if (r < cur.r1) {
      double s1 = 0.0, s2 = 0.0;
      int t = cur.rs;
      for (; t + 8 <= cur.re; t += 8) {
        double2 pp[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) pp[u] = s_p[t + u + ((t + u) >> 4)];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          s1 += pp[u].x;
          s2 += pp[u].y;
        }
      }
      for (; t + 4 <= cur.re; t += 4) {
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
      }
      for (; t < cur.re; ++t) {
        const double2 pp = s_p[t + (t >> 4)];
        s1 += pp.x;
        s2 += pp.y;
      }
      const double tt = s1 - cur.a1;
      pt1 += tt * tt;
      y2[r] = s2;
      pt2 += cur.a2 * s2;
    }
    __syncthreads();
  };
  WinStage<CAP> sa, sb;
  if (b0 < b1) {
    load_ids(b0, ids);
    load(sa, b0, ids);
    load_ids(b0 + bs, ids);
  }
  for (int blk = b0; blk < b1; blk += 2 * bs) {
    step(sa, sb, blk);
    if (blk + bs >= b1) break;
    step(sb, sa, blk + bs);
  }
  const double tot1 = block_sum(pt1, s_wave);
  const double tot2 = block_sum(pt2, s_wave);
  if (threadIdx.x == 0) {
    part1[blockIdx.x] = tot1;
    part2[blockIdx.x] = tot2;
  }
}

}  // namespace spis
