// sptrsv.hip — K8: sync-free level-blocked triangular solves of a device ILU apply (sptrsv.h).
//
// Roofline: latency, not bandwidth.  The factors are read once per apply (12 B per entry +
// 16 B per row ≈ 150 MB for swe M=256), which at HBM rate is ~30 us; the apply's floor is the
// critical path — one in-launch hand-off (~1 us, MI355X_MICROARCH.md handoff-1to1) per block
// boundary along the longest dependency chain, plus one LDS round trip per level inside a block.
#include "sptrsv.h"

#include <algorithm>

namespace spis {
namespace {

typedef __attribute__((address_space(1))) unsigned long long gu64;
constexpr int kTriWaves = 4;  // independent waves per workgroup, each with its own tickets
constexpr unsigned long long kWaitTicks = 500000000ull;  // 5 s at 100 MHz

__device__ __forceinline__ unsigned long long ld_granule(const double* p) {
  return __hip_atomic_load((gu64*)(p), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_granule(double* p, double v) {
  __hip_atomic_store((gu64*)(p), static_cast<unsigned long long>(__double_as_longlong(v)),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// value of a position another wave publishes: poll its granule until it is no longer the sentinel
// (rows of earlier tickets); a wait longer than ~5 s of wall clock (s_memrealtime, 100 MHz) is a
// plan bug: flag it and go on with NaN so that no wave is left waiting
template <int SLEEP>
__device__ __forceinline__ double poll(const double* g, unsigned* err) {
  unsigned long long x = ld_granule(g);
  if (x != kTriSentinel) return __longlong_as_double(static_cast<long long>(x));
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (unsigned spins = 1;; ++spins) {
    __builtin_amdgcn_s_sleep(SLEEP);
    x = ld_granule(g);
    if (x != kTriSentinel) return __longlong_as_double(static_cast<long long>(x));
    if ((spins & 255) == 0 && __builtin_amdgcn_s_memrealtime() - t0 > kWaitTicks) {
      atomicOr(err, 1u);
      return __longlong_as_double(0x7FF8000000000000ll);
    }
  }
}

template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// sum over aligned groups of g lanes (g = 1, 2, 4, 8, 16; uniform), result in every lane of the
// group: DPP moves (ALU latency) instead of ds_bpermute (LDS latency) on the critical path
__device__ __forceinline__ double group_sum(double v, int g) {
  if (g >= 2) v += dpp_d<0xB1>(v);   // quad_perm [1,0,3,2]
  if (g >= 4) v += dpp_d<0x4E>(v);   // quad_perm [2,3,0,1]
  if (g >= 8) v += dpp_d<0x141>(v);  // row_half_mirror: lane i <-> 7 - i of each 8
  if (g >= 16) v += dpp_d<0x140>(v); // row_mirror: lane i <-> 15 - i of each 16
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// one wave's LDS: the block's rows, entries and values (staged once per block, one round trip)
struct WaveLds {
  double v[kTriBlockCap];      // row values; before a row's step: q (L) or the diagonal (U)
  double a[kTriBlockNnz];      // entry values
  int32_t c[kTriBlockNnz];     // entry positions
  int32_t rp[kTriBlockCap + 1];  // row starts, relative to the block's first entry
  int32_t st[kTriBlockCap + 1];  // step starts, relative to the block's first row
  int32_t in[kTriBlockCap];    // L: index of q; U: position of y
  double y[kTriBlockCap];      // U: y of the block's rows (fetched at staging)
  int32_t out[kTriBlockCap];   // U: index of z
};
constexpr int kStageEnt = kTriBlockNnz / 64;        // entries per lane
constexpr int kStageRow = (kTriBlockCap + 64) / 64; // row-array words per lane (cap + 1)

template <typename T, int PER>
__device__ __forceinline__ void stage_load(T (&r)[PER], const T* __restrict__ src, int cnt, int lane) {
#pragma unroll
  for (int k = 0; k < PER; ++k) r[k] = src[min(lane + 64 * k, max(cnt - 1, 0))];
}
template <typename T, int PER>
__device__ __forceinline__ void stage_store(T* dst, const T (&r)[PER], int cnt, int lane) {
#pragma unroll
  for (int k = 0; k < PER; ++k)
    if (lane + 64 * k < cnt) dst[lane + 64 * k] = r[k];
}

__device__ __forceinline__ void wave_lds_sync() {  // this wave's LDS writes before its next reads
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

// a staged block: consecutive narrow levels (or one 64-row slice of a wide level), every
// structure read from LDS; only dependencies of earlier blocks are read from granules
template <bool UPPER, int SLEEP>
__device__ __forceinline__ void solve_staged(const TriDev& F, int b, const double* __restrict__ q,
                                             const double* gin, double* gout, double* __restrict__ z,
                                             WaveLds& W, unsigned* err, int lane) {
  const int r0 = F.blk_row[b], nr = F.blk_row[b + 1] - r0;
  const int s0 = F.blk_step[b], ns = F.blk_step[b + 1] - s0;
  const int e0 = F.blk_ent[b], ne = F.blk_ent[b + 1] - e0;
  {  // every load of the block's structure in flight at once
    int32_t c[kStageEnt], rp[kStageRow], st[kStageRow], in[kStageRow], out[kStageRow];
    double a[kStageEnt], d[kStageRow];
    stage_load(c, F.col + e0, ne, lane);
    stage_load(a, F.val + e0, ne, lane);
    stage_load(rp, F.rowptr + r0, nr + 1, lane);
    stage_load(st, F.step_row + s0, ns + 1, lane);
    stage_load(in, F.in_idx + r0, nr, lane);
    double y[kStageRow];
    if (UPPER) {
      stage_load(out, F.out_idx + r0, nr, lane);
      stage_load(d, F.diag + r0, nr, lane);
      unsigned long long gy[kStageRow];  // L finished these long ago (all L tickets come first)
#pragma unroll
      for (int k = 0; k < kStageRow; ++k) gy[k] = ld_granule(gin + in[k]);
#pragma unroll
      for (int k = 0; k < kStageRow; ++k)
        y[k] = (gy[k] == kTriSentinel && lane + 64 * k < nr) ? poll<SLEEP>(gin + in[k], err)
                                                               : __longlong_as_double(static_cast<long long>(gy[k]));
    } else {
#pragma unroll
      for (int k = 0; k < kStageRow; ++k) d[k] = q[in[k]];
    }
#pragma unroll
    for (int k = 0; k < kStageRow; ++k) {
      rp[k] -= e0;
      st[k] -= r0;
    }
    stage_store(W.c, c, ne, lane);
    stage_store(W.a, a, ne, lane);
    stage_store(W.rp, rp, nr + 1, lane);
    stage_store(W.st, st, ns + 1, lane);
    stage_store(W.in, in, nr, lane);
    if (UPPER) {
      stage_store(W.out, out, nr, lane);
      stage_store(W.y, y, nr, lane);
    }
    stage_store(W.v, d, nr, lane);
  }
  wave_lds_sync();
  for (int s = 0; s < ns; ++s) {
    const int a0 = W.st[s], m = W.st[s + 1] - a0;
    // g lanes per row (a power of two, <= 16): narrow steps split each row over a lane group
    const int lg = m <= 4 ? 4 : m <= 8 ? 3 : m <= 16 ? 2 : m <= 32 ? 1 : 0;
    const int g = 1 << lg, sub = lane & (g - 1);
    const int lr = a0 + (lane >> lg);  // local row
    const bool active = (lane >> lg) < m;
    double part = 0.0;
    if (active) {
      // the row's right-hand side starts the sum of the group's first lane, so a lone lane
      // computes ((b - a_1 v_1) - a_2 v_2) - ... exactly as the column sweep does
      if (sub == 0) part = UPPER ? W.y[lr] : W.v[lr];
      const int eb = W.rp[lr], ee = W.rp[lr + 1];
      // a lone lane (g = 1) subtracts in SuperLU's order (increasing columns for L, decreasing
      // for U: the builder stores each row's entries in that order); a group sums its share
      for (int e = eb + sub; e < ee; e += 8 * g) {
        int c[8];
        double a[8], v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int ek = min(e + k * g, ee - 1);
          c[k] = W.c[ek];
          a[k] = W.a[ek];
        }
        bool far = false;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          v[k] = W.v[max(c[k] - r0, 0)];
          far |= c[k] < r0;
        }
        if (far) {  // some dependency lives in an earlier block: read its granules
          unsigned long long gr[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) gr[k] = ld_granule(gout + c[k]);
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if (c[k] < r0) v[k] = __longlong_as_double(static_cast<long long>(gr[k]));
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if (e + k * g < ee) {
            if (static_cast<unsigned long long>(__double_as_longlong(v[k])) == kTriSentinel)
              v[k] = poll<SLEEP>(gout + c[k], err);
            part -= a[k] * v[k];
          }
        }
      }
    }
    part = group_sum(part, g);
    if (active && sub == 0) {
      double acc = part;
      if (UPPER) acc /= W.v[lr];
      W.v[lr] = acc;
      st_granule(gout + r0 + lr, acc);
      if (UPPER) z[W.out[lr]] = acc;
    }
    wave_lds_sync();  // the next step's lanes read this step's values
  }
}

// a long-row block: one step of <= kLongStep rows of a level holding a row longer than kLongRow;
// each row is split over the wave's lanes and summed by a wave reduction
template <bool UPPER, int SLEEP>
__device__ __forceinline__ void solve_long(const TriDev& F, int b, const double* __restrict__ q,
                                           const double* gin, double* gout, double* __restrict__ z,
                                           unsigned* err, int lane) {
  const int r0 = F.blk_row[b], r1 = F.blk_row[b + 1];
  for (int row = r0; row < r1; ++row) {
    const int e0 = F.rowptr[row], e1 = F.rowptr[row + 1];
    double part = 0.0;
    for (int e = e0 + lane; e < e1; e += 256) {  // 4 entries per lane in flight
      int c[4];
      double a[4], v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int ek = e + 64 * k < e1 ? e + 64 * k : e0;
        c[k] = F.col[ek];
        a[k] = F.val[ek];
      }
      unsigned long long g[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) g[k] = ld_granule(gout + c[k]);  // rows of this block are one level
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (e + 64 * k < e1) {
          v[k] = g[k] == kTriSentinel ? poll<SLEEP>(gout + c[k], err)
                                      : __longlong_as_double(static_cast<long long>(g[k]));
          part += a[k] * v[k];
        }
      }
    }
    const double sum = wave_sum_d(part);
    double acc = UPPER ? poll<SLEEP>(gin + F.in_idx[row], err) : q[F.in_idx[row]];
    acc -= sum;
    if (UPPER) acc /= F.diag[row];
    if (lane == 0) {
      st_granule(gout + row, acc);
      if (UPPER) z[F.out_idx[row]] = acc;
    }
  }
}

template <int SLEEP>
__global__ __launch_bounds__(kTriWaves * 64) void ilu_apply_kernel(TriDev L, TriDev U,
                                                                   const double* __restrict__ q, double* gy,
                                                                   double* gv, double* __restrict__ z,
                                                                   unsigned* ticket, unsigned* err) {
  __shared__ WaveLds lds[kTriWaves];
  const int lane = threadIdx.x & 63;
  WaveLds& W = lds[threadIdx.x >> 6];
  const int nb = L.nb + U.nb;
  for (;;) {
    int t = 0;
    if (lane == 0) t = static_cast<int>(atomicAdd(ticket, 1u));
    t = __builtin_amdgcn_readfirstlane(t);
    if (t >= nb) break;
    if (t < L.nb) {
      if (L.blk_long[t]) solve_long<false, SLEEP>(L, t, q, nullptr, gy, nullptr, err, lane);
      else solve_staged<false, SLEEP>(L, t, q, nullptr, gy, nullptr, W, err, lane);
    } else {
      const int b = t - L.nb;
      if (U.blk_long[b]) solve_long<true, SLEEP>(U, b, nullptr, gy, gv, z, err, lane);
      else solve_staged<true, SLEEP>(U, b, nullptr, gy, gv, z, W, err, lane);
    }
  }
}

}  // namespace

hipError_t launch_ilu_apply(int64_t n, const TriDev& L, const TriDev& U, const double* q, double* gran,
                            double* z, unsigned* ticket, unsigned* err, hipStream_t s) {
  if (n == 0) return hipSuccess;
  // granules back to the sentinel and the ticket to 0 before EVERY launch
  double* gy = gran;
  double* gv = gran + n;
  hipError_t e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(gran), 0xFFF7FFF7u,
                                   static_cast<size_t>(2 * n) * 2, s);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(ticket, 0, sizeof(unsigned), s);
  if (e != hipSuccess) return e;
  const int nb = L.nb + U.nb;
  // one workgroup per CU (the four waves' LDS windows take 128 KiB); polling waves sleep 64
  // clocks between polls (a sweep of 64-512 workgroups and 1-16 sleeps moved the time < 3 %)
  const int grid = std::max(1, std::min((nb + kTriWaves - 1) / kTriWaves, 256));
  hipLaunchKernelGGL(ilu_apply_kernel<1>, dim3(grid), dim3(kTriWaves * 64), 0, s, L, U, q, gy, gv, z, ticket, err);
  return hipGetLastError();
}

}  // namespace spis
