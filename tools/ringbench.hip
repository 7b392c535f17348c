// ringbench.hip — prototype of K1r, the SELL-64 SpMV fed by an LDS-DMA ring (tuning tool, not
// part of libspis).  VERDICT r3 item 4 / DESIGN.md §3 "what would lift it": the matrix stream's
// bytes in flight are bounded, in K1p, by the VGPRs that stage them and by the one in-order vmcnt
// the stream shares with the x gathers.  Here dedicated loader waves copy the (val, col) stream into
// a 3-slot LDS ring with global_load_lds (no VGPR staging, their own vmcnt), and consumer waves
// read it lane = row (SELL-64: entry t of a slice's 64 rows contiguous, so conflict-free LDS reads
// and no product array), gather x, and sum each row left to right (contraction off: SciPy's
// csr_matvec order, rows bit-identical to A @ x).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ringbench.hip -o tools/ringbench
//   python tools/dump_matrix.py 913 /tmp/m913 && tools/ringbench /tmp/m913
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../structurepreservingiterativesolvers_amd/csrc/col16.h"
#include "../structurepreservingiterativesolvers_amd/csrc/slab_order.h"

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

constexpr int kSl = 64;  // rows per SELL slice (a wave, lane = row)
constexpr int kR = 3;    // ring slots

// s_waitcnt vmcnt(N) alone (gfx9 encoding: vmcnt [3:0] + [15:14], expcnt and lgkmcnt at their max)
#define WAIT_VM(N) __builtin_amdgcn_s_waitcnt(((N) & 0xF) | ((((N) >> 4) & 3) << 14) | (0x7 << 4) | (0xF << 8))

__device__ __forceinline__ void glds16(const void* src, void* lds_dst) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}

// slot k of the plan: {first storage slice, slices, first entry, entries}
// MODE 0: y2 = A x2, pt2 += aux2 . y2 (the Arnoldi SpMV with its q0 dot); MODE 1: the dual, also
// ||A x1 - aux1||^2 partials (the true residual of x1)
template <int MODE, int NC, int NL, int SLOT, bool C16>
__global__ __launch_bounds__((NC + NL) * 64) void spmv_ring_kernel(
    const int4* __restrict__ slots, const int* __restrict__ wg_slot, const int* __restrict__ s_ent,
    const int* __restrict__ s_row, const uint8_t* __restrict__ rlen, const double* __restrict__ sval,
    const void* __restrict__ scol, const int4* __restrict__ s_base, int64_t n, const double* __restrict__ x1, const double* __restrict__ aux1,
    double* __restrict__ part1, const double* __restrict__ x2, const double* __restrict__ aux2,
    double* __restrict__ y2, double* __restrict__ part2) {
#pragma clang fp contract(off)
  constexpr int CB = C16 ? 2 : 4;                 // column bytes
  constexpr int VI = SLOT * 8 / 1024;             // 1-KiB DMA pieces of values per slot
  constexpr int CI = SLOT * CB / 1024;            // ... of columns
  static_assert((VI + CI) % NL == 0, "pieces split evenly over the loader waves");
  constexpr int L = (VI + CI) / NL;               // pieces per loader wave per slot
  static_assert(2 * L <= 63, "two slots in flight fit vmcnt");
  constexpr int SB = SLOT * (8 + CB);             // slot bytes
  __shared__ __attribute__((aligned(16))) char ring[kR][SB];
  __shared__ double s_red[2][NC];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int G = gridDim.x;
  const int ri = (G & 7) == 0 ? (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  const int k0 = wg_slot[ri], k1 = wg_slot[ri + 1];
  if (wid < NL) {  // ---- loader wave: DMA only (no ordinary loads whose results it waits for)
    auto issue = [&](int k) {
      const int e0 = slots[k].z;
      const char* vs = reinterpret_cast<const char*>(sval + e0) + lane * 16;
      const char* cs = reinterpret_cast<const char*>(scol) + static_cast<int64_t>(e0) * CB + lane * 16;
      char* d = ring[(k - k0) % kR];
#pragma unroll
      for (int u = 0; u < L; ++u) {
        const int i = wid + u * NL;
        if (i < VI)
          glds16(vs + i * 1024, d + i * 1024);
        else
          glds16(cs + (i - VI) * 1024, d + SLOT * 8 + (i - VI) * 1024);
      }
    };
    if (k0 < k1) issue(k0);
    if (k0 + 1 < k1) {
      issue(k0 + 1);
      WAIT_VM(L);
    } else {
      WAIT_VM(0);
    }
    __builtin_amdgcn_s_barrier();
    for (int k = k0; k < k1; ++k) {
      if (k + 2 < k1) {
        issue(k + 2);  // into the slot step k - 1 consumed (a barrier ago)
        WAIT_VM(L);    // slot k + 1 has landed
      } else {
        WAIT_VM(0);
      }
      __builtin_amdgcn_s_barrier();
    }
  } else {  // ---- consumer wave c: slices c, c + NC, ... of each slot, lane = row
    const int c = wid - NL;
    double pt1 = 0.0, pt2 = 0.0;
    __builtin_amdgcn_s_barrier();
    for (int k = k0; k < k1; ++k) {
      const int4 sl = slots[k];
      const char* buf = ring[(k - k0) % kR];
      for (int i = c; i < sl.y; i += NC) {
        const int s = sl.x + i;
        const int e0 = s_ent[s] - sl.z;
        const int w = (s_ent[s + 1] - s_ent[s]) / kSl;
        const int4 bs = C16 ? s_base[s] : int4{0, 0, 0, 0};
        const double* lv = reinterpret_cast<const double*>(buf) + e0;
        const int64_t r = static_cast<int64_t>(s_row[s]) + lane;
        const bool valid = r < n;
        const int len = valid ? rlen[r] : 0;
        // the epilogue's row values go out with the gathers (one memory round trip per slice)
        const double b1 = (MODE == 1 && valid) ? aux1[r] : 0.0;
        const double b2 = valid ? aux2[r] : 0.0;
        double a1 = 0.0, a2 = 0.0;
        constexpr int TW = 16;
        for (int t0 = 0; t0 < w; t0 += TW) {
          int cc[TW];
          double v[TW], g1[TW], g2[TW];
          // entries beyond the slice width re-read its last column (no branches around the loads:
          // a wave-uniform branch per entry made the compiler wait for every load at each join)
#pragma unroll
          for (int u = 0; u < TW; ++u) {
            const int t = min(t0 + u, w - 1) * kSl + lane;
            if (C16) {  // 2-bit base index + 14-bit offset (col16.h, per slice)
              const int cw = reinterpret_cast<const uint16_t*>(buf + SLOT * 8)[e0 + t];
              const int j = cw >> 14;
              cc[u] = (j == 0 ? bs.x : j == 1 ? bs.y : j == 2 ? bs.z : bs.w) + (cw & 0x3fff);
            } else
              cc[u] = reinterpret_cast<const int*>(buf + SLOT * 8)[e0 + t];
            v[u] = lv[t];
          }
#pragma unroll
          for (int u = 0; u < TW; ++u) {
            if (MODE == 1) g1[u] = x1[cc[u]];
            g2[u] = x2[cc[u]];
          }
#pragma unroll
          for (int u = 0; u < TW; ++u)
            if (t0 + u < len) {
              if (MODE == 1) a1 += v[u] * g1[u];
              a2 += v[u] * g2[u];
            }
        }
        if (valid) {
          if (MODE == 1) {
            const double t = a1 - b1;
            pt1 += t * t;
          }
          y2[r] = a2;
          pt2 += b2 * a2;
        }
      }
      __builtin_amdgcn_s_barrier();
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      pt1 += __shfl_xor(pt1, o, 64);
      pt2 += __shfl_xor(pt2, o, 64);
    }
    if (lane == 0) {
      s_red[0][c] = pt1;
      s_red[1][c] = pt2;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double t1 = 0.0, t2 = 0.0;
    for (int c = 0; c < NC; ++c) {
      t1 += s_red[0][c];
      t2 += s_red[1][c];
    }
    if (MODE == 1) part1[blockIdx.x] = t1;
    part2[blockIdx.x] = t2;
  }
}

__global__ void evict_kernel(int64_t m, const double2* __restrict__ x, double* __restrict__ out) {
  double a = 0.0;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < m;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const double2 v = x[i];
    a += v.x + v.y;
  }
  if (a == 12345.678) out[0] = a;
}

template <typename T>
static std::vector<T> load(const std::string& p, size_t n) {
  std::vector<T> v(n);
  FILE* f = fopen(p.c_str(), "rb");
  if (!f || fread(v.data(), sizeof(T), n, f) != n) {
    fprintf(stderr, "cannot read %s\n", p.c_str());
    exit(1);
  }
  fclose(f);
  return v;
}

struct Plan {
  std::vector<int4> slots;
  std::vector<int> wg_slot;
};

// greedy slots of consecutive storage slices (<= slot entries, <= maxs slices), then G contiguous
// ranges balanced by entries, range index (b % 8) * G / 8 + b / 8 for workgroup b (XCD b % 8 walks
// the b % 8-th eighth of the storage order)
static Plan make_plan(const std::vector<int>& s_ent, int slot, int maxs, int G) {
  Plan p;
  const int ns = static_cast<int>(s_ent.size()) - 1;
  int s = 0;
  while (s < ns) {
    int4 q{s, 0, s_ent[s], 0};
    while (s < ns && q.y < maxs && q.w + (s_ent[s + 1] - s_ent[s]) <= slot) {
      q.w += s_ent[s + 1] - s_ent[s];
      ++q.y;
      ++s;
    }
    if (q.y == 0) {
      fprintf(stderr, "slice %d wider than a slot\n", s);
      exit(1);
    }
    p.slots.push_back(q);
  }
  const int nk = static_cast<int>(p.slots.size());
  std::vector<double> cum(nk + 1, 0.0);
  for (int k = 0; k < nk; ++k) cum[k + 1] = cum[k] + p.slots[k].w;
  p.wg_slot.assign(G + 1, 0);
  int k = 0;
  for (int r = 0; r <= G; ++r) {
    const double target = cum[nk] * r / G;
    while (k < nk && cum[k] < target) ++k;
    p.wg_slot[r] = r == G ? nk : k;
  }
  return p;
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp/kbench_mat";
  const bool use_slab = !(argc > 2 && std::string(argv[2]) == "natural");
  auto shp = load<int64_t>(dir + "/shape.bin", 2);
  const int64_t n = shp[0], nnz = shp[1];
  auto rp = load<int32_t>(dir + "/indptr.bin", n + 1);
  auto ci = load<int32_t>(dir + "/indices.bin", nnz);
  auto va = load<double>(dir + "/data.bin", nnz);
  const int ns = static_cast<int>((n + kSl - 1) / kSl);
  std::vector<int32_t> sblk(ns + 1);
  for (int s = 0; s <= ns; ++s) sblk[s] = static_cast<int32_t>(std::min<int64_t>(n, int64_t(s) * kSl));
  std::vector<int64_t> order(ns);
  for (int s = 0; s < ns; ++s) order[s] = s;
  if (use_slab) {
    std::vector<uint8_t> lab;
    std::vector<double> key;
    std::vector<int32_t> pairs;
    if (spis::slab_labels(n, rp.data(), ci.data(), lab, &key))
      spis::build_slab_order(rp.data(), lab, sblk, pairs, &order, &key);
  }
  // SELL storage in slab order; 16-bit columns as offsets from the slice's first column range are
  // not modelled here: C16 stores the column mod 65536 only when every column of the matrix fits
  std::vector<int> s_ent(ns + 1), s_row(ns);
  std::vector<uint8_t> rlen(n);
  int wmax = 0;
  for (int64_t r = 0; r < n; ++r) {
    const int l = rp[r + 1] - rp[r];
    if (l > 255) {
      fprintf(stderr, "row %lld longer than 255\n", (long long)r);
      return 1;
    }
    rlen[r] = static_cast<uint8_t>(l);
  }
  int64_t ent = 0;
  for (int i = 0; i < ns; ++i) {
    const int s = static_cast<int>(order[i]);
    int w = 0;
    for (int32_t r = sblk[s]; r < sblk[s + 1]; ++r) w = std::max(w, rp[r + 1] - rp[r]);
    s_ent[i] = static_cast<int>(ent);
    s_row[i] = sblk[s];
    ent += int64_t(w) * kSl;
    wmax = std::max(wmax, w);
  }
  s_ent[ns] = static_cast<int>(ent);
  const int kSlotMax = 8192;
  std::vector<double> sv(ent + kSlotMax, 0.0);
  std::vector<int32_t> sc(ent + kSlotMax, 0);
  for (int i = 0; i < ns; ++i) {
    const int64_t e0 = s_ent[i];
    const int w = (s_ent[i + 1] - s_ent[i]) / kSl;
    for (int l = 0; l < kSl; ++l) {
      const int64_t r = int64_t(s_row[i]) + l;
      for (int t = 0; t < w; ++t) {
        const int64_t e = e0 + int64_t(t) * kSl + l;
        if (r < n && t < rlen[r]) {
          sv[e] = va[rp[r] + t];
          sc[e] = ci[rp[r] + t];
        } else {
          sc[e] = r < n ? static_cast<int32_t>(r) : 0;
        }
      }
    }
  }
  std::vector<uint16_t> sc16;
  std::vector<int32_t> sbase;
  bool have16 = false;
  {
    std::vector<int32_t> ident(ns + 1);
    for (int i = 0; i <= ns; ++i) ident[i] = i;
    have16 = spis::build_col16(s_ent.data(), sc.data(), ident, sc16, sbase);
    sc16.resize(ent + kSlotMax, 0);
  }
  printf("n %lld nnz %lld slices %d entries %lld (pad %.4f) wmax %d order %s\n", (long long)n, (long long)nnz, ns,
         (long long)ent, double(ent) / nnz, wmax, use_slab ? "slab" : "natural");
  int *d_sent, *d_srow;
  uint8_t* d_rlen;
  double* d_sv;
  int32_t* d_sc;
  CK(hipMalloc(&d_sent, 4 * (ns + 1)));
  CK(hipMalloc(&d_srow, 4 * ns));
  CK(hipMalloc(&d_rlen, n));
  CK(hipMalloc(&d_sv, 8 * sv.size()));
  CK(hipMalloc(&d_sc, 4 * sc.size()));
  CK(hipMemcpy(d_sent, s_ent.data(), 4 * (ns + 1), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_srow, s_row.data(), 4 * ns, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_rlen, rlen.data(), n, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_sv, sv.data(), 8 * sv.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_sc, sc.data(), 4 * sc.size(), hipMemcpyHostToDevice));
  uint16_t* d_sc16 = nullptr;
  int4* d_sbase = nullptr;
  if (have16) {
    CK(hipMalloc(&d_sc16, 2 * sc16.size()));
    CK(hipMalloc(&d_sbase, 4 * sbase.size()));
    CK(hipMemcpy(d_sc16, sc16.data(), 2 * sc16.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_sbase, sbase.data(), 4 * sbase.size(), hipMemcpyHostToDevice));
  }
  printf("16-bit columns: %s\n", have16 ? "yes" : "no");
  std::vector<double> hx1(n), hx2(n);
  for (int64_t i = 0; i < n; ++i) {
    hx1[i] = 1e-3 * ((i * 7919) % 1000);
    hx2[i] = 1e-3 * ((i * 104729) % 997) - 0.4;
  }
  double *dx1, *dx2, *db, *dy, *p1, *p2;
  CK(hipMalloc(&dx1, 8 * n));
  CK(hipMalloc(&dx2, 8 * n));
  CK(hipMalloc(&db, 8 * n));
  CK(hipMalloc(&dy, 8 * n));
  CK(hipMalloc(&p1, 8 * 4096));
  CK(hipMalloc(&p2, 8 * 4096));
  CK(hipMemcpy(dx1, hx1.data(), 8 * n, hipMemcpyHostToDevice));
  CK(hipMemcpy(dx2, hx2.data(), 8 * n, hipMemcpyHostToDevice));
  CK(hipMemcpy(db, hx2.data(), 8 * n, hipMemcpyHostToDevice));
  // host reference y = A x2 (left to right, no contraction: the compile line has -ffp-contract=off)
  std::vector<double> yref(n);
  for (int64_t r = 0; r < n; ++r) {
    double a = 0.0;
    for (int32_t i = rp[r]; i < rp[r + 1]; ++i) {
      const double p = va[i] * hx2[ci[i]];
      a += p;
    }
    yref[r] = a;
  }
  const int64_t big = int64_t(1) << 26;
  double2* ev;
  double* evo;
  CK(hipMalloc(&ev, 16 * big));
  CK(hipMalloc(&evo, 8));
  CK(hipMemset(ev, 0, 16 * big));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // algorithmic bytes: the CSR stream (12 nnz + 4 (n + 1)) + gathers and vectors as bench.py counts
  const double bytes_arn = 12.0 * nnz + 4.0 * (n + 1) + 8.0 * n * 3;  // x2 gather, aux2, y2
  const double bytes_dual = 12.0 * nnz + 4.0 * (n + 1) + 8.0 * n * 5;  // + x1 gather, aux1

  auto run = [&](const char* name, int slot, int maxs, int G, auto kern, int threads, bool dual, bool c16) {
    if (c16 && !have16) return;
    Plan p = make_plan(s_ent, slot, maxs, G);
    int4* d_slots;
    int* d_wg;
    CK(hipMalloc(&d_slots, 16 * p.slots.size()));
    CK(hipMalloc(&d_wg, 4 * p.wg_slot.size()));
    CK(hipMemcpy(d_slots, p.slots.data(), 16 * p.slots.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_wg, p.wg_slot.data(), 4 * p.wg_slot.size(), hipMemcpyHostToDevice));
    double fill = 0;
    for (auto& q : p.slots) fill += q.w;
    fill /= double(p.slots.size()) * slot;
    auto launch = [&] {
      hipLaunchKernelGGL(kern, dim3(G), dim3(threads), 0, st, d_slots, d_wg, d_sent, d_srow, d_rlen, d_sv,
                         c16 ? (const void*)d_sc16 : (const void*)d_sc, d_sbase, n, dx1, db, p1, dx2, db, dy, p2);
    };
    CK(hipMemset(dy, 0, 8 * n));
    launch();
    CK(hipStreamSynchronize(st));
    CK(hipGetLastError());
    std::vector<double> y(n);
    CK(hipMemcpy(y.data(), dy, 8 * n, hipMemcpyDeviceToHost));
    int64_t bad = 0;
    for (int64_t i = 0; i < n; ++i) bad += memcmp(&y[i], &yref[i], 8) != 0;
    for (int i = 0; i < 3; ++i) launch();
    CK(hipEventRecord(e0, st));
    const int reps = 20;
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double warm = 1e3 * ms / reps;
    double cold = 0;
    for (int i = 0; i < 10; ++i) {
      hipLaunchKernelGGL(evict_kernel, dim3(4096), dim3(256), 0, st, big, ev, evo);
      CK(hipEventRecord(e0, st));
      launch();
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      cold += 1e3 * ms / 10;
    }
    const double B = (dual ? bytes_dual : bytes_arn) - (c16 ? 2.0 * nnz : 0.0);
    printf("%-34s slot %5d maxs %d G %4d slots %7zu fill %.3f | rows differ %lld | warm %8.2f us %6.0f GB/s | cold %8.2f us %6.0f GB/s\n",
           name, slot, maxs, G, p.slots.size(), fill, (long long)bad, warm, B / warm * 1e-3, cold, B / cold * 1e-3);
    CK(hipFree(d_slots));
    CK(hipFree(d_wg));
  };
#define RUN(MODE, NC, NL, SLOT, MAXS, G, C16)                                                           \
  run("ring mode=" #MODE " nc=" #NC " nl=" #NL " c16=" #C16, SLOT, MAXS, G,                             \
      spmv_ring_kernel<MODE, NC, NL, SLOT, C16>, (NC + NL) * 64, MODE == 1, C16)
  RUN(0, 8, 4, 4096, 8, 256, false);
  RUN(1, 8, 4, 4096, 8, 256, false);
  RUN(0, 4, 4, 2048, 8, 512, false);
  RUN(1, 4, 4, 2048, 8, 512, false);
  RUN(0, 4, 4, 2048, 4, 512, false);
  RUN(1, 4, 4, 2048, 4, 512, false);
  RUN(0, 2, 2, 1024, 8, 1024, false);
  RUN(1, 2, 2, 1024, 8, 1024, false);
  RUN(0, 2, 2, 1024, 2, 1024, false);
  RUN(1, 2, 2, 1024, 2, 1024, false);
  RUN(0, 4, 2, 1024, 4, 1024, false);
  RUN(1, 4, 2, 1024, 4, 1024, false);
  RUN(0, 8, 4, 4096, 8, 256, true);
  RUN(1, 8, 4, 4096, 8, 256, true);
  RUN(0, 4, 4, 2048, 8, 512, true);
  RUN(1, 4, 4, 2048, 8, 512, true);
  RUN(0, 2, 2, 1024, 8, 1024, true);
  RUN(1, 2, 2, 1024, 8, 1024, true);
  return 0;
}
