// kbench.hip — kernel-variant micro-benchmark (tuning tool, not part of libspis).
// Times SpMV and MGS-step variants on the real bench matrix (tools/dump_matrix.py) with HIP
// events, back-to-back launches like the solver issues them.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../structurepreservingiterativesolvers_amd/csrc/kernels.hip"
#include "spmv_variants.hip"
#include "../structurepreservingiterativesolvers_amd/csrc/slab_order.h"
#include "../structurepreservingiterativesolvers_amd/csrc/col16.h"

using namespace spis;

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

template <typename T>
std::vector<T> load(const std::string& p, size_t n) {
  std::vector<T> v(n);
  FILE* f = fopen(p.c_str(), "rb");
  if (!f || fread(v.data(), sizeof(T), n, f) != n) {
    fprintf(stderr, "cannot read %s\n", p.c_str());
    exit(1);
  }
  fclose(f);
  return v;
}

static void blocks(int64_t n, const int32_t* rp, int item_cap, int row_cap, int nnz_cap, std::vector<int32_t>& blk) {
  blk.clear();
  blk.push_back(0);
  int64_t rows = 0, nnz = 0;
  for (int64_t r = 0; r < n; ++r) {
    const int64_t len = rp[r + 1] - rp[r];
    if (rows > 0 && (rows + 1 > row_cap || nnz + len > nnz_cap || rows + 1 + nnz + len > item_cap)) {
      blk.push_back(static_cast<int32_t>(r));
      rows = nnz = 0;
    }
    ++rows;
    nnz += len;
  }
  blk.push_back(static_cast<int32_t>(n));
}

// ---- SpMV variant: all val/col loads of the block issued first (fixed trip count) ------------
// SWZ 0: blk = blockIdx (grid-stride); 1: XCD-swizzled logical id (grid-stride); 2: swizzled id,
// contiguous chunk of row blocks per workgroup.  NT: nontemporal val/col loads.
template <int EPI, int PER, int SWZ = 0, bool NT = false>
__global__ __launch_bounds__(kBlock) void spmv_v1(const int32_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                                  const double* __restrict__ va, const int32_t* __restrict__ blk_row,
                                                  int n_blk, const double* __restrict__ x, double* __restrict__ y,
                                                  const double* __restrict__ aux, double* __restrict__ partials) {
  __shared__ double s_prod[kBlock * PER];
  __shared__ double s_wave[4];
  double part = 0.0;
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
    int cols[PER];
    double vals[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int i = threadIdx.x + u * kBlock;
      if (NT) {
        cols[u] = i < nnz ? __builtin_nontemporal_load(ci + nz0 + i) : 0;
        vals[u] = i < nnz ? __builtin_nontemporal_load(va + nz0 + i) : 0.0;
      } else {
        cols[u] = i < nnz ? ci[nz0 + i] : 0;
        vals[u] = i < nnz ? va[nz0 + i] : 0.0;
      }
    }
    double xs[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) xs[u] = x[cols[u]];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
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
      if (EPI == kEpiDot) {
        y[r] = sum;
        part += aux[r] * sum;
      } else {
        y[r] = sum;
      }
    }
    __syncthreads();
  }
  if (EPI != kEpiPlain) {
    const double tot = block_sum(part, s_wave);
    if (threadIdx.x == 0) partials[blockIdx.x] = tot;
  }
}

// ---- dual SpMV with x1/x2 interleaved (one 16-B gather per nonzero) ------------------------------
template <int CAP>
__global__ __launch_bounds__(kBlock) void spmv_dual_il(const int32_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                                       const double* __restrict__ va, const int32_t* __restrict__ blk_row,
                                                       int n_blk, const double2* __restrict__ xz,
                                                       const double* __restrict__ b, double* __restrict__ part1,
                                                       double* __restrict__ w, const double* __restrict__ q0,
                                                       double* __restrict__ part2) {
  __shared__ double2 s_p[CAP];
  __shared__ double s_wave[4];
  double pt1 = 0.0, pt2 = 0.0;
  for (int blk = blockIdx.x; blk < n_blk; blk += gridDim.x) {
    const int r0 = blk_row[blk];
    const int r1 = blk_row[blk + 1];
    const int nz0 = rp[r0];
    const int nnz = rp[r1] - nz0;
    constexpr int kPer = CAP / kBlock;
    int cols[kPer];
    double vals[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int i = threadIdx.x + u * kBlock;
      cols[u] = i < nnz ? ci[nz0 + i] : 0;
      vals[u] = i < nnz ? va[nz0 + i] : 0.0;
    }
    double2 g[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) g[u] = xz[cols[u]];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int i = threadIdx.x + u * kBlock;
      if (i < nnz) s_p[i] = make_double2(vals[u] * g[u].x, vals[u] * g[u].y);
    }
    __syncthreads();
    const int r = r0 + threadIdx.x;
    if (r < r1) {
      const int s0 = rp[r] - nz0;
      const int e = rp[r + 1] - nz0;
      double s1 = 0.0, s2 = 0.0;
      for (int t = s0; t < e; ++t) {
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

// ---- MGS variant: PER pairs per thread, all loads first ---------------------------------------
template <int PER>
__global__ __launch_bounds__(kBlock) void mgs_v1(int64_t n, double* __restrict__ y, const double* __restrict__ qi,
                                                 const double* __restrict__ qn, const double* __restrict__ part_in,
                                                 int n_in, double* __restrict__ part_out, double* __restrict__ h_out) {
#pragma clang fp contract(off)
  __shared__ double s_wave[4];
  const int64_t npair = n >> 1;
  double2* y2 = reinterpret_cast<double2*>(y);
  const double2* q2 = reinterpret_cast<const double2*>(qi);
  const double2* n2 = reinterpret_cast<const double2*>(qn);
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kBlock * PER + threadIdx.x;
  double2 yv[PER], qv[PER], nv[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int64_t p = base + u * kBlock;
    if (p < npair) {
      qv[u] = q2[p];
      yv[u] = y2[p];
      nv[u] = n2[p];
    }
  }
  const double h = sum_partials(part_in, n_in, s_wave);
  if (blockIdx.x == 0 && threadIdx.x == 0) *h_out = h;
  double part = 0.0;
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int64_t p = base + u * kBlock;
    if (p < npair) {
      const double a0 = h * qv[u].x, a1 = h * qv[u].y;
      yv[u].x = yv[u].x - a0;
      yv[u].y = yv[u].y - a1;
      y2[p] = yv[u];
      part += nv[u].x * yv[u].x;
      part += nv[u].y * yv[u].y;
    }
  }
  const double tot = block_sum(part, s_wave);
  if (threadIdx.x == 0) part_out[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kBlock) void copy2_kernel(int64_t m, const double2* __restrict__ x, double2* __restrict__ y) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < m; i += static_cast<int64_t>(gridDim.x) * kBlock)
    y[i] = x[i];
}
__global__ __launch_bounds__(kBlock) void read2_kernel(int64_t m, const double2* __restrict__ x, double* __restrict__ out) {
  double a = 0.0;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < m; i += static_cast<int64_t>(gridDim.x) * kBlock) {
    const double2 v = x[i];
    a += v.x + v.y;
  }
  if (a == 12345.678) out[0] = a;
}

// calibration streams for PMC byte counters: known bytes, fixed access width per lane
__global__ __launch_bounds__(kBlock) void calib_read8(int64_t m, const double* __restrict__ x, double* __restrict__ out) {
  double a = 0.0;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < m; i += static_cast<int64_t>(gridDim.x) * kBlock)
    a += x[i];
  if (a == 12345.678) out[0] = a;
}
__global__ __launch_bounds__(kBlock) void calib_read4(int64_t m, const int32_t* __restrict__ x, double* __restrict__ out) {
  int64_t a = 0;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < m; i += static_cast<int64_t>(gridDim.x) * kBlock)
    a += x[i];
  if (a == 1234567) out[0] = 1.0;
}
__global__ __launch_bounds__(kBlock) void calib_write8(int64_t m, double* __restrict__ y) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < m; i += static_cast<int64_t>(gridDim.x) * kBlock)
    y[i] = 1.0;
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp/kbench_mat";
  auto shp = load<int64_t>(dir + "/shape.bin", 2);
  const int64_t n = shp[0], nnz = shp[1];
  auto rp = load<int32_t>(dir + "/indptr.bin", n + 1);
  auto ci = load<int32_t>(dir + "/indices.bin", nnz);
  auto va = load<double>(dir + "/data.bin", nnz);
  int32_t *drp, *dci, *dblk;
  double *dva, *dx, *dy, *dpart, *dpart2, *dh;
  CK(hipMalloc(&drp, 4 * (n + 1)));
  CK(hipMalloc(&dci, 4 * nnz));
  CK(hipMalloc(&dva, 8 * nnz));
  CK(hipMemcpy(drp, rp.data(), 4 * (n + 1), hipMemcpyHostToDevice));
  CK(hipMemcpy(dci, ci.data(), 4 * nnz, hipMemcpyHostToDevice));
  CK(hipMemcpy(dva, va.data(), 8 * nnz, hipMemcpyHostToDevice));
  const int64_t pitch = (n + 63) / 64 * 64;
  const int K = 31;
  double* dQ;
  CK(hipMalloc(&dQ, 8 * pitch * K));
  CK(hipMalloc(&dx, 8 * pitch));
  CK(hipMalloc(&dy, 8 * pitch));
  CK(hipMalloc(&dpart, 8 * 8192));
  CK(hipMalloc(&dpart2, 8 * 8192));
  CK(hipMalloc(&dh, 8 * 64));
  std::vector<double> hx(pitch);
  for (int64_t i = 0; i < pitch; ++i) hx[i] = i < n ? 1e-3 * ((i * 7919) % 1000) : 0.0;
  for (int k = 0; k < K; ++k) CK(hipMemcpy(dQ + k * pitch, hx.data(), 8 * pitch, hipMemcpyHostToDevice));
  CK(hipMemcpy(dx, hx.data(), 8 * pitch, hipMemcpyHostToDevice));
  CK(hipMemset(dpart, 0, 8 * 8192));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double S = 12.0 * nnz + 4.0 * (n + 1) + 16.0 * n;
  if (argc > 2 && std::string(argv[2]) == "sig") {
    // cost of host-visible completion signals between dependent kernels: 100 x (copy 8 MB)
    const int64_t m = (n / 2) & ~int64_t(1);
    auto k = [&](const LaunchEv* ev) {
      launch_k(copy2_kernel, dim3(2048), dim3(kBlock), 0, s, ev, m / 2, reinterpret_cast<const double2*>(dx),
               reinterpret_cast<double2*>(dy));
    };
    hipEvent_t evd, evs, evn, evt;
    CK(hipEventCreateWithFlags(&evd, hipEventDisableTiming | hipEventReleaseToDevice));
    CK(hipEventCreateWithFlags(&evs, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&evn, hipEventDisableTiming | hipEventDisableSystemFence));
    CK(hipEventCreate(&evt));
    uint64_t* flag;
    CK(hipHostMalloc(reinterpret_cast<void**>(&flag), 64, hipHostMallocMapped | hipHostMallocCoherent));
    void* flag_dev;
    CK(hipHostGetDevicePointer(&flag_dev, flag, 0));
    auto run = [&](const char* name, int mode) {
      for (int w = 0; w < 2; ++w) {
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < 100; ++i) {
          LaunchEv le;
          if (mode == 4) le.stop = evd;
          if (mode == 5) le.stop = evs;
          if (mode == 6) le.stop = evn;
          if (mode == 7) le.stop = evt;
          k(mode >= 4 && mode <= 7 ? &le : nullptr);
          if (mode == 1) CK(hipEventRecord(evd, s));
          if (mode == 2) CK(hipEventRecord(evs, s));
          if (mode == 3) CK(hipEventRecord(evn, s));
          if (mode == 8) CK(hipStreamWriteValue64(s, flag_dev, i + 1, 0));
        }
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (w == 1) printf("%-52s %8.2f us per kernel\n", name, 1e3 * ms / 100);
      }
    };
    {  // host-side enqueue cost of back-to-back MGS-step launches (GPU kept busy by a long copy)
      double* big;
      const int64_t mb = int64_t(1) << 27;
      CK(hipMalloc(&big, 16 * mb));
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipStreamSynchronize(s));
        hipLaunchKernelGGL(copy2_kernel, dim3(4096), dim3(kBlock), 0, s, mb / 2, reinterpret_cast<const double2*>(big),
                           reinterpret_cast<double2*>(big + mb));  // ~0.5 ms of GPU work queued first
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < 60; ++i)
          (void)launch_mgs_step(n, dy, dQ, dQ + pitch, dpart, 1024, dpart2, dh, 490, s);
        const auto t1 = std::chrono::steady_clock::now();
        CK(hipStreamSynchronize(s));
        if (rep == 1)
          printf("host enqueue, launch_mgs_step: %.2f us per launch\n",
                 std::chrono::duration<double, std::micro>(t1 - t0).count() / 60);
      }
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipStreamSynchronize(s));
        hipLaunchKernelGGL(copy2_kernel, dim3(4096), dim3(kBlock), 0, s, mb / 2, reinterpret_cast<const double2*>(big),
                           reinterpret_cast<double2*>(big + mb));
        LaunchEv le;
        le.stop = evt;
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < 60; ++i)
          (void)launch_mgs_step(n, dy, dQ, dQ + pitch, dpart, 1024, dpart2, dh, 490, s, &le);
        const auto t1 = std::chrono::steady_clock::now();
        CK(hipStreamSynchronize(s));
        if (rep == 1)
          printf("host enqueue, ext launch + stop event: %.2f us per launch\n",
                 std::chrono::duration<double, std::micro>(t1 - t0).count() / 60);
      }
      CK(hipFree(big));
    }
    {  // 30-step MGS chain: eager launches vs one captured graph (host enqueue + GPU time)
      auto chain = [&]() {
        for (int i = 0; i < 30; ++i)
          (void)launch_mgs_step(n, dy, dQ + i * pitch, dQ + (i + 1) * pitch, (i & 1) ? dpart2 : dpart, 490,
                                (i & 1) ? dpart : dpart2, dh + i, 490, s);
      };
      hipGraph_t gr;
      hipGraphExec_t ge;
      CK(hipStreamSynchronize(s));
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      chain();
      CK(hipStreamEndCapture(s, &gr));
      CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
      for (int mode = 0; mode < 2; ++mode) {
        double host = 0.0;
        float gpu = 0.f;
        for (int rep = 0; rep < 6; ++rep) {
          CK(hipStreamSynchronize(s));
          CK(hipEventRecord(e0, s));
          const auto t0 = std::chrono::steady_clock::now();
          if (mode == 0) chain();
          else CK(hipGraphLaunch(ge, s));
          const auto t1 = std::chrono::steady_clock::now();
          CK(hipEventRecord(e1, s));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          if (rep >= 2) {
            host += std::chrono::duration<double, std::micro>(t1 - t0).count();
            gpu += ms;
          }
        }
        printf("MGS chain x30 %-6s: host enqueue %7.1f us, GPU %7.1f us\n", mode == 0 ? "eager" : "graph", host / 4,
               1e3 * gpu / 4);
      }
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(gr));
    }
    {  // graph boundary cost: 20 replays of a 5-step MGS graph vs 100 eager steps (GPU time)
      auto chain5 = [&]() {
        for (int i = 0; i < 5; ++i)
          (void)launch_mgs_step(n, dy, dQ + i * pitch, dQ + (i + 1) * pitch, (i & 1) ? dpart2 : dpart, 490,
                                (i & 1) ? dpart : dpart2, dh + i, 490, s);
      };
      hipGraph_t gr;
      hipGraphExec_t ge;
      CK(hipStreamSynchronize(s));
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      chain5();
      CK(hipStreamEndCapture(s, &gr));
      CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
      for (int mode = 0; mode < 3; ++mode) {
        float best = 1e30f;
        for (int rep = 0; rep < 4; ++rep) {
          CK(hipStreamSynchronize(s));
          CK(hipEventRecord(e0, s));
          for (int g = 0; g < 20; ++g) {
            if (mode == 0) chain5();
            if (mode == 1) CK(hipGraphLaunch(ge, s));
            if (mode == 2) {  // graph + one eager kernel between replays
              CK(hipGraphLaunch(ge, s));
              (void)launch_mgs_step(n, dy, dQ, dQ + pitch, dpart, 490, dpart2, dh, 490, s);
            }
          }
          CK(hipEventRecord(e1, s));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          best = ms < best ? ms : best;
        }
        const int steps = mode == 2 ? 120 : 100;
        printf("MGS steps %-22s: %6.2f us per step\n", mode == 0 ? "eager" : mode == 1 ? "20 x graph(5)" : "graph(5) + eager",
               1e3 * best / steps);
      }
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(gr));
    }
    {  // MGS chain writing h to device memory vs to mapped pinned host memory (as the solver does)
      double* hp;
      CK(hipHostMalloc(reinterpret_cast<void**>(&hp), 8 * 64, hipHostMallocMapped | hipHostMallocCoherent));
      double* hpd;
      CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hpd), hp, 0));
      for (int mode = 0; mode < 2; ++mode) {
        double* hh = mode == 0 ? dh : hpd;
        float best = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
          CK(hipStreamSynchronize(s));
          CK(hipEventRecord(e0, s));
          for (int i = 0; i < 30; ++i)
            (void)launch_mgs_step(n, dy, dQ + i * pitch, dQ + (i + 1) * pitch, (i & 1) ? dpart2 : dpart, 490,
                                  (i & 1) ? dpart : dpart2, hh + i, 490, s);
          CK(hipEventRecord(e1, s));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          best = ms < best ? ms : best;
        }
        printf("MGS chain x30, h to %-12s: %6.2f us per step\n", mode == 0 ? "device" : "pinned host", 1e3 * best / 30);
      }
    }
    run("copy 8 MB, no signal", 0);
    run("copy + marker event (device-scope release)", 1);
    run("copy + marker event (system-scope release)", 2);
    run("copy + marker event (no fence)", 3);
    run("copy with ext stop event (device-scope flags)", 4);
    run("copy with ext stop event (system-scope flags)", 5);
    run("copy with ext stop event (no fence flags)", 6);
    run("copy with ext stop event (timing event)", 7);
    run("copy + hipStreamWriteValue64 to host", 8);
    return 0;
  }
  if (argc > 2 && std::string(argv[2]) == "gap") {
    // kernel-boundary gaps around the persistent MGS chain (read them from a rocprofv3 kernel
    // trace): 20 x [chain(j=15) -> gemv(p=16)], 20 x [chain -> copy], 20 x [copy -> gemv]
    unsigned long long* gran;
    unsigned *ep, *err;
    CK(hipMalloc(&gran, 8 * (4 * kChainMaxWG + 8)));
    CK(hipMemset(gran, 0, 8 * (4 * kChainMaxWG + 8)));
    CK(hipMalloc(&ep, 16));
    CK(hipMemset(ep, 0, 16));
    CK(hipMalloc(&err, 16));
    CK(hipMemset(err, 0, 16));
    double* dhost;
    CK(hipHostMalloc(reinterpret_cast<void**>(&dhost), 8 * 64, hipHostMallocMapped));
    double* dhost_dev;
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dhost_dev), dhost, 0));
    std::vector<double> y(16, 0.01);
    const int64_t m = (n / 2);
    auto chain = [&](double* hc) {
      CK(launch_mgs_chain(n, dy, dQ, pitch, 15, dpart, 1024, hc, gran, ep, err, s, nullptr, nullptr, 0, nullptr,
                          nullptr, nullptr));
    };
    auto gemv = [&] { CK(launch_gemv(n, 16, dQ, pitch, y.data(), true, dx, dy, s, nullptr)); };
    auto copy = [&] {
      hipLaunchKernelGGL(copy2_kernel, dim3(2048), dim3(kBlock), 0, s, m, reinterpret_cast<const double2*>(dx),
                         reinterpret_cast<double2*>(dy));
    };
    for (int r = 0; r < 20; ++r) { chain(dhost_dev); gemv(); }
    for (int r = 0; r < 20; ++r) { chain(dhost_dev); copy(); }
    for (int r = 0; r < 20; ++r) { chain(dh); copy(); }  // H column in device memory
    for (int r = 0; r < 20; ++r) { copy(); gemv(); }
    CK(hipStreamSynchronize(s));
    printf("gap mode done\n");
    return 0;
  }
  if (argc > 2 && std::string(argv[2]) == "pmc") {
    // PMC mode: 3 calibration streams of 1 GiB each (known bytes), then 5 Arnoldi SpMVs
    const int64_t m8 = int64_t(1) << 27;
    double* big;
    CK(hipMalloc(&big, 8 * m8));
    CK(hipMemset(big, 0, 8 * m8));
    hipLaunchKernelGGL(calib_read8, dim3(4096), dim3(kBlock), 0, s, m8, big, dpart);
    hipLaunchKernelGGL(calib_read4, dim3(4096), dim3(kBlock), 0, s, 2 * m8, reinterpret_cast<const int32_t*>(big), dpart);
    hipLaunchKernelGGL(calib_write8, dim3(4096), dim3(kBlock), 0, s, m8, big);
    CK(hipStreamSynchronize(s));
    std::vector<int32_t> blk;
    blocks(n, rp.data(), 2048, 256, 2048, blk);
    CK(hipMalloc(&dblk, 4 * blk.size()));
    CK(hipMemcpy(dblk, blk.data(), 4 * blk.size(), hipMemcpyHostToDevice));
    CsrView A{n, drp, dci, dva, dblk, static_cast<int>(blk.size()) - 1};
    const int g = A.n_blk < 2048 ? A.n_blk : 2048;
    for (int i = 0; i < 5; ++i) CK(launch_spmv(A, kEpiDot, dx, dy, dQ, dpart, g, s));
    const int nb = A.n_blk;
    {  // the solver's fused residual + Arnoldi SpMV on its kDualCap row blocks
      std::vector<int32_t> blkd;
      blocks(n, rp.data(), kDualCap, 256, kDualCap, blkd);
      int32_t* dblkd;
      CK(hipMalloc(&dblkd, 4 * blkd.size()));
      CK(hipMemcpy(dblkd, blkd.data(), 4 * blkd.size(), hipMemcpyHostToDevice));
      CsrView Ad{n, drp, dci, dva, dblkd, static_cast<int>(blkd.size()) - 1};
      double *dx2, *dw, *dpr;
      CK(hipMalloc(&dx2, 8 * pitch));
      CK(hipMalloc(&dw, 8 * pitch));
      CK(hipMalloc(&dpr, 8 * 8192));
      CK(hipMemcpy(dx2, hx.data(), 8 * pitch, hipMemcpyHostToDevice));
      for (int i = 0; i < 5; ++i) CK(launch_spmv_dual(Ad, dx, dy, dpr, dx2, dw, dQ, dpart, g, s));
      const int nbd = Ad.n_blk;
      const int gd = nbd < 2048 ? nbd : 2048;
      for (int i = 0; i < 5; ++i)
        hipLaunchKernelGGL((spmv_dual_kernel<1024, 1>), dim3(gd), dim3(kBlock), 0, s, drp, dci, dva, dblkd, nbd, dx, dy,
                           dpr, dx2, dw, dQ, dpart);
      for (int i = 0; i < 5; ++i)
        hipLaunchKernelGGL((spmv_dual_kernel<1024, 2>), dim3(gd), dim3(kBlock), 0, s, drp, dci, dva, dblkd, nbd, dx, dy,
                           dpr, dx2, dw, dQ, dpart);
      CK(hipStreamSynchronize(s));
      // the solver's pipelined dual (XCD-local walk, 1280 workgroups): 5 back to back ("warm"),
      // then 5 each behind 1 GiB of reads that evict L2 and the Infinity Cache ("cold")
      std::vector<int2> meta(blkd.size());
      for (size_t i = 0; i < blkd.size(); ++i) meta[i] = make_int2(blkd[i], rp[blkd[i]]);
      int2* dmeta;
      CK(hipMalloc(&dmeta, 8 * meta.size()));
      CK(hipMemcpy(dmeta, meta.data(), 8 * meta.size(), hipMemcpyHostToDevice));
      const int64_t big = int64_t(1) << 27;
      double* bx;
      CK(hipMalloc(&bx, 8 * big));
      CK(hipMemset(bx, 0, 8 * big));
      for (int i = 0; i < 10; ++i) {
        if (i >= 5)
          hipLaunchKernelGGL(read2_kernel, dim3(4096), dim3(kBlock), 0, s, big / 2, reinterpret_cast<const double2*>(bx),
                             dpr + 4096);
        hipLaunchKernelGGL((spmv_pipe_var_kernel<1024, 4, false, 1>), dim3(1280), dim3(kBlock), 0, s, drp, dci, dva, dmeta,
                           nbd, 1, dx, dy, (double*)nullptr, dpr, dx2, dQ, dw, dpart, (const uint16_t*)nullptr, (const int4*)nullptr);
      }
      // the same on the solver's default table (kPipeCap = 2048-nnz blocks, resident grid): 5 warm,
      // then 5 cold
      std::vector<int2> meta2(blk.size());
      for (size_t i = 0; i < blk.size(); ++i) meta2[i] = make_int2(blk[i], rp[blk[i]]);
      int2* dmeta2;
      CK(hipMalloc(&dmeta2, 8 * meta2.size()));
      CK(hipMemcpy(dmeta2, meta2.data(), 8 * meta2.size(), hipMemcpyHostToDevice));
      const int g2 = resident_grid(spmv_pipe_var_kernel<kPipeCap, 4>);
      printf("pmc mode: kPipeCap dual on %d blocks, grid %d\n", nb, g2);
      for (int i = 0; i < 10; ++i) {
        if (i >= 5)
          hipLaunchKernelGGL(read2_kernel, dim3(4096), dim3(kBlock), 0, s, big / 2, reinterpret_cast<const double2*>(bx),
                             dpr + 4096);
        hipLaunchKernelGGL((spmv_pipe_var_kernel<kPipeCap, 4>), dim3(g2), dim3(kBlock), 0, s, drp, dci, dva, dmeta2, nb, 1, dx,
                           dy, (double*)nullptr, dpr, dx2, dQ, dw, dpart, (const uint16_t*)nullptr, (const int4*)nullptr);
      }
      // and on the solver's default order (slab-ordered (start, end) pairs, walk 2): 5 warm, 5 cold
      std::vector<int32_t> pairs;
      if (build_slab_order(n, rp.data(), ci.data(), blk, pairs)) {
        int2* dpairs;
        CK(hipMalloc(&dpairs, 4 * pairs.size()));
        CK(hipMemcpy(dpairs, pairs.data(), 4 * pairs.size(), hipMemcpyHostToDevice));
        printf("pmc mode: slab-ordered dual on %d blocks\n", nb);
        for (int i = 0; i < 10; ++i) {
          if (i >= 5)
            hipLaunchKernelGGL(read2_kernel, dim3(4096), dim3(kBlock), 0, s, big / 2,
                               reinterpret_cast<const double2*>(bx), dpr + 4096);
          hipLaunchKernelGGL((spmv_pipe_var_kernel<kPipeCap, 4>), dim3(g2), dim3(kBlock), 0, s, drp, dci, dva,
                             dpairs, nb, 2, dx, dy, (double*)nullptr, dpr, dx2, dQ, dw, dpart, (const uint16_t*)nullptr, (const int4*)nullptr);
        }
      }
      CK(hipStreamSynchronize(s));
      CK(hipFree(bx));
    }
    for (int i = 0; i < 5; ++i)
      hipLaunchKernelGGL((spmv_v1<kEpiDot, 8, 1, false>), dim3(g), dim3(kBlock), 0, s, drp, dci, dva, dblk, nb, dx, dy, dQ, dpart);
    for (int i = 0; i < 5; ++i)
      hipLaunchKernelGGL((spmv_v1<kEpiDot, 8, 2, false>), dim3(g), dim3(kBlock), 0, s, drp, dci, dva, dblk, nb, dx, dy, dQ, dpart);
    for (int i = 0; i < 5; ++i)
      hipLaunchKernelGGL((spmv_v1<kEpiDot, 8, 1, true>), dim3(g), dim3(kBlock), 0, s, drp, dci, dva, dblk, nb, dx, dy, dQ, dpart);
    CK(hipStreamSynchronize(s));
    printf("pmc mode: calib 1 GiB read8 / read4 / write8, then 5 x spmv (S = %.1f MB)\n", S / 1e6);
    return 0;
  }
  auto timeit = [&](const char* name, int reps, double bytes, auto&& fn) {
    for (int i = 0; i < 3; ++i) fn();
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < reps; ++i) fn();
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1e3 * ms / reps;
    printf("%-44s %8.2f us  %7.0f GB/s  (%.0f%% of 8 TB/s)\n", name, us, bytes / (us * 1e-6) / 1e9,
           100.0 * bytes / (us * 1e-6) / 8e12);
  };
  if (argc > 2 && std::string(argv[2]) == "cap4k") {
    // the dual on 2,048- vs 4,096-nnz row blocks (<= 256 rows each), both in slab order with the
    // slab key, 32-bit columns, resident grids; warm and cold; rows compared
    double *dx2, *dw, *dw2, *db, *pa, *pb;
    CK(hipMalloc(&dx2, 8 * pitch));
    CK(hipMalloc(&dw, 8 * pitch));
    CK(hipMalloc(&dw2, 8 * pitch));
    CK(hipMalloc(&db, 8 * pitch));
    CK(hipMalloc(&pa, 8 * 16384));
    CK(hipMalloc(&pb, 8 * 16384));
    std::vector<double> h2(pitch);
    for (int64_t i = 0; i < pitch; ++i) h2[i] = i < n ? 1e-3 * ((i * 104729) % 997) - 0.4 : 0.0;
    CK(hipMemcpy(dx2, h2.data(), 8 * pitch, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, h2.data(), 8 * pitch, hipMemcpyHostToDevice));
    const double SD = 12.0 * nnz + 4.0 * (n + 1) + 32.0 * n;
    std::vector<uint8_t> lab;
    std::vector<double> key;
    if (!slab_labels(n, rp.data(), ci.data(), lab, &key)) return 1;
    auto table = [&](int cap, int& nb_out) {
      std::vector<int32_t> blk, pairs;
      blocks(n, rp.data(), cap + 256, 256, cap, blk);
      nb_out = static_cast<int>(blk.size()) - 1;
      if (!build_slab_order(rp.data(), lab, blk, pairs, nullptr, &key)) {
        printf("no slab order\n");
        exit(1);
      }
      int2* d;
      CK(hipMalloc(&d, 4 * pairs.size()));
      CK(hipMemcpy(d, pairs.data(), 4 * pairs.size(), hipMemcpyHostToDevice));
      return d;
    };
    int nb2 = 0, nb4 = 0;
    int2* t2 = table(2048, nb2);
    int2* t4 = table(4096, nb4);
    const int64_t big = int64_t(1) << 26;
    double* bx;
    CK(hipMalloc(&bx, 8 * big));
    CK(hipMemset(bx, 0, 8 * big));
    const int g2 = resident_grid(spmv_pipe_var_kernel<2048, 4>);
    const int g4 = resident_grid(spmv_pipe_var_kernel<4096, 4, false, 2>);
    printf("blocks %d / %d, resident grids %d / %d\n", nb2, nb4, g2, g4);
    auto run = [&](const char* name, auto&& launch) {
      for (int cold = 0; cold < 2; ++cold) {
        double tot = 0;
        const int reps = 20;
        for (int r = 0; r < reps + 3; ++r) {
          if (cold) hipLaunchKernelGGL(read2_kernel, dim3(4096), dim3(kBlock), 0, s, big / 2,
                                       reinterpret_cast<const double2*>(bx), pb + 8192);
          launch();
          CK(hipEventSynchronize(e1));
          float ms_;
          CK(hipEventElapsedTime(&ms_, e0, e1));
          if (r >= 3) tot += ms_;
        }
        const double us = 1e3 * tot / reps;
        printf("%s %-36s %8.2f us  %7.0f GB/s  (%.3f of 8 TB/s)\n", cold ? "COLD" : "WARM", name, us,
               SD / (us * 1e-6) / 1e9, SD / (us * 1e-6) / 8e12);
        fflush(stdout);
      }
    };
    char nm[96];
    for (int g : {g2, g2 * 4 / 3 / 8 * 8}) {
      snprintf(nm, sizeof nm, "cap 2048 grid %d", g);
      run(nm, [&] {
        hipExtLaunchKernelGGL((spmv_pipe_var_kernel<2048, 4>), dim3(g), dim3(kBlock), 0, s, e0, e1, 0, drp, dci, dva, t2,
                              nb2, 2, dx, db, (double*)nullptr, pa, dx2, dQ, dw, pb, (const uint16_t*)nullptr,
                              (const int4*)nullptr);
      });
    }
    for (int g : {g4, 512}) {
      snprintf(nm, sizeof nm, "cap 4096 WPE2 grid %d", g);
      run(nm, [&] {
        hipExtLaunchKernelGGL((spmv_pipe_var_kernel<4096, 4, false, 2>), dim3(g), dim3(kBlock), 0, s, e0, e1, 0, drp, dci,
                              dva, t4, nb4, 2, dx, db, (double*)nullptr, pa, dx2, dQ, dw2, pb,
                              (const uint16_t*)nullptr, (const int4*)nullptr);
      });
      snprintf(nm, sizeof nm, "cap 4096 WPE2 BUF grid %d", g);
      run(nm, [&] {
        hipExtLaunchKernelGGL((spmv_pipe_var_kernel<4096, 4, false, 2, false, true>), dim3(g), dim3(kBlock), 0, s, e0, e1,
                              0, drp, dci, dva, t4, nb4, 2, dx, db, (double*)nullptr, pa, dx2, dQ, dw2, pb,
                              (const uint16_t*)nullptr, (const int4*)nullptr);
      });
    }
    std::vector<double> w1(n), w2(n);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(w1.data(), dw, 8 * n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(w2.data(), dw2, 8 * n, hipMemcpyDeviceToHost));
    int64_t bad = 0;
    for (int64_t i = 0; i < n; ++i) bad += w1[i] != w2[i];
    printf("cap 4096 vs 2048, dual rows: %lld differ\n", (long long)bad);
    return 0;
  }
  if (argc > 2 && std::string(argv[2]) == "win") {
    // K1w (windowed gathers, spmv_variants.hip spmv_win_kernel) against K1dp, both on slab-ordered
    // tables (K1w's split by windows of <= kWinChunks 64-column chunks), warm and cold; dual rows
    // bitwise against K1dp
    double *dx2, *dw, *db, *pa, *pb;
    CK(hipMalloc(&dx2, 8 * pitch));
    CK(hipMalloc(&dw, 8 * pitch));
    CK(hipMalloc(&db, 8 * pitch));
    CK(hipMalloc(&pa, 8 * 16384));
    CK(hipMalloc(&pb, 8 * 16384));
    std::vector<double> h2(pitch);
    for (int64_t i = 0; i < pitch; ++i) h2[i] = i < n ? 1e-3 * ((i * 104729) % 997) - 0.4 : 0.0;
    CK(hipMemcpy(dx2, h2.data(), 8 * pitch, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, h2.data(), 8 * pitch, hipMemcpyHostToDevice));
    const double SD = 12.0 * nnz + 4.0 * (n + 1) + 32.0 * n;
    const double SW = 10.0 * nnz + 4.0 * (n + 1) + 32.0 * n;  // K1w: 16-bit window positions
    std::vector<int32_t> blk, pairs, bw, pw;
    blocks(n, rp.data(), kPipeCap, 256, kPipeCap, blk);
    std::vector<uint8_t> lab;
    std::vector<double> key;
    std::vector<int64_t> order, ow;
    if (!slab_labels(n, rp.data(), ci.data(), lab, &key) || !build_slab_order(rp.data(), lab, blk, pairs, &order, &key)) {
      printf("no slab order\n");
      return 1;
    }
    bw = blk;
    const auto tb = std::chrono::steady_clock::now();
    if (!win_split_blocks(rp.data(), ci.data(), bw) || !build_slab_order(rp.data(), lab, bw, pw, &ow, &key)) {
      printf("no window table\n");
      return 1;
    }
    std::vector<int32_t> chunks;
    std::vector<uint16_t> lidx;
    win_build(rp.data(), ci.data(), bw, ow, chunks, lidx);
    const double tbuild = std::chrono::duration<double>(std::chrono::steady_clock::now() - tb).count();
    const int nb = static_cast<int>(blk.size()) - 1, nbw = static_cast<int>(bw.size()) - 1;
    int2 *ms, *msw;
    int32_t* dch;
    uint16_t* dli;
    CK(hipMalloc(&ms, 4 * pairs.size()));
    CK(hipMemcpy(ms, pairs.data(), 4 * pairs.size(), hipMemcpyHostToDevice));
    CK(hipMalloc(&msw, 4 * pw.size()));
    CK(hipMemcpy(msw, pw.data(), 4 * pw.size(), hipMemcpyHostToDevice));
    CK(hipMalloc(&dch, 4 * chunks.size()));
    CK(hipMemcpy(dch, chunks.data(), 4 * chunks.size(), hipMemcpyHostToDevice));
    CK(hipMalloc(&dli, 2 * lidx.size()));
    CK(hipMemcpy(dli, lidx.data(), 2 * lidx.size(), hipMemcpyHostToDevice));
    const int64_t big = int64_t(1) << 26;
    double* bx;
    CK(hipMalloc(&bx, 8 * big));
    CK(hipMemset(bx, 0, 8 * big));
    const int gr = resident_grid(spmv_pipe_var_kernel<kPipeCap, 4>);
    const int gw = resident_grid(spmv_win_kernel<kPipeCap, 4>);
    printf("blocks %d (K1w %d after the window split, table built in %.2f s), resident grid %d / K1w %d\n", nb, nbw,
           tbuild, gr, gw);
    auto run = [&](const char* name, double bytes, auto&& launch) {
      for (int cold = 0; cold < 2; ++cold) {
        double tot = 0;
        const int reps = 30;
        for (int r = 0; r < reps + 3; ++r) {
          if (cold) hipLaunchKernelGGL(read2_kernel, dim3(4096), dim3(kBlock), 0, s, big / 2,
                                       reinterpret_cast<const double2*>(bx), pb + 8192);
          launch();
          CK(hipEventSynchronize(e1));
          float ms_;
          CK(hipEventElapsedTime(&ms_, e0, e1));
          if (r >= 3) tot += ms_;
        }
        const double us = 1e3 * tot / reps;
        printf("%s %-40s %8.2f us  %7.0f GB/s  (%.3f of 8 TB/s; K1dp bytes %.3f)\n", cold ? "COLD" : "WARM", name, us,
               bytes / (us * 1e-6) / 1e9, bytes / (us * 1e-6) / 8e12, SD / (us * 1e-6) / 8e12);
      }
    };
    auto k1dp = [&] {
      hipExtLaunchKernelGGL((spmv_pipe_var_kernel<kPipeCap, 4>), dim3(gr), dim3(kBlock), 0, s, e0, e1, 0, drp, dci, dva, ms,
                            nb, 2, dx, db, (double*)nullptr, pa, dx2, dQ, dw, pb, (const uint16_t*)nullptr,
                            (const int4*)nullptr);
    };
    auto k1w = [&](int g) {
      hipExtLaunchKernelGGL((spmv_win_kernel<kPipeCap, 4>), dim3(g), dim3(kBlock), 0, s, e0, e1, 0, drp, dci, dva, dli, dch,
                            msw, nbw, 2, dx, db, pa, dx2, dQ, dw, pb);
    };
    run("K1dp slab (the solver's)", SD, k1dp);
    run("K1w slab, windows", SW, [&] { k1w(gw); });
    for (int g : {256, 768}) {
      char nm[64];
      snprintf(nm, sizeof nm, "K1w slab, windows, grid %d", g);
      run(nm, SW, [&] { k1w(g); });
    }
    std::vector<double> w1(n), w2(n), p1(16384), p2(16384);
    k1dp();
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(w1.data(), dw, 8 * n, hipMemcpyDeviceToHost));
    CK(hipMemset(dw, 0, 8 * n));
    k1w(gw);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(w2.data(), dw, 8 * n, hipMemcpyDeviceToHost));
    int64_t bad = 0;
    for (int64_t i = 0; i < n; ++i) bad += w1[i] != w2[i];
    std::vector<double> hb(n), hw(n);
    double res_ref = 0, res_w = 0;
    CK(hipMemcpy(p1.data(), pa, 8 * gw, hipMemcpyDeviceToHost));
    for (int i = 0; i < gw; ++i) res_w += p1[i];
    printf("K1w vs K1dp dual rows: %lld differ; K1w ||r||^2 partial sum %.17g\n", (long long)bad, res_w);
    (void)res_ref;
    return bad ? 1 : 0;
  }
  if (argc > 2 && std::string(argv[2]) == "slab") {
    // the solver's dual (kPipeCap table) in natural vs slab block order, resident grid vs more
    // workgroups, nontemporal matrix loads; warm (back to back: the matrix Infinity-Cache
    // resident, as in the solver) and cold
    double *dx2, *dw, *db, *pa, *pb;
    CK(hipMalloc(&dx2, 8 * pitch));
    CK(hipMalloc(&dw, 8 * pitch));
    CK(hipMalloc(&db, 8 * pitch));
    CK(hipMalloc(&pa, 8 * 16384));
    CK(hipMalloc(&pb, 8 * 16384));
    std::vector<double> h2(pitch);
    for (int64_t i = 0; i < pitch; ++i) h2[i] = i < n ? 1e-3 * ((i * 104729) % 997) - 0.4 : 0.0;
    CK(hipMemcpy(dx2, h2.data(), 8 * pitch, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, h2.data(), 8 * pitch, hipMemcpyHostToDevice));
    const double SD = 12.0 * nnz + 4.0 * (n + 1) + 32.0 * n;
    std::vector<int32_t> blk, pairs;
    blocks(n, rp.data(), kPipeCap, 256, kPipeCap, blk);
    const int nb = static_cast<int>(blk.size()) - 1;
    std::vector<int2> meta(nb + 1);
    for (int i = 0; i <= nb; ++i) meta[i] = make_int2(blk[i], rp[blk[i]]);
    int2 *mn, *ms;
    CK(hipMalloc(&mn, 8 * meta.size()));
    CK(hipMemcpy(mn, meta.data(), 8 * meta.size(), hipMemcpyHostToDevice));
    std::vector<uint8_t> lab;
    std::vector<int64_t> order;
    if (!slab_labels(n, rp.data(), ci.data(), lab) || !build_slab_order(rp.data(), lab, blk, pairs, &order)) {
      printf("no slab order\n");
      return 1;
    }
    std::vector<uint16_t> c16;
    std::vector<int32_t> bases;
    if (!build_col16(rp.data(), ci.data(), blk, c16, bases)) {
      printf("no col16 copy\n");
      return 1;
    }
    std::vector<int32_t> bslab(bases.size());
    for (size_t i = 0; i < order.size(); ++i)
      for (int q = 0; q < kCol16Bases; ++q) bslab[kCol16Bases * i + q] = bases[kCol16Bases * order[i] + q];
    uint16_t* dc16;
    int4 *dbn, *dbs;
    CK(hipMalloc(&dc16, 2 * c16.size()));
    CK(hipMemcpy(dc16, c16.data(), 2 * c16.size(), hipMemcpyHostToDevice));
    CK(hipMalloc(&dbn, 4 * bases.size()));
    CK(hipMemcpy(dbn, bases.data(), 4 * bases.size(), hipMemcpyHostToDevice));
    CK(hipMalloc(&dbs, 4 * bslab.size()));
    CK(hipMemcpy(dbs, bslab.data(), 4 * bslab.size(), hipMemcpyHostToDevice));
    CK(hipMalloc(&ms, 4 * pairs.size()));
    CK(hipMemcpy(ms, pairs.data(), 4 * pairs.size(), hipMemcpyHostToDevice));
    const int64_t big = int64_t(1) << 26;
    double* bx;
    CK(hipMalloc(&bx, 8 * big));
    CK(hipMemset(bx, 0, 8 * big));
    const int gr = resident_grid(spmv_pipe_var_kernel<kPipeCap, 4>);
    printf("blocks %d, resident grid %d (NT %d, WPE2 %d)\n", nb, gr, resident_grid(spmv_pipe_var_kernel<kPipeCap, 4, true>),
           resident_grid(spmv_pipe_var_kernel<kPipeCap, 4, false, 2>));
    auto run = [&](const char* name, auto&& launch) {
      for (int cold = 0; cold < 2; ++cold) {
        double tot = 0;
        const int reps = 30;
        for (int r = 0; r < reps + 3; ++r) {
          if (cold) hipLaunchKernelGGL(read2_kernel, dim3(4096), dim3(kBlock), 0, s, big / 2,
                                       reinterpret_cast<const double2*>(bx), pb + 8192);
          launch();
          CK(hipEventSynchronize(e1));
          float ms_;
          CK(hipEventElapsedTime(&ms_, e0, e1));
          if (r >= 3) tot += ms_;
        }
        const double us = 1e3 * tot / reps;
        printf("%s %-44s %8.2f us  %7.0f GB/s  (%.0f%% of 8 TB/s)\n", cold ? "COLD" : "WARM", name, us,
               SD / (us * 1e-6) / 1e9, 100.0 * SD / (us * 1e-6) / 8e12);
      }
    };
    char nm[128];
#define SLABRUN(LABEL, NTV, WPEV, MT, WALK, G)                                                                  \
  snprintf(nm, sizeof nm, "%s grid=%d", LABEL, G);                                                             \
  run(nm, [&] {                                                                                                \
    hipExtLaunchKernelGGL((spmv_pipe_var_kernel<kPipeCap, 4, NTV, WPEV>), dim3(G), dim3(kBlock), 0, s, e0, e1, 0, drp, \
                          dci, dva, MT, nb, WALK, dx, db, (double*)nullptr, pa, dx2, dQ, dw, pb, (const uint16_t*)nullptr, (const int4*)nullptr);             \
  })
    SLABRUN("natural", false, 1, mn, 1, gr);
    SLABRUN("slab", false, 1, ms, 2, gr);
#define FAKERUN(LABEL, FG)                                                                                      \
  snprintf(nm, sizeof nm, "%s grid=%d", LABEL, gr);                                                            \
  run(nm, [&] {                                                                                                \
    hipExtLaunchKernelGGL((spmv_pipe_var_kernel<kPipeCap, 4, false, 1, false, false, false, FG>), dim3(gr), dim3(kBlock), 0, s, \
                          e0, e1, 0, drp, dci, dva, ms, nb, 2, dx, db, (double*)nullptr, pa, dx2, dQ, dw, pb,          \
                          (const uint16_t*)nullptr, (const int4*)nullptr);                                      \
  })
    FAKERUN("slab, gathers -> coalesced rows (probe)", 1);
    FAKERUN("slab, gathers -> one address (probe)", 2);
#undef FAKERUN
    {  // interleaved (x_j, z) pairs: one 16-B gather per nonzero, rows checked bit-equal
      std::vector<double> hx(n), hp(2 * pitch, 0.0);
      CK(hipMemcpy(hx.data(), dx, 8 * n, hipMemcpyDeviceToHost));
      for (int64_t i = 0; i < n; ++i) {
        hp[2 * i] = hx[i];
        hp[2 * i + 1] = h2[i];
      }
      double* dp;
      CK(hipMalloc(&dp, 16 * pitch));
      CK(hipMemcpy(dp, hp.data(), 16 * pitch, hipMemcpyHostToDevice));
      snprintf(nm, sizeof nm, "slab, (x, z) pair gathers grid=%d", gr);
      run(nm, [&] {
        hipExtLaunchKernelGGL((spmv_pipe_var_kernel<kPipeCap, 4, false, 1, false, false, false, 3>), dim3(gr), dim3(kBlock),
                              0, s, e0, e1, 0, drp, dci, dva, ms, nb, 2, dp, db, (double*)nullptr, pa, dx2, dQ, dw, pb,
                              (const uint16_t*)nullptr, (const int4*)nullptr);
      });
      std::vector<double> w1(n), w2(n), p1(gr), p2(gr), q1(gr), q2(gr);
      hipLaunchKernelGGL((spmv_pipe_var_kernel<kPipeCap, 4>), dim3(gr), dim3(kBlock), 0, s, drp, dci, dva, ms, nb, 2, dx, db,
                         (double*)nullptr, pa, dx2, dQ, dw, pb, (const uint16_t*)nullptr, (const int4*)nullptr);
      CK(hipStreamSynchronize(s));
      CK(hipMemcpy(w1.data(), dw, 8 * n, hipMemcpyDeviceToHost));
      CK(hipMemcpy(p1.data(), pa, 8 * gr, hipMemcpyDeviceToHost));
      CK(hipMemcpy(q1.data(), pb, 8 * gr, hipMemcpyDeviceToHost));
      hipLaunchKernelGGL((spmv_pipe_var_kernel<kPipeCap, 4, false, 1, false, false, false, 3>), dim3(gr), dim3(kBlock), 0, s,
                         drp, dci, dva, ms, nb, 2, dp, db, (double*)nullptr, pa, dx2, dQ, dw, pb, (const uint16_t*)nullptr,
                         (const int4*)nullptr);
      CK(hipStreamSynchronize(s));
      CK(hipMemcpy(w2.data(), dw, 8 * n, hipMemcpyDeviceToHost));
      CK(hipMemcpy(p2.data(), pa, 8 * gr, hipMemcpyDeviceToHost));
      CK(hipMemcpy(q2.data(), pb, 8 * gr, hipMemcpyDeviceToHost));
      int64_t bad = 0;
      for (int64_t i = 0; i < n; ++i) bad += w1[i] != w2[i];
      for (int i = 0; i < gr; ++i) bad += (p1[i] != p2[i]) + (q1[i] != q2[i]);
      printf("pair gathers vs two gathers: %lld rows / partials differ\n", (long long)bad);
      CK(hipFree(dp));
    }
    for (int g : {512, 1024, 1280}) { SLABRUN("slab", false, 1, ms, 2, g); }
    SLABRUN("slab NT", true, 1, ms, 2, gr);
    SLABRUN("slab WPE2", false, 2, ms, 2, gr);
    SLABRUN("slab WPE2", false, 2, ms, 2, 1024);
#undef SLABRUN
    const int gc = resident_grid(spmv_pipe_var_kernel<kPipeCap, 4, false, 1, true>);
    printf("C16 resident grid %d\n", gc);
    const double SD16 = SD - 2.0 * nnz;
    auto run16 = [&](const char* name, const int2* mt, int walk, const int4* bb, int G) {
      for (int cold = 0; cold < 2; ++cold) {
        double tot = 0;
        const int reps = 30;
        for (int r = 0; r < reps + 3; ++r) {
          if (cold) hipLaunchKernelGGL(read2_kernel, dim3(4096), dim3(kBlock), 0, s, big / 2,
                                       reinterpret_cast<const double2*>(bx), pb + 8192);
          hipExtLaunchKernelGGL((spmv_pipe_var_kernel<kPipeCap, 4, false, 1, true>), dim3(G), dim3(kBlock), 0, s, e0, e1, 0,
                                drp, dci, dva, mt, nb, walk, dx, db, (double*)nullptr, pa, dx2, dQ, dw, pb, dc16, bb);
          CK(hipEventSynchronize(e1));
          float ms_;
          CK(hipEventElapsedTime(&ms_, e0, e1));
          if (r >= 3) tot += ms_;
        }
        const double us = 1e3 * tot / reps;
        printf("%s %-44s %8.2f us  %7.0f GB/s of 10 B/nnz  (%.0f%% of 8 TB/s)\n", cold ? "COLD" : "WARM", name, us,
               SD16 / (us * 1e-6) / 1e9, 100.0 * SD16 / (us * 1e-6) / 8e12);
      }
    };
    run16("C16 natural", mn, 1, dbn, gc);
    run16("C16 slab", ms, 2, dbs, gc);
    {  // rows bit-equal to the 32-bit columns
      std::vector<double> w1(n), w2(n);
      hipLaunchKernelGGL((spmv_pipe_var_kernel<kPipeCap, 4>), dim3(gr), dim3(kBlock), 0, s, drp, dci, dva, ms, nb, 2, dx, db,
                         (double*)nullptr, pa, dx2, dQ, dw, pb, (const uint16_t*)nullptr, (const int4*)nullptr);
      CK(hipStreamSynchronize(s));
      CK(hipMemcpy(w1.data(), dw, 8 * n, hipMemcpyDeviceToHost));
      hipLaunchKernelGGL((spmv_pipe_var_kernel<kPipeCap, 4, false, 1, true>), dim3(gc), dim3(kBlock), 0, s, drp, dci, dva, ms,
                         nb, 2, dx, db, (double*)nullptr, pa, dx2, dQ, dw, pb, dc16, dbs);
      CK(hipStreamSynchronize(s));
      CK(hipMemcpy(w2.data(), dw, 8 * n, hipMemcpyDeviceToHost));
      int64_t bad = 0;
      for (int64_t i = 0; i < n; ++i) bad += w1[i] != w2[i];
      printf("C16 vs 32-bit columns, dual rows: %lld differ\n", (long long)bad);
    }
    return 0;
  }
  if (argc > 2 && std::string(argv[2]) == "cap") {
    // K1dp / K1p block capacity: 512 / 1024 / 2048 nnz per row block (<= 256 rows), warm (back to
    // back: the matrix Infinity-Cache resident, as in the solver) and cold; rows checked bit-equal
    double *dx2, *dw, *dw2, *db, *pa, *pb;
    CK(hipMalloc(&dx2, 8 * pitch));
    CK(hipMalloc(&dw, 8 * pitch));
    CK(hipMalloc(&dw2, 8 * pitch));
    CK(hipMalloc(&db, 8 * pitch));
    CK(hipMalloc(&pa, 8 * 16384));
    CK(hipMalloc(&pb, 8 * 16384));
    std::vector<double> h2(pitch);
    for (int64_t i = 0; i < pitch; ++i) h2[i] = i < n ? 1e-3 * ((i * 104729) % 997) - 0.4 : 0.0;
    CK(hipMemcpy(dx2, h2.data(), 8 * pitch, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, h2.data(), 8 * pitch, hipMemcpyHostToDevice));
    const double SD = 12.0 * nnz + 4.0 * (n + 1) + 32.0 * n;
    auto table = [&](int cap, int& nb) {
      std::vector<int32_t> blk;
      blocks(n, rp.data(), cap, 256, cap, blk);
      nb = static_cast<int>(blk.size()) - 1;
      std::vector<int2> meta(nb + 1);
      for (int i = 0; i <= nb; ++i) meta[i] = make_int2(blk[i], rp[blk[i]]);
      int2* d;
      CK(hipMalloc(&d, 8 * meta.size()));
      CK(hipMemcpy(d, meta.data(), 8 * meta.size(), hipMemcpyHostToDevice));
      return d;
    };
    int nb5, nb1, nb2;
    int2* m5 = table(512, nb5);
    int2* m1 = table(1024, nb1);
    int2* m2 = table(2048, nb2);
    printf("blocks: cap512 %d cap1024 %d cap2048 %d\n", nb5, nb1, nb2);
    const int64_t big = int64_t(1) << 26;
    double* bx;
    CK(hipMalloc(&bx, 8 * big));
    CK(hipMemset(bx, 0, 8 * big));
    auto run = [&](const char* name, double bytes, auto&& launch) {
      for (int cold = 0; cold < 2; ++cold) {
        double tot = 0;
        const int reps = 30;
        for (int r = 0; r < reps + 3; ++r) {
          if (cold) hipLaunchKernelGGL(read2_kernel, dim3(4096), dim3(kBlock), 0, s, big / 2,
                                       reinterpret_cast<const double2*>(bx), pb + 8192);
          launch();
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          if (r >= 3) tot += ms;
        }
        const double us = 1e3 * tot / reps;
        printf("%s %-40s %8.2f us  %7.0f GB/s  (%.0f%% of 8 TB/s)\n", cold ? "COLD" : "WARM", name, us,
               bytes / (us * 1e-6) / 1e9, 100.0 * bytes / (us * 1e-6) / 8e12);
      }
    };
    char nm[128];
#define CAPRUN(CAPV, MT, NB, G)                                                                                \
  snprintf(nm, sizeof nm, "dual cap%d grid=%d", CAPV, G);                                                      \
  run(nm, SD, [&] {                                                                                            \
    hipExtLaunchKernelGGL((spmv_pipe_var_kernel<CAPV, 4, false, 1>), dim3(G), dim3(kBlock), 0, s, e0, e1, 0, drp, dci, \
                          dva, MT, NB, 1, dx, db, (double*)nullptr, pa, dx2, dQ, dw, pb, (const uint16_t*)nullptr, (const int4*)nullptr);                      \
  });                                                                                                          \
  snprintf(nm, sizeof nm, "K1 dot cap%d grid=%d", CAPV, G);                                                    \
  run(nm, S, [&] {                                                                                             \
    hipExtLaunchKernelGGL((spmv_pipe_var_kernel<CAPV, 1, false, 1>), dim3(G), dim3(kBlock), 0, s, e0, e1, 0, drp, dci, \
                          dva, MT, NB, 1, dx, dQ, dw, pa, dx, dQ, dw, pb, (const uint16_t*)nullptr, (const int4*)nullptr);                                     \
  })
    for (int g : {1280, 2048}) { CAPRUN(512, m5, nb5, g); }
    for (int g : {1024, 1280}) { CAPRUN(1024, m1, nb1, g); }
    for (int g : {512, 768, 1024, 1280}) { CAPRUN(2048, m2, nb2, g); }
#undef CAPRUN
    {  // rows bit-equal across capacities (each row sum is left to right in every table)
      hipLaunchKernelGGL((spmv_pipe_var_kernel<1024, 4, false, 1>), dim3(1280), dim3(kBlock), 0, s, drp, dci, dva, m1,
                         nb1, 1, dx, db, (double*)nullptr, pa, dx2, dQ, dw, pb, (const uint16_t*)nullptr, (const int4*)nullptr);
      hipLaunchKernelGGL((spmv_pipe_var_kernel<2048, 4, false, 1>), dim3(768), dim3(kBlock), 0, s, drp, dci, dva, m2,
                         nb2, 1, dx, db, (double*)nullptr, pa, dx2, dQ, dw2, pb, (const uint16_t*)nullptr, (const int4*)nullptr);
      CK(hipStreamSynchronize(s));
      std::vector<double> w1(n), w2(n);
      CK(hipMemcpy(w1.data(), dw, 8 * n, hipMemcpyDeviceToHost));
      CK(hipMemcpy(w2.data(), dw2, 8 * n, hipMemcpyDeviceToHost));
      int64_t bad = 0;
      for (int64_t i = 0; i < n; ++i) bad += w1[i] != w2[i];
      printf("cap2048 vs cap1024 dual rows: %lld differ\n", (long long)bad);
    }
    return 0;
  }
  if (argc > 2 && std::string(argv[2]) == "pipe") {
    // pipelined K1p / K1dp vs the current kernels: bit-identity check, then timings
    std::vector<int32_t> blk;
    blocks(n, rp.data(), kDualCap, 256, kDualCap, blk);
    const int nb = static_cast<int>(blk.size()) - 1;
    std::vector<int2> meta(nb + 1);
    for (int i = 0; i <= nb; ++i) meta[i] = make_int2(blk[i], rp[blk[i]]);
    int32_t* dblkd;
    int2* dmeta;
    CK(hipMalloc(&dblkd, 4 * blk.size()));
    CK(hipMalloc(&dmeta, 8 * meta.size()));
    CK(hipMemcpy(dblkd, blk.data(), 4 * blk.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dmeta, meta.data(), 8 * meta.size(), hipMemcpyHostToDevice));
    double *dx2, *dw, *dw2, *db, *pa, *pb, *pc, *pd;
    CK(hipMalloc(&dx2, 8 * pitch));
    CK(hipMalloc(&dw, 8 * pitch));
    CK(hipMalloc(&dw2, 8 * pitch));
    CK(hipMalloc(&db, 8 * pitch));
    for (double** p : {&pa, &pb, &pc, &pd}) CK(hipMalloc(p, 8 * 16384));
    std::vector<double> h2(pitch);
    for (int64_t i = 0; i < pitch; ++i) h2[i] = i < n ? 1e-3 * ((i * 104729) % 997) - 0.4 : 0.0;
    CK(hipMemcpy(dx2, h2.data(), 8 * pitch, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, h2.data(), 8 * pitch, hipMemcpyHostToDevice));
    CsrView A0{n, drp, dci, dva, dblkd, nb};
    CsrView AP = A0;
    AP.blk_meta = dmeta;
    const double SD = 12.0 * nnz + 4.0 * (n + 1) + 32.0 * n;
    // bit identity (walk 0 groups partials exactly as the current kernel at the same grid)
    {
      const int g = 2048;
      CK(launch_spmv_dual(A0, dx, db, pa, dx2, dw, dQ, pb, g, s));
      CK(launch_spmv_dual(AP, dx, db, pc, dx2, dw2, dQ, pd, g, s));
      CK(hipStreamSynchronize(s));
      std::vector<double> w1(n), w2(n), a(g), b2(g), c(g), d(g);
      CK(hipMemcpy(w1.data(), dw, 8 * n, hipMemcpyDeviceToHost));
      CK(hipMemcpy(w2.data(), dw2, 8 * n, hipMemcpyDeviceToHost));
      CK(hipMemcpy(a.data(), pa, 8 * g, hipMemcpyDeviceToHost));
      CK(hipMemcpy(b2.data(), pb, 8 * g, hipMemcpyDeviceToHost));
      CK(hipMemcpy(c.data(), pc, 8 * g, hipMemcpyDeviceToHost));
      CK(hipMemcpy(d.data(), pd, 8 * g, hipMemcpyDeviceToHost));
      int64_t bad = 0;
      for (int64_t i = 0; i < n; ++i) bad += w1[i] != w2[i];
      int pbad = 0;
      for (int i = 0; i < g; ++i) pbad += (a[i] != c[i]) + (b2[i] != d[i]);
      printf("pipe dual vs dual: %lld rows differ, %d partials differ\n", (long long)bad, pbad);
      CK(launch_spmv(A0, kEpiDot, dx, dw, dQ, pa, g, s));
      CK(launch_spmv(AP, kEpiDot, dx, dw2, dQ, pc, g, s));
      CK(hipStreamSynchronize(s));
      CK(hipMemcpy(w1.data(), dw, 8 * n, hipMemcpyDeviceToHost));
      CK(hipMemcpy(w2.data(), dw2, 8 * n, hipMemcpyDeviceToHost));
      CK(hipMemcpy(a.data(), pa, 8 * g, hipMemcpyDeviceToHost));
      CK(hipMemcpy(c.data(), pc, 8 * g, hipMemcpyDeviceToHost));
      bad = 0;
      for (int64_t i = 0; i < n; ++i) bad += w1[i] != w2[i];
      pbad = 0;
      for (int i = 0; i < g; ++i) pbad += a[i] != c[i];
      printf("pipe K1 dot vs K1 dot: %lld rows differ, %d partials differ\n", (long long)bad, pbad);
    }
    char nm[128];
    for (int g : {1024, 2048}) {
      snprintf(nm, sizeof nm, "dual cur grid=%d", g);
      timeit(nm, 50, SD, [&] { (void)launch_spmv_dual(A0, dx, db, pa, dx2, dw, dQ, pb, g, s); });
    }
    for (int walk : {0, 1})
      for (int g : {1024, 1280, 1536, 2048, 2560, 4096, 8192}) {
        AP.walk = walk;
        snprintf(nm, sizeof nm, "dual pipe walk=%d grid=%d", walk, g);
        timeit(nm, 50, SD, [&] { (void)launch_spmv_dual(AP, dx, db, pa, dx2, dw, dQ, pb, g, s); });
      }
    {
      AP.walk = 1;
      const int2* mt = dmeta;
#define VAR(NAME, CAPV, NTV, WPEV, G)                                                                         \
  snprintf(nm, sizeof nm, "dual pipe walk=1 %s grid=%d", NAME, G);                                            \
  timeit(nm, 50, SD, [&] {                                                                                    \
    hipLaunchKernelGGL((spmv_pipe_var_kernel<CAPV, 4, NTV, WPEV>), dim3(G), dim3(kBlock), 0, s, drp, dci, dva, mt, \
                       nb, 1, dx, db, (double*)nullptr, pa, dx2, dQ, dw, pb, (const uint16_t*)nullptr, (const int4*)nullptr);                                  \
  })
      VAR("nt", 1024, true, 1, 1280);
      for (int g : {768, 1024, 1280, 2048}) {
        snprintf(nm, sizeof nm, "dual pipe2 walk=1 grid=%d", g);
        timeit(nm, 50, SD, [&] {
          hipLaunchKernelGGL((spmv_pipe2_kernel<1024, 4>), dim3(g), dim3(kBlock), 0, s, drp, dci, dva, mt,
                             nb, 1, dx, db, (double*)nullptr, pa, dx2, dQ, dw, pb);
        });
        snprintf(nm, sizeof nm, "K1 dot pipe2 walk=1 grid=%d", g);
        timeit(nm, 50, S, [&] {
          hipLaunchKernelGGL((spmv_pipe2_kernel<1024, 1>), dim3(g), dim3(kBlock), 0, s, drp, dci, dva, mt,
                             nb, 1, dx, dQ, dw, pa, dx, dQ, dw, pb);
        });
      }
      {  // pipe2 bit identity vs pipe at the same grid / walk
        hipLaunchKernelGGL((spmv_pipe_var_kernel<1024, 4, false, 1>), dim3(1024), dim3(kBlock), 0, s, drp, dci, dva, mt,
                           nb, 1, dx, db, (double*)nullptr, pa, dx2, dQ, dw, pb, (const uint16_t*)nullptr, (const int4*)nullptr);
        hipLaunchKernelGGL((spmv_pipe2_kernel<1024, 4>), dim3(1024), dim3(kBlock), 0, s, drp, dci, dva, mt,
                           nb, 1, dx, db, (double*)nullptr, pc, dx2, dQ, dw2, pd);
        CK(hipStreamSynchronize(s));
        std::vector<double> w1(n), w2(n), a(4096), c(4096);
        CK(hipMemcpy(w1.data(), dw, 8 * n, hipMemcpyDeviceToHost));
        CK(hipMemcpy(w2.data(), dw2, 8 * n, hipMemcpyDeviceToHost));
        CK(hipMemcpy(a.data(), pa, 8 * 1024, hipMemcpyDeviceToHost));
        CK(hipMemcpy(c.data(), pc, 8 * 1024, hipMemcpyDeviceToHost));
        int64_t bad = 0;
        for (int64_t i = 0; i < n; ++i) bad += w1[i] != w2[i];
        int pbad = 0;
        for (int i = 0; i < 1024; ++i) pbad += a[i] != c[i];
        printf("pipe2 vs pipe: %lld rows differ, %d partials differ\n", (long long)bad, pbad);
      }
      {  // cold: 1 GiB of reads evict L2 and the 256 MB Infinity Cache before every launch (as the
         // MGS chain and GEMV between two dual SpMVs do in the solver); kernel time from the
         // dispatch's own events
        const int64_t big = int64_t(1) << 26;  // doubles per buffer (512 MiB)
        double *bx, *by;
        CK(hipMalloc(&bx, 8 * big));
        CK(hipMalloc(&by, 8 * big));
        CK(hipMemset(bx, 0, 8 * big));
        CK(hipMemset(by, 0, 8 * big));
        CK(hipStreamSynchronize(s));
        auto cold = [&](const char* name, double bytes, auto&& launch) {
          double tot = 0;
          const int reps = 20;
          for (int r = 0; r < reps + 2; ++r) {
            hipLaunchKernelGGL(read2_kernel, dim3(4096), dim3(kBlock), 0, s, big / 2,
                               reinterpret_cast<const double2*>(bx), pd + 8192);
            hipLaunchKernelGGL(read2_kernel, dim3(4096), dim3(kBlock), 0, s, big / 2,
                               reinterpret_cast<const double2*>(by), pd + 8192);
            launch();
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 2) tot += ms;
          }
          const double us = 1e3 * tot / reps;
          printf("COLD %-39s %8.2f us  %7.0f GB/s  (%.0f%% of 8 TB/s)\n", name, us, bytes / (us * 1e-6) / 1e9,
                 100.0 * bytes / (us * 1e-6) / 8e12);
        };
        cold("dual cur grid=2048", SD, [&] {
          hipExtLaunchKernelGGL((spmv_dual_kernel<1024, 0>), dim3(2048), dim3(kBlock), 0, s, e0, e1, 0, drp, dci, dva,
                                dblkd, nb, dx, db, pa, dx2, dw, dQ, pb);
        });
        for (int g : {1024, 1280, 2560}) {
          snprintf(nm, sizeof nm, "dual pipe walk=1 grid=%d", g);
          cold(nm, SD, [&] {
            hipExtLaunchKernelGGL((spmv_pipe_var_kernel<1024, 4, false, 1>), dim3(g), dim3(kBlock), 0, s, e0, e1, 0, drp,
                                  dci, dva, mt, nb, 1, dx, db, (double*)nullptr, pa, dx2, dQ, dw, pb, (const uint16_t*)nullptr, (const int4*)nullptr);
          });
        }
        for (int g : {768, 1024, 2048}) {
          snprintf(nm, sizeof nm, "dual pipe2 walk=1 grid=%d", g);
          cold(nm, SD, [&] {
            hipExtLaunchKernelGGL((spmv_pipe2_kernel<1024, 4>), dim3(g), dim3(kBlock), 0, s, e0, e1, 0, drp, dci, dva,
                                  mt, nb, 1, dx, db, (double*)nullptr, pa, dx2, dQ, dw, pb);
          });
          snprintf(nm, sizeof nm, "dual pipe2 walk=0 grid=%d", g);
          cold(nm, SD, [&] {
            hipExtLaunchKernelGGL((spmv_pipe2_kernel<1024, 4>), dim3(g), dim3(kBlock), 0, s, e0, e1, 0, drp, dci, dva,
                                  mt, nb, 0, dx, db, (double*)nullptr, pa, dx2, dQ, dw, pb);
          });
        }
        for (double mb : {150.0, 170.0, 186.0}) {
          const int64_t m2 = static_cast<int64_t>(mb * 1e6 / 16);
          snprintf(nm, sizeof nm, "plain read %.0f MB", mb);
          cold(nm, 16.0 * m2, [&] {
            hipExtLaunchKernelGGL(read2_kernel, dim3(2048), dim3(kBlock), 0, s, e0, e1, 0, m2,
                                  reinterpret_cast<const double2*>(bx + (big >> 1)), pd + 8192);
          });
        }
        for (int g : {1024, 1280}) {
          snprintf(nm, sizeof nm, "K1 dot pipe walk=1 grid=%d", g);
          cold(nm, S, [&] {
            hipExtLaunchKernelGGL((spmv_pipe_var_kernel<1024, 1, false, 1>), dim3(g), dim3(kBlock), 0, s, e0, e1, 0, drp,
                                  dci, dva, mt, nb, 1, dx, dQ, dw, pa, dx, dQ, dw, pb, (const uint16_t*)nullptr, (const int4*)nullptr);
          });
          snprintf(nm, sizeof nm, "K1 dot pipe2 walk=1 grid=%d", g);
          cold(nm, S, [&] {
            hipExtLaunchKernelGGL((spmv_pipe2_kernel<1024, 1>), dim3(g), dim3(kBlock), 0, s, e0, e1, 0, drp, dci, dva,
                                  mt, nb, 1, dx, dQ, dw, pa, dx, dQ, dw, pb);
          });
        }
        CK(hipFree(bx));
        CK(hipFree(by));
      }
      snprintf(nm, sizeof nm, "dual pipe walk=1 x2=x1 grid=1280");
      timeit(nm, 50, SD, [&] {
        hipLaunchKernelGGL((spmv_pipe_var_kernel<1024, 4, false, 1>), dim3(1280), dim3(kBlock), 0, s, drp, dci, dva, mt,
                           nb, 1, dx, db, (double*)nullptr, pa, dx, dQ, dw, pb, (const uint16_t*)nullptr, (const int4*)nullptr);
      });
      snprintf(nm, sizeof nm, "dual pipe walk=1 q0=b grid=1280");
      timeit(nm, 50, SD, [&] {
        hipLaunchKernelGGL((spmv_pipe_var_kernel<1024, 4, false, 1>), dim3(1280), dim3(kBlock), 0, s, drp, dci, dva, mt,
                           nb, 1, dx, db, (double*)nullptr, pa, dx2, db, dw, pb, (const uint16_t*)nullptr, (const int4*)nullptr);
      });
      snprintf(nm, sizeof nm, "single pipe walk=1 ResNorm grid=1280");
      timeit(nm, 50, S, [&] {
        hipLaunchKernelGGL((spmv_pipe_var_kernel<1024, 2, false, 1>), dim3(1280), dim3(kBlock), 0, s, drp, dci, dva, mt,
                           nb, 1, dx, db, (double*)nullptr, pa, dx, dQ, dw, pb, (const uint16_t*)nullptr, (const int4*)nullptr);
      });
      snprintf(nm, sizeof nm, "2x single pipe walk=1 (ResNorm + Dot) grid=1280");
      timeit(nm, 50, SD, [&] {
        hipLaunchKernelGGL((spmv_pipe_var_kernel<1024, 2, false, 1>), dim3(1280), dim3(kBlock), 0, s, drp, dci, dva, mt,
                           nb, 1, dx, db, (double*)nullptr, pa, dx, dQ, dw, pb, (const uint16_t*)nullptr, (const int4*)nullptr);
        hipLaunchKernelGGL((spmv_pipe_var_kernel<1024, 1, false, 1>), dim3(1280), dim3(kBlock), 0, s, drp, dci, dva, mt,
                           nb, 1, dx2, dQ, dw, pb, dx, dQ, dw, pb, (const uint16_t*)nullptr, (const int4*)nullptr);
      });
#undef VAR
    }
    AP.walk = 0;
    for (int g : {2048}) {
      snprintf(nm, sizeof nm, "K1 dot cur cap1024 grid=%d", g);
      timeit(nm, 50, S, [&] { (void)launch_spmv(A0, kEpiDot, dx, dw, dQ, pa, g, s); });
    }
    for (int walk : {0, 1})
      for (int g : {1024, 1280, 2048, 4096}) {
        AP.walk = walk;
        snprintf(nm, sizeof nm, "K1 dot pipe walk=%d grid=%d", walk, g);
        timeit(nm, 50, S, [&] { (void)launch_spmv(AP, kEpiDot, dx, dw, dQ, pa, g, s); });
      }
    return 0;
  }
  // ---- SpMV
  for (int cap : {1024, 2048}) {
    std::vector<int32_t> blk;
    blocks(n, rp.data(), cap, 256, 2048, blk);
    CK(hipMalloc(&dblk, 4 * blk.size()));
    CK(hipMemcpy(dblk, blk.data(), 4 * blk.size(), hipMemcpyHostToDevice));
    const int nb = static_cast<int>(blk.size()) - 1;
    CsrView A{n, drp, dci, dva, dblk, nb};
    char nm[128];
    for (int g : {1024, 2048, 4096, nb}) {
      const int gg = g < nb ? g : nb;
      snprintf(nm, sizeof nm, "spmv cur  items=%d grid=%d", cap, gg);
      timeit(nm, 50, S, [&] { (void)launch_spmv(A, kEpiDot, dx, dy, dQ, dpart, gg, s); });
      if (cap == 2048) {
        snprintf(nm, sizeof nm, "spmv v1<8> items=%d grid=%d", cap, gg);
        timeit(nm, 50, S, [&] {
          hipLaunchKernelGGL((spmv_v1<kEpiDot, 8>), dim3(gg), dim3(kBlock), 0, s, drp, dci, dva, dblk, nb, dx, dy, dQ, dpart);
        });
        snprintf(nm, sizeof nm, "spmv v1<8> swz1 items=%d grid=%d", cap, gg);
        timeit(nm, 50, S, [&] {
          hipLaunchKernelGGL((spmv_v1<kEpiDot, 8, 1>), dim3(gg), dim3(kBlock), 0, s, drp, dci, dva, dblk, nb, dx, dy, dQ, dpart);
        });
        snprintf(nm, sizeof nm, "spmv v1<8> swz2 items=%d grid=%d", cap, gg);
        timeit(nm, 50, S, [&] {
          hipLaunchKernelGGL((spmv_v1<kEpiDot, 8, 2>), dim3(gg), dim3(kBlock), 0, s, drp, dci, dva, dblk, nb, dx, dy, dQ, dpart);
        });
        snprintf(nm, sizeof nm, "spmv v1<8> swz1 nt items=%d grid=%d", cap, gg);
        timeit(nm, 50, S, [&] {
          hipLaunchKernelGGL((spmv_v1<kEpiDot, 8, 1, true>), dim3(gg), dim3(kBlock), 0, s, drp, dci, dva, dblk, nb, dx, dy, dQ, dpart);
        });
        snprintf(nm, sizeof nm, "spmv v1<8> nt items=%d grid=%d", cap, gg);
        timeit(nm, 50, S, [&] {
          hipLaunchKernelGGL((spmv_v1<kEpiDot, 8, 0, true>), dim3(gg), dim3(kBlock), 0, s, drp, dci, dva, dblk, nb, dx, dy, dQ, dpart);
        });
      } else {
        snprintf(nm, sizeof nm, "spmv v1<4> items=%d grid=%d", cap, gg);
        timeit(nm, 50, S, [&] {
          hipLaunchKernelGGL((spmv_v1<kEpiDot, 4>), dim3(gg), dim3(kBlock), 0, s, drp, dci, dva, dblk, nb, dx, dy, dQ, dpart);
        });
      }
    }
    CK(hipFree(dblk));
  }
  // ---- fused residual + Arnoldi SpMV vs the two single launches
  {
    double *dx2, *dw, *dpr, *dxz;
    CK(hipMalloc(&dxz, 16 * pitch));
    CK(hipMemset(dxz, 0, 16 * pitch));
    CK(hipMalloc(&dx2, 8 * pitch));
    CK(hipMalloc(&dw, 8 * pitch));
    CK(hipMalloc(&dpr, 8 * 8192));
    CK(hipMemcpy(dx2, hx.data(), 8 * pitch, hipMemcpyHostToDevice));
    const double SD = 12.0 * nnz + 4.0 * (n + 1) + 32.0 * n;
    for (int cap : {1024, 2048}) {
      std::vector<int32_t> blk;
      blocks(n, rp.data(), cap, 256, cap, blk);
      CK(hipMalloc(&dblk, 4 * blk.size()));
      CK(hipMemcpy(dblk, blk.data(), 4 * blk.size(), hipMemcpyHostToDevice));
      const int nb = static_cast<int>(blk.size()) - 1;
      CsrView A{n, drp, dci, dva, dblk, nb};
      for (int g : {1024, 2048, 4096}) {
        const int gg = g < nb ? g : nb;
        char nm[128];
        snprintf(nm, sizeof nm, "spmv res+arn (2 launches) cap=%d grid=%d", cap, gg);
        timeit(nm, 50, SD, [&] {
          (void)launch_spmv(A, kEpiResNorm, dx, nullptr, dy, dpr, gg, s);
          (void)launch_spmv(A, kEpiDot, dx2, dw, dQ, dpart, gg, s);
        });
        snprintf(nm, sizeof nm, "spmv dual interleaved cap=%d grid=%d", cap, gg);
        timeit(nm, 50, SD, [&] {
          if (cap == 1024)
            hipLaunchKernelGGL(spmv_dual_il<1024>, dim3(gg), dim3(kBlock), 0, s, drp, dci, dva, dblk, nb,
                               reinterpret_cast<const double2*>(dxz), dy, dpr, dw, dQ, dpart);
          else
            hipLaunchKernelGGL(spmv_dual_il<2048>, dim3(gg), dim3(kBlock), 0, s, drp, dci, dva, dblk, nb,
                               reinterpret_cast<const double2*>(dxz), dy, dpr, dw, dQ, dpart);
        });
        if (cap == 1024) {
          snprintf(nm, sizeof nm, "spmv dual swz1 cap=%d grid=%d", cap, gg);
          timeit(nm, 50, SD, [&] {
            hipLaunchKernelGGL((spmv_dual_kernel<1024, 1>), dim3(gg), dim3(kBlock), 0, s, drp, dci, dva, dblk, nb, dx,
                               dy, dpr, dx2, dw, dQ, dpart);
          });
          snprintf(nm, sizeof nm, "spmv dual swz2 cap=%d grid=%d", cap, gg);
          timeit(nm, 50, SD, [&] {
            hipLaunchKernelGGL((spmv_dual_kernel<1024, 2>), dim3(gg), dim3(kBlock), 0, s, drp, dci, dva, dblk, nb, dx,
                               dy, dpr, dx2, dw, dQ, dpart);
          });
        }
        snprintf(nm, sizeof nm, "spmv dual cap=%d grid=%d", cap, gg);
        timeit(nm, 50, SD, [&] {
          if (cap == 1024)
            hipLaunchKernelGGL(spmv_dual_kernel<1024>, dim3(gg), dim3(kBlock), 0, s, drp, dci, dva, dblk, nb, dx, dy,
                               dpr, dx2, dw, dQ, dpart);
          else
            hipLaunchKernelGGL(spmv_dual_kernel<2048>, dim3(gg), dim3(kBlock), 0, s, drp, dci, dva, dblk, nb, dx, dy,
                               dpr, dx2, dw, dQ, dpart);
        });
      }
      CK(hipFree(dblk));
    }
  }
  // ---- MGS chain of 30 steps (y, q_i, q_{i+1})
  const double mgsB = 32.0 * n;
  for (int g : {512, 1024, 2048}) {
    char nm[128];
    snprintf(nm, sizeof nm, "mgs cur grid=%d (per step)", g);
    timeit(nm, 1, mgsB * 30, [&] {
      for (int i = 0; i < 30; ++i)
        (void)launch_mgs_step(n, dy, dQ + i * pitch, dQ + (i + 1) * pitch, (i & 1) ? dpart2 : dpart, g,
                              (i & 1) ? dpart : dpart2, dh + i, g, s);
    });
  }
  const int64_t npair = n / 2;
  {
    const int g2 = static_cast<int>((npair + 256 * 2 - 1) / (256 * 2));
    const int g4 = static_cast<int>((npair + 256 * 4 - 1) / (256 * 4));
    const int g1 = static_cast<int>((npair + 256 - 1) / 256);
    timeit("mgs v1<1> (per step x30)", 1, mgsB * 30, [&] {
      for (int i = 0; i < 30; ++i)
        hipLaunchKernelGGL(mgs_v1<1>, dim3(g1), dim3(kBlock), 0, s, n, dy, dQ + i * pitch, dQ + (i + 1) * pitch,
                           (i & 1) ? dpart2 : dpart, 1024, (i & 1) ? dpart : dpart2, dh + i);
    });
    timeit("mgs v1<2> (per step x30)", 1, mgsB * 30, [&] {
      for (int i = 0; i < 30; ++i)
        hipLaunchKernelGGL(mgs_v1<2>, dim3(g2), dim3(kBlock), 0, s, n, dy, dQ + i * pitch, dQ + (i + 1) * pitch,
                           (i & 1) ? dpart2 : dpart, 1024, (i & 1) ? dpart : dpart2, dh + i);
    });
    timeit("mgs v1<4> (per step x30)", 1, mgsB * 30, [&] {
      for (int i = 0; i < 30; ++i)
        hipLaunchKernelGGL(mgs_v1<4>, dim3(g4), dim3(kBlock), 0, s, n, dy, dQ + i * pitch, dQ + (i + 1) * pitch,
                           (i & 1) ? dpart2 : dpart, 1024, (i & 1) ? dpart : dpart2, dh + i);
    });
  }
  // streaming copy ceiling on 2 GiB (far beyond the 256 MiB Infinity Cache), 16 B/lane
  {
    const int64_t big = int64_t(1) << 27;  // doubles per buffer (1 GiB)
    double *bx, *by;
    CK(hipMalloc(&bx, 8 * big));
    CK(hipMalloc(&by, 8 * big));
    CK(hipMemset(bx, 0, 8 * big));
    timeit("copy ceiling 1 GiB -> 1 GiB (double2)", 10, 16.0 * big, [&] {
      hipLaunchKernelGGL(copy2_kernel, dim3(4096), dim3(kBlock), 0, s, big / 2,
                         reinterpret_cast<const double2*>(bx), reinterpret_cast<double2*>(by));
    });
    timeit("read ceiling 1 GiB (double2, sum)", 10, 8.0 * big, [&] {
      hipLaunchKernelGGL(read2_kernel, dim3(4096), dim3(kBlock), 0, s, big / 2,
                         reinterpret_cast<const double2*>(bx), dpart);
    });
    CK(hipFree(bx));
    CK(hipFree(by));
  }
  printf("n=%lld nnz=%lld S=%.1f MB\n", (long long)n, (long long)nnz, S / 1e6);
  return 0;
}
