// chainbench.hip — MGS chain variants at solver size, timed with HIP events (tuning tool, not
// part of libspis): K2p (dedicated gatherer), K2q (pipelined), K2q + fused update GEMV, and the
// standalone GEMV, for Arnoldi steps j in {1, 5, 15, 29}.  Build: make tools/chainbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#define SPIS_CHAIN_TRACE 1
#include "../structurepreservingiterativesolvers_amd/csrc/kernels.hip"

using namespace spis;

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 1002252;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const int kmax = 31;
  const int64_t pitch = (n + 63) / 64 * 64;
  std::vector<double> h(static_cast<size_t>(pitch) * (kmax + 1));
  std::mt19937_64 rng(1);
  std::normal_distribution<double> nd;
  for (auto& v : h) v = nd(rng) * 1e-3;
  double *Q, *w, *x0, *xo, *part, *gsub;
  CK(hipMalloc(&Q, sizeof(double) * pitch * (kmax + 1)));
  CK(hipMalloc(&w, sizeof(double) * pitch));
  CK(hipMalloc(&x0, sizeof(double) * pitch));
  CK(hipMalloc(&xo, sizeof(double) * pitch));
  CK(hipMalloc(&part, sizeof(double) * 4096));
  CK(hipMalloc(&gsub, sizeof(double) * kChainGsub));
  CK(hipMemcpy(Q, h.data(), sizeof(double) * pitch * (kmax + 1), hipMemcpyHostToDevice));
  CK(hipMemcpy(w, h.data(), sizeof(double) * pitch, hipMemcpyHostToDevice));
  CK(hipMemcpy(x0, h.data() + pitch, sizeof(double) * pitch, hipMemcpyHostToDevice));
  CK(hipMemset(part, 0, sizeof(double) * 4096));
  CK(hipMemset(gsub, 0, sizeof(double) * kChainGsub));
  unsigned long long* gran;
  unsigned *ep, *err;
  CK(hipMalloc(&gran, sizeof(unsigned long long) * kChainGranLag));
  CK(hipMemset(gran, 0, sizeof(unsigned long long) * kChainGranLag));
  CK(hipMalloc(&ep, 16));
  CK(hipMemset(ep, 0, 16));
  {  // tag base 1 (as libspis): K2q's E_0 tag must never be the slots' initial 0
    const unsigned one = 1;
    CK(hipMemcpy(ep, &one, sizeof one, hipMemcpyHostToDevice));
  }
  CK(hipMalloc(&err, 16));
  CK(hipMemset(err, 0, 16));
  double* hcol;
  CK(hipHostMalloc(&hcol, sizeof(double) * 64, hipHostMallocMapped | hipHostMallocCoherent));
  double* hcol_dev;
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hcol_dev), hcol, 0));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<double> y(64, 0.01);
  // the chain reads w and never writes it: repeated launches see the same inputs
  if (argc > 3 && std::string(argv[3]) == "trace") {  // phase timestamps of K2q + FX (the solver's chain)
    set_chain_lag(2);
    for (int j : {1, 2, 5, 15, 29}) {
      auto run = [&]() {
        CK(launch_mgs_chain(n, w, Q, pitch, j, part, 1024, hcol_dev, gran, ep, err, s, nullptr, nullptr, 0, nullptr,
                            nullptr, nullptr, true, 1, gsub, y.data(), j, x0, xo));
      };
      for (int r = 0; r < 3; ++r) run();
      CK(hipStreamSynchronize(s));
      for (int rep = 0; rep < 3; ++rep) {
        unsigned long long tr[3][48] = {};
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_chain_trace), tr, sizeof(tr)));
        CK(hipEventRecord(e0, s));
        run();
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipMemcpyFromSymbol(tr, HIP_SYMBOL(g_chain_trace), sizeof(tr)));
        unsigned long long t0 = ~0ull;
        for (int r = 0; r < 3; ++r)
          if (tr[r][0] && tr[r][0] < t0) t0 = tr[r][0];
        printf("j=%2d event %.1f us\n", j, 1e3 * ms);
        const char* rn[3] = {"wg0", "wgL", "gat"};
        for (int r = 0; r < 3; ++r) {
          printf("  %s start %.2f loaded %.2f |", rn[r], 0.01 * (tr[r][0] - t0), 0.01 * (tr[r][1] - t0));
          for (int m = 1; m <= j + 1; ++m) printf(" %.2f", tr[r][2 + m] ? 0.01 * (tr[r][2 + m] - t0) : -1.0);
          if (r < 2) printf(" | stored %.2f", 0.01 * (tr[r][40] - t0));
          printf("\n");
        }
      }
    }
    return 0;
  }
  if (argc > 3 && std::string(argv[3]) == "ring") {  // K2q + FX at other (data waves, pairs, ring) shapes
    const int64_t npr = (n + 1) >> 1;
    YArg ya;
    for (int i = 0; i < kYArg; ++i) ya.v[i] = 0.01;
    auto shape = [&](const char* name, auto kern, int DW, int PER) {
      const int64_t span = int64_t(DW) * 64 * PER;
      const int GD = static_cast<int>((npr + span - 1) / span);
      if (GD > kChainMaxWG - 1) {
        printf("%s: %d workgroups, too many\n", name, GD);
        return;
      }
      for (int j : {5, 15, 29}) {
        auto run = [&]() {
          hipLaunchKernelGGL(kern, dim3(GD + 1), dim3(DW * 64 + 64), 0, s, n, w, Q, pitch, j, part, 1024, hcol_dev, gran,
                             ep, err, (const double*)nullptr, 0, (double*)nullptr, (unsigned long long*)nullptr,
                             (const unsigned long long*)nullptr, gsub, ya, j, x0, xo, 0, 1);
        };
        for (int r = 0; r < 3; ++r) run();
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        for (int r = 0; r < reps; ++r) run();
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        unsigned he = 0;
        CK(hipMemcpy(&he, err, 4, hipMemcpyDeviceToHost));
        printf("%-28s GD %3d j=%2d %7.1f us%s\n", name, GD, j, 1e3 * ms / reps, he ? "  CHAIN ERROR" : "");
        if (he) return;
      }
    };
    shape("DW8 PER4 NS5 (default)", mgs_chain_lag_kernel<8, 4, 5, 2, true, true>, 8, 4);
    shape("DW7 PER5 NS5", mgs_chain_lag_kernel<7, 5, 5, 2, true, true>, 7, 5);
    shape("DW7 PER5 NS6", mgs_chain_lag_kernel<7, 5, 6, 2, true, true>, 7, 5);
    shape("DW6 PER6 NS6", mgs_chain_lag_kernel<6, 6, 6, 2, true, true>, 6, 6);
    return 0;
  }
  const char* names[] = {"K2p agg", "K2q", "K2q+gemv", "gemv"};
  for (int lag = 1; lag <= 2; ++lag)
  for (int nt = 0; nt < 2; ++nt)
    for (int j : {1, 2, 5, 15, 29}) {
      set_chain_lag(lag);
      printf("n=%lld lag=%d nt=%d j=%2d:", static_cast<long long>(n), lag, nt, j);
      for (int v = 0; v < 4; ++v) {
        auto run = [&]() {
          if (v == 0)
            CK(launch_mgs_chain(n, w, Q, pitch, j, part, 1024, hcol_dev, gran, ep, err, s, nullptr, nullptr, 0,
                                nullptr, nullptr, nullptr, true, nt));
          else if (v == 1)
            CK(launch_mgs_chain(n, w, Q, pitch, j, part, 1024, hcol_dev, gran, ep, err, s, nullptr, nullptr, 0,
                                nullptr, nullptr, nullptr, true, nt, gsub));
          else if (v == 2)
            CK(launch_mgs_chain(n, w, Q, pitch, j, part, 1024, hcol_dev, gran, ep, err, s, nullptr, nullptr, 0,
                                nullptr, nullptr, nullptr, true, nt, gsub, y.data(), j, x0, xo));
          else
            CK(launch_gemv(n, j, Q, pitch, y.data(), true, x0, xo, s));
        };
        run();
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        for (int r = 0; r < reps; ++r) run();
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("  %s %7.1f us", names[v], 1e3 * ms / reps);
      }
      unsigned he = 0;
      CK(hipMemcpy(&he, err, 4, hipMemcpyDeviceToHost));
      printf("%s\n", he ? "  CHAIN ERROR" : "");
      if (he) return 1;
    }
  return 0;
}
