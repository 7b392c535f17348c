// hash.cpp — host-array scans of the drop-in boundary (include/spis.h): the content digest of
// cached uploads (spis_host_hash) and the all-zero test of input vectors (spis_host_nonzero).
//
// The drop-in keeps one HBM copy per SciPy matrix object (device.py): the reference's callers
// hand the same csr_matrix to solvers.cgmres on every call (e.g. lkdv/Evolve.py:41 through
// lkdv/LinearSolver.py), so re-uploading it each call would cost more than the solve.  Every call
// re-verifies the full contents against the digest taken at upload, beside the solve (device.py
// runs this on a second host thread while spis_solve runs; ctypes releases the GIL), so an
// in-place edit of any entry is caught and the solve redone on the new values.
//
// The digest: the bytes are cut into 1 MiB pieces; each piece is hashed by 4 independent 64-bit
// multiply-xor lanes, and the piece digests are folded in piece order, so the result does not
// depend on how many threads ran.  The pieces are handed out one at a time from an atomic counter
// to a persistent pool of workers (created on first use; a call that finds the pool busy — the
// verifier thread and the caller's thread hashing at once — runs on its own thread), so a scan of
// the C3 operator (~154 MB) pays no thread start-up and no core waits on a slower one's share.
// The digests and the zero scans have a pool each.
//
// The zero test (spis_host_nonzero) is numpy's truthiness of every fp64 entry (-0.0 counts as
// zero, NaN as nonzero; solvers.py drops an all-zero constraint vector, its v.Z term being 0) or
// bitwise (solvers.py passes an x0 of +0.0 entries as the shared device zero vector, no upload;
// -0.0 entries keep their sign through x_j = Z y + x0).  It stops at the first nonzero entry.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include <emmintrin.h>

#include "spis.h"

namespace {

constexpr int64_t kPiece = int64_t(1) << 20;
// the copies and zero scans of the calling thread (b, x0: one vector of a few MiB) split finer,
// so a 1.5 MiB vector still spreads over the pool (two 1 MiB pieces ran on one thread; six
// 256 KiB pieces wake six workers, where 64 KiB ones woke all sixteen for no gain)
#ifndef SPIS_FINE_SHIFT
#define SPIS_FINE_SHIFT 18  // 256 KiB (tools/r06_hostcopy.sh: 2^16, 2^18, 2^20 A/B on the box)
#endif
constexpr int64_t kFine = int64_t(1) << SPIS_FINE_SHIFT;

inline uint64_t mix(uint64_t h) {  // murmur3's finaliser
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ull;
  h ^= h >> 33;
  return h;
}

uint64_t piece_digest(const unsigned char* p, int64_t n, uint64_t index) {
  uint64_t a0 = 0x9E3779B97F4A7C15ull ^ index, a1 = 0xC2B2AE3D27D4EB4Full, a2 = 0x165667B19E3779F9ull,
           a3 = 0x27D4EB2F165667C5ull;
  auto round = [&](const uint64_t* w) {
    a0 = (a0 ^ w[0]) * 0xff51afd7ed558ccdull;
    a1 = (a1 ^ w[1]) * 0xc4ceb9fe1a85ec53ull;
    a2 = (a2 ^ w[2]) * 0xff51afd7ed558ccdull;
    a3 = (a3 ^ w[3]) * 0xc4ceb9fe1a85ec53ull;
    a0 ^= a0 >> 29;
    a1 ^= a1 >> 29;
    a2 ^= a2 >> 29;
    a3 ^= a3 >> 29;
  };
  int64_t i = 0;
  uint64_t w[4];
  for (; i + 32 <= n; i += 32) {
    std::memcpy(w, p + i, 32);
    round(w);
  }
  if (i < n) {  // the last < 32 bytes, zero-padded, through the same lanes: every byte keeps its
                // position (a tail folded by shifts alone let bytes 8 apart commute)
    std::memset(w, 0, sizeof w);
    std::memcpy(w, p + i, static_cast<size_t>(n - i));
    round(w);
  }
  return mix(mix(a0) ^ mix(a1 + 1) ^ mix(a2 + 2) ^ mix(a3 + 3) ^ mix(static_cast<uint64_t>(n)));
}

// any entry of p[0 .. n) nonzero: in numpy's sense (bits << 1) != 0 (the sign bit alone is
// -0.0), or bitwise (any bit set: -0.0 counts)
bool piece_nonzero(const uint64_t* p, int64_t n, bool bitwise) {
  uint64_t acc = 0;
  int64_t i = 0;
  for (; i + 8 <= n; i += 8)
    acc |= p[i] | p[i + 1] | p[i + 2] | p[i + 3] | p[i + 4] | p[i + 5] | p[i + 6] | p[i + 7];
  for (; i < n; ++i) acc |= p[i];
  return (bitwise ? acc : acc << 1) != 0;  // (a | b) << 1 == (a << 1) | (b << 1): sign bits dropped
}

// Persistent workers running one job at a time: job(piece) for piece = 0 .. n_pieces - 1, each
// piece claimed from an atomic counter by whichever thread (the caller included) is free.
class Pool {
 public:
  // one pool per kind of caller (0: the digests, run on the verifier thread; 1: the zero scans of
  // the calling thread), so a scan never finds the pool held by a digest of a cached operator and
  // runs alone, nor a digest by a scan
  static Pool& get(int which) {
    static Pool* p[2] = {new Pool(), new Pool()};  // never destroyed: workers may outlive static destructors
    return *p[which & 1];
  }

  // false when another caller holds the pool (the caller then runs the job alone)
  bool run(int threads, int64_t n_pieces, const std::function<void(int64_t)>& job) {
    std::unique_lock<std::mutex> busy(run_mu_, std::try_to_lock);
    if (!busy.owns_lock()) return false;
    const int helpers = std::max(0, std::min<int>(threads, kMaxThreads) - 1);
    if (!ensure(helpers)) return false;
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &job;
      n_ = n_pieces;
      next_.store(0);
      active_ = helpers;
      want_ = helpers;
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return active_ == 0; });
    job_ = nullptr;
    return true;
  }

 private:
  static constexpr int kMaxThreads = 32;

  bool ensure(int helpers) {
    try {
      while (static_cast<int>(workers_.size()) < helpers) {
        const int id = static_cast<int>(workers_.size());
        workers_.emplace_back([this, id] { loop(id); });
        workers_.back().detach();
      }
    } catch (...) {
      return static_cast<int>(workers_.size()) >= helpers;
    }
    return true;
  }

  void work() {
    for (int64_t k = next_.fetch_add(1); k < n_; k = next_.fetch_add(1)) (*job_)(k);
  }

  void loop(int id) {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (id >= want_) continue;  // not needed for this job
      }
      work();
      std::lock_guard<std::mutex> lk(mu_);
      if (--active_ == 0) done_cv_.notify_all();
    }
  }

  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::thread> workers_;
  const std::function<void(int64_t)>* job_ = nullptr;
  int64_t n_ = 0;
  std::atomic<int64_t> next_{0};
  int active_ = 0, want_ = 0;
  uint64_t gen_ = 0;
};

// dst <- src with streaming (non-temporal) 16-byte stores where both are 16-byte aligned: the
// staging buffer is read next by the DMA engine, not by this CPU, so its lines are written without
// being read first (16 B moved per byte copied instead of 24); sfence before the piece counts as
// done, since streaming stores are not ordered by the pool's mutex hand-off
void copy_stream(unsigned char* d, const unsigned char* s, int64_t n) {
  int64_t i = 0;
  if (((reinterpret_cast<uintptr_t>(d) | reinterpret_cast<uintptr_t>(s)) & 15) == 0) {
    for (; i + 64 <= n; i += 64) {
      const __m128i a = _mm_load_si128(reinterpret_cast<const __m128i*>(s + i));
      const __m128i b = _mm_load_si128(reinterpret_cast<const __m128i*>(s + i + 16));
      const __m128i c = _mm_load_si128(reinterpret_cast<const __m128i*>(s + i + 32));
      const __m128i e = _mm_load_si128(reinterpret_cast<const __m128i*>(s + i + 48));
      _mm_stream_si128(reinterpret_cast<__m128i*>(d + i), a);
      _mm_stream_si128(reinterpret_cast<__m128i*>(d + i + 16), b);
      _mm_stream_si128(reinterpret_cast<__m128i*>(d + i + 32), c);
      _mm_stream_si128(reinterpret_cast<__m128i*>(d + i + 48), e);
    }
    _mm_sfence();
  }
  if (i < n) std::memcpy(d + i, s + i, static_cast<size_t>(n - i));
}

void for_pieces(int pool, int threads, int64_t n_pieces, const std::function<void(int64_t)>& job) {
  if (threads > 1 && n_pieces >= 4 && Pool::get(pool).run(threads, n_pieces, job)) return;
  for (int64_t k = 0; k < n_pieces; ++k) job(k);
}

}  // namespace

extern "C" int spis_host_hash(const void* data, int64_t bytes, int32_t threads, uint64_t* out) {
  if (!out || bytes < 0 || (bytes > 0 && !data)) return SPIS_ERR_ARG;
  const unsigned char* p = static_cast<const unsigned char*>(data);
  const int64_t np = (bytes + kPiece - 1) / kPiece;
  try {
    std::vector<uint64_t> d(static_cast<size_t>(std::max<int64_t>(np, 1)), 0);
    for_pieces(0, threads, np, [&](int64_t k) {
      const int64_t o = k * kPiece;
      d[k] = piece_digest(p + o, std::min(kPiece, bytes - o), static_cast<uint64_t>(k));
    });
    uint64_t h = mix(static_cast<uint64_t>(bytes) ^ 0x5350495348415348ull);
    for (int64_t k = 0; k < np; ++k) h = mix(h ^ d[k]) + 0x9E3779B97F4A7C15ull;
    *out = h;
  } catch (...) {
    return SPIS_ERR_STATE;
  }
  return SPIS_OK;
}

extern "C" int spis_host_copy(void* dst, const void* src, int64_t bytes, int32_t threads) {
  if (bytes < 0 || (bytes > 0 && (!dst || !src))) return SPIS_ERR_ARG;
  unsigned char* d = static_cast<unsigned char*>(dst);
  const unsigned char* s = static_cast<const unsigned char*>(src);
  const int64_t np = (bytes + kFine - 1) / kFine;
  try {
    // the scan pool (1): the caller's thread is the one that runs the zero scans, one at a time
    for_pieces(1, threads, np, [&](int64_t k) {
      const int64_t o = k * kFine;
      copy_stream(d + o, s + o, std::min(kFine, bytes - o));
    });
  } catch (...) {
    return SPIS_ERR_STATE;
  }
  return SPIS_OK;
}

extern "C" int spis_host_nonzero(const double* data, int64_t count, int32_t bitwise, int32_t threads,
                                 int32_t* any_out) {
  if (!any_out || count < 0 || (count > 0 && !data)) return SPIS_ERR_ARG;
  const uint64_t* w = reinterpret_cast<const uint64_t*>(data);
  constexpr int64_t kHead = 4096;  // most nonzero vectors show it in the first entries
  if (piece_nonzero(w, std::min(count, kHead), bitwise != 0)) {
    *any_out = 1;
    return SPIS_OK;
  }
  if (count <= kHead) {
    *any_out = 0;
    return SPIS_OK;
  }
  constexpr int64_t kEl = kFine / 8;
  const int64_t rest = count - kHead, np = (rest + kEl - 1) / kEl;
  std::atomic<int> found{0};
  try {
    for_pieces(1, threads, np, [&](int64_t k) {
      if (found.load(std::memory_order_relaxed)) return;
      const int64_t o = kHead + k * kEl;
      if (piece_nonzero(w + o, std::min(kEl, count - o), bitwise != 0)) found.store(1, std::memory_order_relaxed);
    });
  } catch (...) {
    return SPIS_ERR_STATE;
  }
  *any_out = found.load();
  return SPIS_OK;
}

// The host least squares (lsq.cpp) is built for x86-64-v3 (Makefile LSQFLAGS: AVX2, FMA); this
// translation unit is not, so the loader (_lib.py) can ask before the first KKT solve would
// fault on an older host CPU with an illegal instruction.
extern "C" int spis_host_isa_ok(void) {
  __builtin_cpu_init();
  return (__builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma") && __builtin_cpu_supports("bmi2")) ? 1 : 0;
}
