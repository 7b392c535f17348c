// hash.cpp — content digest of host arrays (spis_host_hash, include/spis.h).
//
// The drop-in keeps one HBM copy per SciPy matrix object (device.py): the reference's callers
// hand the same csr_matrix to solvers.cgmres on every call (e.g. lkdv/Evolve.py:41 through
// lkdv/LinearSolver.py), so re-uploading it each call would cost more than the solve.  Every call
// re-verifies the full contents against the digest taken at upload, beside the solve (device.py
// runs this on a second host thread while spis_solve runs; ctypes releases the GIL), so an
// in-place edit of any entry is caught and the solve redone on the new values.
//
// The digest: the bytes are cut into 1 MiB pieces; each piece is hashed by 4 independent 64-bit
// multiply-xor lanes (memory-bound: ~6 GB/s per thread), and the piece digests are folded in piece
// order, so the result does not depend on how many threads ran.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "spis.h"

namespace {

constexpr int64_t kPiece = int64_t(1) << 20;

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

}  // namespace

extern "C" int spis_host_hash(const void* data, int64_t bytes, int32_t threads, uint64_t* out) {
  if (!out || bytes < 0 || (bytes > 0 && !data)) return SPIS_ERR_ARG;
  const unsigned char* p = static_cast<const unsigned char*>(data);
  const int64_t np = (bytes + kPiece - 1) / kPiece;
  std::vector<uint64_t> d(static_cast<size_t>(std::max<int64_t>(np, 1)), 0);
  auto run = [&](int64_t k0, int64_t k1) {
    for (int64_t k = k0; k < k1; ++k) {
      const int64_t o = k * kPiece;
      d[k] = piece_digest(p + o, std::min(kPiece, bytes - o), static_cast<uint64_t>(k));
    }
  };
  int nt = std::max(1, std::min<int>(threads, static_cast<int>(np / 4)));  // >= 4 MiB per thread
  try {
    if (nt <= 1) {
      run(0, np);
    } else {
      std::vector<std::thread> th;
      const int64_t per = (np + nt - 1) / nt;
      for (int t = 1; t < nt; ++t)
        th.emplace_back(run, std::min(np, t * per), std::min(np, (t + 1) * per));
      run(0, std::min(np, per));
      for (auto& x : th) x.join();
    }
  } catch (...) {
    return SPIS_ERR_STATE;
  }
  uint64_t h = mix(static_cast<uint64_t>(bytes) ^ 0x5350495348415348ull);
  for (int64_t k = 0; k < np; ++k) h = mix(h ^ d[k]) + 0x9E3779B97F4A7C15ull;
  *out = h;
  return SPIS_OK;
}
