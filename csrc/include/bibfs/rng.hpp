// Counter-based random numbers shared by host and device generators.
//
// The reference generator (graphs/generate_graph.py:31) calls networkx
// fast_gnp_random_graph unseeded, so its graphs are unreproducible.  Every
// generator here is a pure function of (seed, stream, counter): the host
// implementation (csrc/gen/gen.cpp) and the device implementation
// (csrc/hip/gen_device.hip) produce bit-identical edge lists, which the tests
// check.  splitmix64 finalisers are cheap on both a CPU core and a CDNA4 lane
// (only 64-bit multiplies and shifts).
#pragma once

#include <cmath>
#include <cstdint>

#include "bibfs/common.hpp"

namespace bibfs {

BIBFS_HD inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

// One 64-bit draw for (seed, stream, counter).
BIBFS_HD inline uint64_t rng64(uint64_t seed, uint64_t stream, uint64_t counter) {
  uint64_t s = mix64(seed + 0x9e3779b97f4a7c15ULL);
  uint64_t t = mix64(s ^ (stream * 0xd1b54a32d192ed03ULL));
  return mix64(t + counter * 0x9e3779b97f4a7c15ULL);
}

// Uniform double in (0, 1].
BIBFS_HD inline double rng_unit(uint64_t x) {
  return (double)((x >> 11) + 1) * (1.0 / 9007199254740992.0);
}

// ---------------------------------------------------------------------------
// G(n, p) by geometric skipping over the strictly-lower-triangular pair space
// (same model as networkx fast_gnp_random_graph, Batagelj & Brandes 2005).
// Pair index i enumerates (v, w), 0 <= w < v < n, as i = v(v-1)/2 + w.  The
// index space is cut into a fixed number of chunks (a function of n and p
// only, never of the thread count) so that every chunk is an independent RNG
// stream: host and device produce the same edges in the same order.
// ---------------------------------------------------------------------------
BIBFS_HD inline uint64_t gnp_total_pairs(uint64_t n) { return n < 2 ? 0 : n * (n - 1) / 2; }

BIBFS_HD inline uint64_t gnp_num_chunks(uint64_t n, double p) {
  const uint64_t T = gnp_total_pairs(n);
  if (T == 0 || p <= 0.0) return 1;
  double expect = (double)T * (p < 1.0 ? p : 1.0);
  uint64_t k = (uint64_t)(expect / 256.0);  // ~256 edges per chunk
  if (k < 1) k = 1;
  if (k > (1ULL << 22)) k = 1ULL << 22;
  if (k > T) k = T;
  return k;
}

BIBFS_HD inline void gnp_chunk_range(uint64_t n, uint64_t nchunks, uint64_t c, uint64_t* lo,
                                     uint64_t* hi) {
  const uint64_t T = gnp_total_pairs(n);
  // 128-bit free split: (T / k) * c + min(c, T % k)
  const uint64_t q = T / nchunks, r = T % nchunks;
  *lo = q * c + (c < r ? c : r);
  *hi = *lo + q + (c < r ? 1 : 0);
}

// Decode pair index -> (v, w), w < v.
BIBFS_HD inline void gnp_decode(uint64_t idx, uint32_t* v, uint32_t* w) {
  double d = std::sqrt(8.0 * (double)idx + 1.0);
  uint64_t vv = (uint64_t)((1.0 + d) * 0.5);
  // fix rounding: need vv(vv-1)/2 <= idx < vv(vv+1)/2
  while (vv * (vv - 1) / 2 > idx) --vv;
  while ((vv + 1) * vv / 2 <= idx) ++vv;
  *v = (uint32_t)vv;
  *w = (uint32_t)(idx - vv * (vv - 1) / 2);
}

// Walk one chunk; calls emit(v, w) for every edge.  Returns the edge count.
template <typename Emit>
BIBFS_HD inline uint64_t gnp_walk_chunk(uint64_t n, double p, uint64_t seed, uint64_t nchunks,
                                        uint64_t c, Emit&& emit) {
  uint64_t lo, hi;
  gnp_chunk_range(n, nchunks, c, &lo, &hi);
  if (lo >= hi || p <= 0.0) return 0;
  uint64_t cnt = 0;
  if (p >= 1.0) {
    for (uint64_t i = lo; i < hi; ++i) {
      uint32_t v, w;
      gnp_decode(i, &v, &w);
      emit(v, w);
      ++cnt;
    }
    return cnt;
  }
  const double lp = std::log1p(-p);
  uint64_t draw = 0;
  uint64_t i = lo;
  bool first = true;
  for (;;) {
    double r = rng_unit(rng64(seed, c, draw++));
    double skip = std::floor(std::log(r) / lp);  // >= 0
    if (skip > (double)(hi - lo)) break;
    i = first ? lo + (uint64_t)skip : i + 1 + (uint64_t)skip;
    first = false;
    if (i >= hi) break;
    uint32_t v, w;
    gnp_decode(i, &v, &w);
    emit(v, w);
    ++cnt;
  }
  return cnt;
}

// ---------------------------------------------------------------------------
// R-MAT / Kronecker (Graph500 initiator a=.57 b=.19 c=.19 d=.05 by default).
// Edge e is a pure function of (seed, e): `scale` quadrant choices from
// counter-based draws, then a bijective scramble of [0, 2^scale) so that hub
// ids are spread over the id space (as the Graph500 generator does).  For a
// vertex count n that is not a power of two the edge is re-drawn (attempt
// counter) until both endpoints are < n; self loops are re-drawn as well, so
// the edge count is exact.
// ---------------------------------------------------------------------------
struct RmatParams {
  uint32_t n = 0;
  int scale = 0;  // ceil(log2 n)
  double a = 0.57, b = 0.19, c = 0.19;
  uint64_t seed = 1;
  bool scramble = true;
};

BIBFS_HD inline uint64_t rmat_scramble(uint64_t x, int scale, uint64_t seed) {
  const uint64_t mask = (scale >= 64) ? ~0ULL : ((1ULL << scale) - 1);
  uint64_t k1 = (mix64(seed ^ 0x1234567ULL) | 1ULL);
  uint64_t k2 = (mix64(seed ^ 0x89abcdefULL) | 1ULL);
  uint64_t add = mix64(seed ^ 0x55aa55aaULL);
  const int sh = scale / 2 > 0 ? scale / 2 : 1;
  x = (x * k1 + add) & mask;
  x ^= x >> sh;
  x = (x * k2) & mask;
  x ^= x >> sh;
  x = (x * k1 + (add >> 7)) & mask;
  return x;
}

BIBFS_HD inline void rmat_edge(const RmatParams& P, uint64_t e, uint32_t* uo, uint32_t* vo) {
  for (uint64_t attempt = 0;; ++attempt) {
    uint64_t u = 0, v = 0;
    const uint64_t stream = e * 64 + (attempt & 63) + ((attempt >> 6) << 40);
    for (int l = 0; l < P.scale; l += 2) {
      uint64_t x = rng64(P.seed, stream, (uint64_t)l);
      // two quadrant draws per 64-bit word (32 bits each)
      for (int h = 0; h < 2 && l + h < P.scale; ++h) {
        double r = ((double)((x >> (32 * h)) & 0xffffffffULL) + 0.5) * (1.0 / 4294967296.0);
        int q = r < P.a ? 0 : (r < P.a + P.b ? 1 : (r < P.a + P.b + P.c ? 2 : 3));
        u = (u << 1) | (uint64_t)(q >> 1);
        v = (v << 1) | (uint64_t)(q & 1);
      }
    }
    if (P.scramble) {
      u = rmat_scramble(u, P.scale, P.seed);
      v = rmat_scramble(v, P.scale, P.seed);
    }
    if (u < P.n && v < P.n && u != v) {
      *uo = (uint32_t)u;
      *vo = (uint32_t)v;
      return;
    }
  }
}

BIBFS_HD inline int ceil_log2_u64(uint64_t x) {
  int s = 0;
  while ((1ULL << s) < x) ++s;
  return s;
}

}  // namespace bibfs
