// Host graph generators: chunked G(n,p) geometric skipping and counter-based
// R-MAT.  Parallel over fixed chunks, so the output does not depend on the
// thread count.
#include "bibfs/gen.hpp"

#include <algorithm>
#include <thread>
#include <vector>

namespace bibfs {

namespace {
int nthreads(int t) {
  if (t <= 0) t = (int)std::max(1u, std::thread::hardware_concurrency());
  return std::min(t, 64);
}
template <typename F>
void run_threads(int t, F&& f) {
  if (t <= 1) {
    f(0, 1);
    return;
  }
  std::vector<std::thread> pool;
  for (int i = 0; i < t; ++i) pool.emplace_back([&, i] { f(i, t); });
  for (auto& th : pool) th.join();
}
}  // namespace

EdgeList gen_gnp(uint32_t n, double p, uint64_t seed, int threads) {
  EdgeList el;
  el.n = n;
  const uint64_t K = gnp_num_chunks(n, p);
  const int t = (K < 64) ? 1 : nthreads(threads);
  // pass 1: count per chunk
  std::vector<uint64_t> cnt(K + 1, 0);
  run_threads(t, [&](int i, int T) {
    for (uint64_t c = i; c < K; c += (uint64_t)T)
      cnt[c] = gnp_walk_chunk(n, p, seed, K, c, [](uint32_t, uint32_t) {});
  });
  uint64_t total = 0;
  for (uint64_t c = 0; c < K; ++c) {
    uint64_t x = cnt[c];
    cnt[c] = total;
    total += x;
  }
  cnt[K] = total;
  BIBFS_REQUIRE(total <= 0xFFFFFFFFULL, "G(n,p): more than 2^32-1 edges does not fit a .bin");
  el.uv.resize(2 * total);
  uint32_t* out = el.uv.data();
  run_threads(t, [&](int i, int T) {
    for (uint64_t c = i; c < K; c += (uint64_t)T) {
      uint64_t pos = cnt[c];
      gnp_walk_chunk(n, p, seed, K, c, [&](uint32_t v, uint32_t w) {
        out[2 * pos] = w;  // (u < v) like networkx's edge tuples
        out[2 * pos + 1] = v;
        ++pos;
      });
    }
  });
  return el;
}

EdgeList gen_rmat(uint32_t n, uint64_t m, uint64_t seed, double a, double b, double c,
                  int threads) {
  BIBFS_REQUIRE(n >= 2, "R-MAT needs n >= 2");
  RmatParams P;
  P.n = n;
  P.scale = ceil_log2_u64(n);
  P.a = a;
  P.b = b;
  P.c = c;
  P.seed = seed;
  EdgeList el;
  el.n = n;
  el.uv.resize(2 * m);
  uint32_t* out = el.uv.data();
  const int t = (m < 4096) ? 1 : nthreads(threads);
  run_threads(t, [&](int i, int T) {
    uint64_t b0 = m * i / T, e0 = m * (i + 1) / T;
    for (uint64_t e = b0; e < e0; ++e) rmat_edge(P, e, &out[2 * e], &out[2 * e + 1]);
  });
  return el;
}

EdgeList gen_kronecker(int scale, int edgefactor, uint64_t seed, int threads) {
  BIBFS_REQUIRE(scale >= 1 && scale <= 31, "kronecker scale must be in [1, 31]");
  const uint32_t n = 1u << scale;
  return gen_rmat(n, (uint64_t)edgefactor * n, seed, 0.57, 0.19, 0.19, threads);
}

}  // namespace bibfs
