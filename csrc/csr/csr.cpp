// Host CSR construction (counting sort: degree histogram -> exclusive scan ->
// scatter), multi-threaded.  Single shared implementation of what the
// reference re-implements inline four times (v1/main-v1.cpp:35-40,
// v2/second_try.cpp:45-50, v3/bibfs_cuda_only.cu:89-99, v4/mpi_bas.cpp:45-57).
// The GPU path builds the same structure on device (csrc/hip/csr_device.hip).
#include <algorithm>
#include <atomic>
#include <thread>

#include "bibfs/graph.hpp"

namespace bibfs {

namespace {

int pick_threads(int t, uint64_t work) {
  if (t <= 0) t = (int)std::max(1u, std::thread::hardware_concurrency());
  if (work < (1u << 16)) t = 1;  // small inputs: sequential => deterministic order
  return std::min(t, 64);
}

template <typename F>
void parallel_for(int threads, uint64_t n, F&& f) {
  if (threads <= 1 || n < 2) {
    f(0, (uint64_t)0, n);
    return;
  }
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t) {
    uint64_t b = n * t / threads, e = n * (t + 1) / threads;
    pool.emplace_back([&, t, b, e] { f(t, b, e); });
  }
  for (auto& th : pool) th.join();
}

void finish_rows(Csr& g, const CsrOptions& opt, int threads) {
  if (!opt.dedup && !opt.sort_rows) return;
  parallel_for(threads, g.n, [&](int, uint64_t b, uint64_t e) {
    for (uint64_t v = b; v < e; ++v)
      std::sort(g.col.begin() + (ptrdiff_t)g.row_off[v], g.col.begin() + (ptrdiff_t)g.row_off[v + 1]);
  });
  if (!opt.dedup) return;
  // compact unique entries (sequential pass over sorted rows)
  uint64_t w = 0;
  uint64_t prev_end = 0;
  for (uint32_t v = 0; v < g.n; ++v) {
    uint64_t b = prev_end, e = g.row_off[v + 1];
    prev_end = e;
    g.row_off[v] = w;
    for (uint64_t i = b; i < e; ++i)
      if (i == b || g.col[i] != g.col[i - 1]) g.col[w++] = g.col[i];
  }
  g.row_off[g.n] = w;
  g.col.resize(w);
  g.col.shrink_to_fit();
}

// Generic builder over an edge predicate: keep(u) says whether row u is stored
// and row(u) maps it to a local row index.
template <typename Keep, typename Row>
Csr build_impl(const EdgeList& el, uint32_t nrows, const CsrOptions& opt, Keep keep, Row row) {
  Csr g;
  g.n = nrows;
  g.m_input = el.m();
  const uint64_t m = el.m();
  const uint32_t* uv = el.uv.data();
  const int threads = pick_threads(opt.threads, m);
  std::vector<std::atomic<uint64_t>> deg(nrows + 1ULL);
  for (auto& d : deg) d.store(0, std::memory_order_relaxed);
  parallel_for(threads, m, [&](int, uint64_t b, uint64_t e) {
    for (uint64_t i = b; i < e; ++i) {
      uint32_t u = uv[2 * i], v = uv[2 * i + 1];
      if (opt.drop_self_loops && u == v) continue;
      if (keep(u)) deg[row(u)].fetch_add(1, std::memory_order_relaxed);
      if (keep(v)) deg[row(v)].fetch_add(1, std::memory_order_relaxed);
    }
  });
  g.row_off.resize(nrows + 1ULL);
  uint64_t acc = 0;
  for (uint32_t r = 0; r < nrows; ++r) {
    g.row_off[r] = acc;
    acc += deg[r].load(std::memory_order_relaxed);
  }
  g.row_off[nrows] = acc;
  g.col.resize(acc);
  // cursors reuse the degree array
  for (uint32_t r = 0; r < nrows; ++r) deg[r].store(g.row_off[r], std::memory_order_relaxed);
  uint32_t* col = g.col.data();
  parallel_for(threads, m, [&](int, uint64_t b, uint64_t e) {
    for (uint64_t i = b; i < e; ++i) {
      uint32_t u = uv[2 * i], v = uv[2 * i + 1];
      if (opt.drop_self_loops && u == v) continue;
      if (keep(u)) col[deg[row(u)].fetch_add(1, std::memory_order_relaxed)] = v;
      if (keep(v)) col[deg[row(v)].fetch_add(1, std::memory_order_relaxed)] = u;
    }
  });
  finish_rows(g, opt, threads);
  return g;
}

}  // namespace

Csr build_csr(const EdgeList& el, const CsrOptions& opt) {
  return build_impl(
      el, el.n, opt, [](uint32_t) { return true; }, [](uint32_t u) { return u; });
}

Csr build_csr_rows(const EdgeList& el, const Partition& part, const CsrOptions& opt) {
  const uint32_t lo = part.lo, hi = part.hi;
  return build_impl(
      el, hi - lo, opt, [lo, hi](uint32_t u) { return u >= lo && u < hi; },
      [lo](uint32_t u) { return u - lo; });
}

EdgeList csr_to_edges(const Csr& g) {
  EdgeList el;
  el.n = g.n;
  for (uint32_t u = 0; u < g.n; ++u)
    for (uint64_t i = g.row_off[u]; i < g.row_off[u + 1]; ++i)
      if (u < g.col[i]) {
        el.uv.push_back(u);
        el.uv.push_back(g.col[i]);
      }
  return el;
}

}  // namespace bibfs
