// C ABI wrapper around bibfs::HipBiBfs (include/bibfs/bibfs_hip.h).
#include <cstring>
#include <string>

#include "bibfs/bibfs_hip.h"
#include "bibfs/hip_engine.hpp"
#include "bibfs/io.hpp"

struct bibfs_ctx {
  bibfs::HipBiBfs eng;
  explicit bibfs_ctx(int d) : eng(d) {}
};

namespace {
thread_local std::string g_err;

template <typename F>
int guarded(F&& f) {
  try {
    f();
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

void fill(const bibfs::SearchResult& r, bibfs_result* out, uint32_t* path, size_t cap) {
  if (!out) return;
  out->found = r.found ? 1 : 0;
  out->hops = r.hops;
  out->meet = r.meet;
  out->levels = r.stats.levels;
  out->edges_inspected = r.stats.edges_inspected;
  out->search_ms = r.search_ms;
  out->total_ms = r.total_ms;
  out->path_len = 0;
  if (path && r.found) {
    out->path_len = std::min(cap, r.path.size());
    std::memcpy(path, r.path.data(), out->path_len * sizeof(uint32_t));
  }
}
}  // namespace

extern "C" {

bibfs_ctx* bibfs_create(int device) {
  bibfs_ctx* c = nullptr;
  guarded([&] { c = new bibfs_ctx(device); });
  return c;
}

void bibfs_destroy(bibfs_ctx* ctx) { delete ctx; }

const char* bibfs_last_error(void) { return g_err.c_str(); }

int bibfs_init_graph(bibfs_ctx* ctx, uint32_t n, uint64_t nnz, const uint64_t* row_off, const uint32_t* col) {
  return guarded([&] {
    bibfs::Csr g;
    g.n = n;
    g.m_input = nnz / 2;
    g.row_off.assign(row_off, row_off + n + 1);
    g.col.assign(col, col + nnz);
    ctx->eng.load_csr(g);
  });
}

int bibfs_init_graph_edges(bibfs_ctx* ctx, uint32_t n, uint64_t m, const uint32_t* uv) {
  return guarded([&] {
    bibfs::EdgeList el;
    el.n = n;
    el.uv.assign(uv, uv + 2 * m);
    ctx->eng.load_edges(el);
  });
}

int bibfs_load_bin(bibfs_ctx* ctx, const char* path) {
  return guarded([&] { ctx->eng.load_edges(bibfs::read_bin(path)); });
}

int bibfs_search(bibfs_ctx* ctx, uint32_t src, uint32_t dst, bibfs_result* out, uint32_t* path, size_t cap) {
  return guarded([&] { fill(ctx->eng.search(src, dst), out, path, cap); });
}

int bibfs_init_frontiers(bibfs_ctx* ctx, uint32_t src, uint32_t dst) {
  return guarded([&] { ctx->eng.begin(src, dst); });
}

int bibfs_expand_frontier(bibfs_ctx* ctx, int side, uint64_t* claimed, int* met) {
  return guarded([&] {
    bool m = false;
    uint64_t c = ctx->eng.expand(side, &m);
    if (claimed) *claimed = c;
    if (met) *met = m ? 1 : 0;
  });
}

int bibfs_check_intersect(bibfs_ctx* ctx, int* found) {
  return guarded([&] {
    bool f = ctx->eng.check_meet();
    if (found) *found = f ? 1 : 0;
  });
}

int bibfs_finish(bibfs_ctx* ctx, bibfs_result* out, uint32_t* path, size_t cap) {
  return guarded([&] { fill(ctx->eng.finish(), out, path, cap); });
}

int bibfs_free_graph(bibfs_ctx* ctx) {
  return guarded([&] { ctx->eng.release(); });  // v4/comp.cu:121-133 cudaFreeGraph
}

}  // extern "C"
