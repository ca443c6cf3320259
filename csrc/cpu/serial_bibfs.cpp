// Serial bidirectional BFS (C1 capability) + BFS oracle + path validator.
#include <algorithm>
#include <chrono>
#include <string>

#include "bibfs/cpu_engine.hpp"

namespace bibfs {

SerialBiBfs::SerialBiBfs(const Csr& g) : g_(g) {
  for (int s = 0; s < 2; ++s) {
    vis_[s].assign(g.n, 0);
    parent_[s].assign(g.n, kNoVertex);
    queue_[s].reserve(1024);
  }
}

namespace {
uint64_t frontier_edges(const Csr& g, const std::vector<vid_t>& q, size_t b, size_t e) {
  uint64_t s = 0;
  for (size_t i = b; i < e; ++i) s += g.degree(q[i]);
  return s;
}
}  // namespace

SearchResult SerialBiBfs::search(vid_t src, vid_t dst, const SearchOptions& opt) {
  const auto t0 = std::chrono::steady_clock::now();
  BIBFS_REQUIRE(src < g_.n && dst < g_.n, "src/dst out of range");
  SearchResult r;
  if (src == dst) {  // reference v1 prints 2 here; the distance is 0
    r.found = true;
    r.hops = 0;
    r.meet = src;
    r.path = {src};
    r.stats.visited = 1;
    r.total_ms = r.search_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return r;
  }
  const vid_t root[2] = {src, dst};
  size_t fb[2], fe[2];
  int depth[2] = {0, 0};
  for (int s = 0; s < 2; ++s) {
    queue_[s].clear();
    queue_[s].push_back(root[s]);
    vis_[s][root[s]] = 1;
    parent_[s][root[s]] = kNoVertex;
    fb[s] = 0;
    fe[s] = 1;
  }
  vid_t meet = kNoVertex;
  int meet_side = 0;
  int turn = 0;
  while (meet == kNoVertex && fb[0] < fe[0] && fb[1] < fe[1]) {
    int s;
    switch (opt.side) {
      case SidePolicy::kSmallerFrontier: s = (fe[0] - fb[0] <= fe[1] - fb[1]) ? 0 : 1; break;
      case SidePolicy::kAlternate: s = turn; turn ^= 1; break;
      default:
        s = frontier_edges(g_, queue_[0], fb[0], fe[0]) <= frontier_edges(g_, queue_[1], fb[1], fe[1]) ? 0 : 1;
    }
    const int o = s ^ 1;
    auto& q = queue_[s];
    auto& vis = vis_[s];
    auto& par = parent_[s];
    const auto& ovis = vis_[o];
    LevelTrace lt;
    lt.side = s;
    lt.depth = depth[s];
    lt.frontier = fe[s] - fb[s];
    lt.mode = 0;
    const size_t e = fe[s];
    for (size_t i = fb[s]; i < e && meet == kNoVertex; ++i) {
      const vid_t u = q[i];
      const uint64_t rb = g_.row_off[u], re = g_.row_off[u + 1];
      lt.edges += re - rb;
      for (uint64_t k = rb; k < re; ++k) {
        const vid_t v = g_.col[k];
        if (vis[v]) continue;
        vis[v] = 1;
        par[v] = u;
        q.push_back(v);
        if (ovis[v]) {
          meet = v;
          meet_side = s;
          break;
        }
      }
    }
    lt.discovered = q.size() - e;
    fb[s] = e;
    fe[s] = q.size();
    ++depth[s];
    r.stats.levels++;
    r.stats.edges_inspected += lt.edges;
    if (opt.trace) r.stats.trace.push_back(lt);
  }
  (void)meet_side;
  if (meet != kNoVertex) {
    r.found = true;
    r.meet = meet;
    std::vector<vid_t> a, b;
    for (vid_t c = meet; c != kNoVertex; c = parent_[0][c]) a.push_back(c);
    for (vid_t c = meet; c != kNoVertex; c = parent_[1][c]) b.push_back(c);
    r.hops = (int64_t)a.size() - 1 + (int64_t)b.size() - 1;
    if (opt.want_path) {
      r.path.assign(a.rbegin(), a.rend());
      r.path.insert(r.path.end(), b.begin() + 1, b.end());
    }
  }
  r.stats.visited = queue_[0].size() + queue_[1].size();
  // reset only what this query touched
  for (int s = 0; s < 2; ++s)
    for (vid_t v : queue_[s]) vis_[s][v] = 0;
  r.total_ms = r.search_ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return r;
}

SearchResult bfs_oracle(const Csr& g, vid_t src, vid_t dst) {
  BIBFS_REQUIRE(src < g.n && dst < g.n, "src/dst out of range");
  SearchResult r;
  std::vector<vid_t> parent(g.n, kNoVertex);
  std::vector<uint8_t> seen(g.n, 0);
  std::vector<vid_t> q;
  q.reserve(1024);
  q.push_back(src);
  seen[src] = 1;
  for (size_t i = 0; i < q.size(); ++i) {
    vid_t u = q[i];
    if (u == dst) break;
    for (uint64_t k = g.row_off[u]; k < g.row_off[u + 1]; ++k) {
      vid_t v = g.col[k];
      if (!seen[v]) {
        seen[v] = 1;
        parent[v] = u;
        q.push_back(v);
      }
    }
  }
  if (!seen[dst]) return r;
  r.found = true;
  for (vid_t c = dst; c != kNoVertex; c = parent[c]) r.path.push_back(c);
  std::reverse(r.path.begin(), r.path.end());
  r.hops = (int64_t)r.path.size() - 1;
  r.meet = dst;
  return r;
}

std::vector<int64_t> bfs_distances(const Csr& g, vid_t src) {
  std::vector<int64_t> d(g.n, -1);
  std::vector<vid_t> q;
  q.push_back(src);
  d[src] = 0;
  for (size_t i = 0; i < q.size(); ++i) {
    vid_t u = q[i];
    for (uint64_t k = g.row_off[u]; k < g.row_off[u + 1]; ++k) {
      vid_t v = g.col[k];
      if (d[v] < 0) {
        d[v] = d[u] + 1;
        q.push_back(v);
      }
    }
  }
  return d;
}

bool validate_path(const Csr& g, vid_t src, vid_t dst, int64_t hops, const std::vector<vid_t>& path,
                   std::string* why) {
  auto fail = [&](const std::string& m) {
    if (why) *why = m;
    return false;
  };
  if ((int64_t)path.size() != hops + 1) return fail("path length != hops + 1");
  if (path.front() != src || path.back() != dst) return fail("path endpoints differ from src/dst");
  for (size_t i = 0; i + 1 < path.size(); ++i) {
    vid_t u = path[i], v = path[i + 1];
    if (u >= g.n || v >= g.n) return fail("vertex out of range");
    bool ok = false;
    for (uint64_t k = g.row_off[u]; k < g.row_off[u + 1] && !ok; ++k) ok = (g.col[k] == v);
    if (!ok) return fail("non-adjacent consecutive vertices " + std::to_string(u) + " " + std::to_string(v));
  }
  return true;
}

}  // namespace bibfs
